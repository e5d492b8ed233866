// 256 x 256 bf16 GEMM with a 4-phase-per-K-tile LDS-DMA pipeline: the hot path's large products
// (frozen-ViT projections, fusion-adapter linears, decoder 1x1 convolutions at batch 32):
//   C[z] = epi(alpha A[z] B[z] + beta C[z]).
//
// fp32 operands arrive as bf16 PIECES along K (vfm_split_f32 below: [hi | mid | lo] for the
// fp32-equivalent f32x6 products, [hi | lo] for the opt-in f32x3 ones), and the kernel walks
// T x K/64 "virtual" K-tiles: term t multiplies piece Terms<NP>::a(t) of A by piece
// Terms<NP>::b(t) of B (vfm_common.h), so the 6 (or 3) bf16 products accumulate in the same fp32
// registers as one GEMM of depth T*K, without duplicated operand copies in HBM.
//
// Schedule (cdna_hip_programming.md §5 "The 256² 8-phase template", T2-T5; written from its rules):
//   * 8 waves as 2 (M) x 4 (N), wave tile 128 x 64 = 8 x 4 blocks of v_mfma_f32_16x16x32_bf16;
//     each K-tile (64) is computed in 4 phases, one C-quadrant (64 x 32, 16 MFMAs) each, in the
//     order (Alo,Blo) (Alo,Bhi) (Ahi,Bhi) (Ahi,Blo): every fragment is read from LDS once per
//     K-tile (A_lo p0, B_lo p0, B_hi p1, A_hi p2; 24 ds_read_b128 per wave) and kept in VGPRs;
//   * each operand tile is staged as two half-tiles: A_lo = the first 64 rows of both wave-rows'
//     128-row bands, A_hi the second 64; B_lo / B_hi the first / second 32 columns of each
//     wave-column's 64. A half-tile is 16 KB = 2 LDS-DMA (global_load_lds_dwordx4) per thread;
//   * phase p of K-tile t issues ONE half-tile of K-tile t+1 into the other LDS buffer (order
//     A_lo, B_lo, B_hi, A_hi), reads its own fragments (made visible by the previous phase's
//     counted wait + barrier), waits with a COUNTED s_waitcnt vmcnt for the next phase's
//     half-tile only (4 DMA stay in flight across every barrier), raw s_barrier, lgkmcnt(0),
//     then its 16 MFMAs under s_setprio(1);
//   * two barriers per phase (after the reads, after the MFMAs) and the wm = 1 wave-row one
//     barrier behind the wm = 0 row (one extra barrier before / after the loop): each row's MFMAs
//     run while the other row issues its DMA and fragment reads (ping-pong);
//   * RAW: the half-tile read in phase p is waited for (counted vmcnt, every wave) before the
//     first barrier of phase p-1, which both rows pass before their phase-p reads;
//   * WAR: with the rows one barrier apart, a half-tile is restaged >= 2 phases after its last
//     read (A_lo: read p0, restaged next tile p0 = 4 phases; B_lo: p0 -> p1 = 5; B_hi: p1 -> p2 = 5;
//     A_hi: p2 -> p3 = 5);
//   * LDS images XOR-swizzled on the DMA source address (destination lane-linear): K-contiguous
//     half-tiles [128 rows][64 k] (128-B rows, chunk ^= (row>>1)&7, ds_read_b128 fragments),
//     MN-contiguous ones [64 k][128] (256-B rows, gemm.hip's 4x4 chunk swizzle, ds_read_b64_tr_b16);
//   * XCD-aware bijective block -> tile remap, grouped tile order; bf16 and fp32 epilogues staged
//     through LDS with 16-B row stores when the tile is full.
#include "vfm_common.h"

namespace {

using namespace vfm;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BM = 256, BN = 256, BK = 64, THREADS = 512;
constexpr int HALF = 128 * 64 * 2;        // bytes of one half-tile image (16 KB)
constexpr int BUF = 4 * HALF;             // A_lo, A_hi, B_lo, B_hi of one K-tile (64 KB)

struct G8Args {
    const __hip_bfloat16* A;
    const __hip_bfloat16* B;
    void* C;
    const float* bias;
    long long lda, ldb, ldc, sA, sB, sC;
    int M, N, K;
    float alpha, beta;
    int bias_mode, act;
    // split-K over "virtual" K-tiles: per output batch (reduce = 0) or over the concatenation of
    // every batch's K (reduce = 1: C = sum_z A[z] B[z]); S = ceil(V / kchunk) splits write fp32
    // partials to ws, gemm8_reduce applies the epilogue. ws == null: direct epilogue.
    float* ws;
    int kchunk, S, reduce, Z;
    // fp32 emulation: T product terms over pieces of Kp columns (rows) each; term t reads piece
    // (pa >> 2t) & 3 of A and (pb >> 2t) & 3 of B (T = 1, pa = pb = 0 for bf16 operands)
    int T, Kp, pa, pb;
};

__device__ __forceinline__ int kc_off(int row, int ch) { return row * 128 + 16 * (ch ^ ((row >> 1) & 7)); }
__device__ __forceinline__ int mc_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int mc_off(int row, int ch) { return row * 256 + 16 * (ch ^ mc_swz(row)); }

__device__ __forceinline__ float gelu_tanh(float x) {
    const float u = 0.7978845608028654f * fmaf(0.044715f * x, x * x, x);
    const float e = __builtin_amdgcn_exp2f(2.8853900817779268f * u);
    return 0.5f * x * (2.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f));
}

// half-tile row / column r (0..127) -> tile row / column, q = lo (0) / hi (1) half
__device__ __forceinline__ int a_outer(int r, int q) { return 128 * (r >> 6) + 64 * q + (r & 63); }
__device__ __forceinline__ int b_outer(int r, int q) { return 64 * (r >> 5) + 32 * q + (r & 31); }

// LDS offsets of the half-tiles inside one buffer
constexpr int OFF_ALO = 0, OFF_AHI = HALF, OFF_BLO = 2 * HALF, OFF_BHI = 3 * HALF;

// One LDS-DMA instruction (global_load_lds_dwordx4: lane l's 16 B land at lds_dst + 16 l). Issued
// from inline asm so that hipcc's waitcnt pass does not see an LDS write in flight and drain it
// with vmcnt(0) before every ds_read (which serialised the pipeline of the builtin form: see
// gemm_fast.hip); the counted waits below are the only ones. m0 is set in the same statement.
__device__ __forceinline__ void glds16(const void* g, const unsigned char* lds_dst) {
    const unsigned la = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_void*)lds_dst);
    asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(la) : "memory", "m0");
}

// Issue the DMA of one half-tile (2 x 16 B per thread).
template <bool KCONT, bool ISA>
__device__ __forceinline__ void dma_half(unsigned char* img, const __hip_bfloat16* base, long long ld, int outer0,
                                         int outer_n, int k0, int q, int tid) {
    const int wave = tid >> 6, lane = tid & 63;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int cbase = wave * 64 + 512 * u;
        const int ci = cbase + lane;
        const __hip_bfloat16* src;
        if (KCONT) {
            const int row = ci >> 3, chs = (ci & 7) ^ ((row >> 1) & 7);
            const int o = min(outer0 + (ISA ? a_outer(row, q) : b_outer(row, q)), outer_n - 1);
            src = base + (long long)o * ld + k0 + 8 * chs;
        } else {
            const int row = ci >> 4, chs = (ci & 15) ^ mc_swz(row);
            int o = outer0 + (ISA ? a_outer(8 * chs, q) : b_outer(8 * chs, q));
            if (o >= outer_n) o = 0;                       // (outer_n % 8 == 0): a valid chunk, result unused
            src = base + (long long)(k0 + row) * ld + o;
        }
        glds16(src, img + cbase * 16);
    }
}

// 16x16x32 fragment of 16-row block `blk` of a half-tile image (blk 0..7), k32 step t
template <bool KCONT>
__device__ __forceinline__ bf16x8 frag16(const unsigned char* img, int blk, int t, int lane) {
    if (KCONT) {
        return *reinterpret_cast<const bf16x8*>(img + kc_off(16 * blk + (lane & 15), 4 * t + (lane >> 4)));
    } else {
        const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
        const int ch = 2 * blk + (p >> 1);
        const int row = 32 * t + 8 * g + q;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + mc_off(row, ch) + 8 * (p & 1)));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(img + mc_off(row + 4, ch) + 8 * (p & 1)));
        return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
}

#define VMCNT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

// wait until at most n half-tiles (2 DMA each) of this wave are in flight (n wave-uniform)
__device__ __forceinline__ void vm_halves(int n) {
    switch (n) {
    case 4: VMCNT(8); break;
    case 3: VMCNT(6); break;
    case 2: VMCNT(4); break;
    case 1: VMCNT(2); break;
    default: VMCNT(0); break;
    }
}

template <bool AK, bool BKC, bool OUTF32, bool DEEP>
__global__ __launch_bounds__(THREADS, 1) void gemm8_kernel(G8Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 2, wn = wave & 3;
    const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.N + BN - 1) / BN;
    const int nwg = tiles_m * tiles_n;
    const int bid = blockIdx.x, xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    // grouped order: consecutive tiles (the ~32 an XCD runs at once) cover GROUP tile-rows x 32/GROUP
    // tile-columns, so the XCD's L2 holds GROUP A panels + 32/GROUP B panels instead of 1 + 32
    constexpr int GROUP = 4;
    const int gsz = GROUP * tiles_n, grp = tile / gsz, rem = tile - grp * gsz;
    const int rows_g = min(GROUP, tiles_m - grp * GROUP);
    const int tm = grp * GROUP + rem % rows_g, tn = rem / rows_g;
    const int m0 = tm * BM, n0 = tn * BN;
    const int KTz = a.Kp / BK;                         // K-tiles per batch and piece
    const int zo = a.reduce ? 0 : (int)blockIdx.y / a.S, sp = (int)blockIdx.y - zo * a.S;
    const int VT = a.reduce ? a.Z * KTz : KTz;         // virtual K-tiles of one product term
    const int V = a.T * VT;                            // virtual K-tiles of this output
    const int v0 = sp * a.kchunk;
    const int KT = min(V, v0 + a.kchunk) - v0;         // >= 1 by construction of S on the host
    const int z = zo;                                  // output batch

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};

    // source of local K-tile t: batch, term -> pieces, k offsets inside each operand (wave-uniform)
    struct Src {
        const __hip_bfloat16* Ab;
        const __hip_bfloat16* Bb;
        int ka, kb;
    };
    auto src_of = [&](int t) {
        const int v = v0 + t;
        const int term = v / VT, rest = v - term * VT;
        const int zt = a.reduce ? rest / KTz : zo, k0 = (a.reduce ? rest - zt * KTz : rest) * BK;
        Src r;
        r.Ab = a.A + (long long)zt * a.sA;
        r.Bb = a.B + (long long)zt * a.sB;
        r.ka = k0 + ((a.pa >> (2 * term)) & 3) * a.Kp;
        r.kb = k0 + ((a.pb >> (2 * term)) & 3) * a.Kp;
        return r;
    };
    // half-tile h of local K-tile t into its buffer: h = 0 A_lo, 1 B_lo, 2 B_hi, 3 A_hi (issue order)
    auto issue = [&](const Src& sr, int t, int h) {
        unsigned char* buf = lds + (t & 1) * BUF;
        if (h == 0) dma_half<AK, true>(buf + OFF_ALO, sr.Ab, a.lda, m0, a.M, sr.ka, 0, tid);
        else if (h == 1) dma_half<BKC, false>(buf + OFF_BLO, sr.Bb, a.ldb, n0, a.N, sr.kb, 0, tid);
        else if (h == 2) dma_half<BKC, false>(buf + OFF_BHI, sr.Bb, a.ldb, n0, a.N, sr.kb, 1, tid);
        else dma_half<AK, true>(buf + OFF_AHI, sr.Ab, a.lda, m0, a.M, sr.ka, 1, tid);
    };
    bf16x8 af[4][2], bl[2][2], bh[2][2];        // A quadrant rows; B_lo / B_hi columns (both kept)
    // half-tile h, phase p: which fragments phase p reads (A_lo + B_lo at p0, B_hi at p1, A_hi at p2;
    // A every second phase) and multiplies (quadrant (qm, qn))
    auto phase_math = [&](const unsigned char* buf, int p) {
        const int qm = p >> 1;                          // 0 0 1 1
        const int qn = (p == 1 || p == 2) ? 1 : 0;      // 0 1 1 0
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int s = 0; s < 2; ++s)
                    acc[4 * qm + i][2 * qn + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        af[i][s], qn ? bh[j][s] : bl[j][s], acc[4 * qm + i][2 * qn + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_s_barrier();
        (void)buf;
    };
    auto phase_reads = [&](const unsigned char* buf, int p) {
        if (p == 0 || p == 2) {
            const unsigned char* ai = buf + (p ? OFF_AHI : OFF_ALO);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int s = 0; s < 2; ++s) af[i][s] = frag16<AK>(ai, 4 * wm + i, s, lane);
        }
        if (p == 0 || p == 1) {                         // B_lo read once (p0, reused p3), B_hi once (p1, reused p2)
            const unsigned char* bi = buf + (p ? OFF_BHI : OFF_BLO);
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    if (p == 0) bl[j][s] = frag16<BKC>(bi, 2 * wn + j, s, lane);
                    else bh[j][s] = frag16<BKC>(bi, 2 * wn + j, s, lane);
                }
        }
    };
    if (DEEP) {
        // Two K-tiles ahead: the fragments of a half-tile live in VGPRs after their phase, so its LDS
        // slot is restaged for K-tile t+2 two phases later (WAR >= 2 phases with the rows one barrier
        // apart). Phase p of tile t issues p0: B_hi(t+1), p1: A_hi(t+1) (buffer (t+1)&1), p2:
        // A_lo(t+2), p3: B_lo(t+2) (buffer t&1); the counted waits leave 4 half-tiles (8 DMA) in
        // flight: each half-tile is issued 5-6 phases before its read instead of 2-4.
        {
            const Src s0 = src_of(0);
            issue(s0, 0, 0);
            issue(s0, 0, 1);
            issue(s0, 0, 2);
            issue(s0, 0, 3);
        }
        Src s1 = src_of(KT > 1 ? 1 : 0);
        if (KT > 1) {
            issue(s1, 1, 0);
            issue(s1, 1, 1);
        }
        vm_halves(2 + (KT > 1 ? 2 : 0));            // A_lo(0), B_lo(0)
        __builtin_amdgcn_s_barrier();
        if (wm == 1) __builtin_amdgcn_s_barrier();
        for (int t = 0; t < KT; ++t) {
            const unsigned char* buf = lds + (t & 1) * BUF;
            const bool n1 = t + 1 < KT, n2 = t + 2 < KT;
            const Src s2 = src_of(n2 ? t + 2 : t);
            // p0: issue B_hi(t+1); read A_lo(t), B_lo(t); wait for B_hi(t)
            if (n1) issue(s1, t + 1, 2);
            phase_reads(buf, 0);
            vm_halves(1 + (n1 ? 3 : 0));
            phase_math(buf, 0);
            // p1: issue A_hi(t+1); read B_hi(t); wait for A_hi(t)
            if (n1) issue(s1, t + 1, 3);
            phase_reads(buf, 1);
            vm_halves(n1 ? 4 : 0);
            phase_math(buf, 1);
            // p2: issue A_lo(t+2); read A_hi(t)
            if (n2) issue(s2, t + 2, 0);
            phase_reads(buf, 2);
            phase_math(buf, 2);
            // p3: issue B_lo(t+2); wait for A_lo(t+1), B_lo(t+1)
            if (n2) issue(s2, t + 2, 1);
            if (n1) vm_halves(2 + (n2 ? 2 : 0));
            phase_math(buf, 3);
            s1 = s2;
        }
    } else {
    {
        const Src s0 = src_of(0);
        issue(s0, 0, 0);
        issue(s0, 0, 1);
        issue(s0, 0, 2);
        issue(s0, 0, 3);
    }
    VMCNT(4);                                   // A_lo, B_lo of tile 0
    __builtin_amdgcn_s_barrier();
    // ping-pong: the wm = 1 wave-row runs one barrier behind (2 barriers per phase), so one
    // wave-row's 16 MFMAs overlap the other's DMA issue + fragment reads (see the header)
    if (wm == 1) __builtin_amdgcn_s_barrier();

    for (int t = 0; t < KT; ++t) {
        const unsigned char* buf = lds + (t & 1) * BUF;
        const bool nxt = t + 1 < KT;
        const Src sn = src_of(nxt ? t + 1 : t);
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            if (nxt) issue(sn, t + 1, p);
            phase_reads(buf, p);
            // wait for the NEXT phase's half-tile (see the header), then the phase barrier
            if (nxt) {
                if (p == 0 || p == 1 || p == 3) VMCNT(4);
            } else {
                if (p == 0) VMCNT(2);
                else if (p == 1) VMCNT(0);
            }
            phase_math(buf, p);
        }
    }
    }
    if (wm == 0) __builtin_amdgcn_s_barrier();
    VMCNT(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    // epilogue: acc[i][j][r] = C[m0 + 128wm + 16i + 4(l>>4) + r][n0 + 64wn + 16j + (l&15)]
    const int cl = lane & 15, rq = 4 * (lane >> 4);
    if (a.ws) {                                        // split-K partial, raw fp32
        float* w = a.ws + (long long)blockIdx.y * a.M * a.N;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + 64 * wn + 16 * j + cl;
            if (n >= a.N) continue;
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int m = m0 + 128 * wm + 16 * i + rq + r;
                    if (m < a.M) w[(long long)m * a.N + n] = acc[i][j][r];
                }
        }
        return;
    }
    typedef typename std::conditional<OUTF32, float, __hip_bfloat16>::type TC;
    TC* Cb = reinterpret_cast<TC*>(a.C) + (long long)z * a.sC;
    if (!OUTF32 && a.beta == 0.f && m0 + BM <= a.M && n0 + BN <= a.N && (a.ldc % 8) == 0 &&
        (reinterpret_cast<uintptr_t>(a.C) % 16) == 0 && (a.sC % 8) == 0) {
        unsigned short* wl = reinterpret_cast<unsigned short*>(lds + wave * 128 * 128);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int nl = 16 * j + cl;
            const int n = n0 + 64 * wn + nl;
            const float bcol = (a.bias_mode == 1) ? a.bias[n] : 0.f;
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int ml = 16 * i + rq + r;
                    float v = a.alpha * acc[i][j][r];
                    v += (a.bias_mode == 2) ? a.bias[m0 + 128 * wm + ml] : bcol;
                    if (a.act == 1) v = gelu_tanh(v);
                    else if (a.act == 2) v = v * gelu_parts(v).cdf;
                    const int ch = (nl >> 3) ^ (ml & 7);
                    wl[ml * 64 + ch * 8 + (nl & 7)] = __builtin_bit_cast(unsigned short, __float2bfloat16(v));
                }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        __hip_bfloat16* crow = reinterpret_cast<__hip_bfloat16*>(a.C) + (long long)z * a.sC +
                               (long long)(m0 + 128 * wm) * a.ldc + n0 + 64 * wn;
#pragma unroll 4
        for (int c = lane; c < 128 * 8; c += 64) {
            const int ml = c >> 3, chl = c & 7;
            const uint4 v = *reinterpret_cast<const uint4*>(wl + ml * 64 + 8 * (chl ^ (ml & 7)));
            *reinterpret_cast<uint4*>(crow + (long long)ml * a.ldc + 8 * chl) = v;
        }
        return;
    }
    if (OUTF32 && a.beta == 0.f && m0 + BM <= a.M && n0 + BN <= a.N && (a.ldc % 4) == 0 &&
        (reinterpret_cast<uintptr_t>(a.C) % 16) == 0 && (a.sC % 4) == 0) {
        // fp32 tile through LDS in two 64-row halves per wave (16 KB each, the wave's share of the
        // operand buffers): 16-B stores of whole 256-B row segments instead of 4-B stores with
        // per-element address arithmetic. 16-B chunk c of row ml sits at chunk c ^ (ml & 15), so
        // both the row-group writes of the accumulator layout and the row reads are conflict-free.
        float* wl = reinterpret_cast<float*>(lds + wave * 128 * 128);
        float* crow0 = reinterpret_cast<float*>(a.C) + (long long)z * a.sC + (long long)(m0 + 128 * wm) * a.ldc +
                       n0 + 64 * wn;
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            if (hf) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int nl = 16 * j + cl;
                const float bcol = (a.bias_mode == 1) ? a.bias[n0 + 64 * wn + nl] : 0.f;
#pragma unroll
                for (int ii = 0; ii < 4; ++ii)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int ml = 16 * ii + rq + r;
                        float v = a.alpha * acc[4 * hf + ii][j][r];
                        v += (a.bias_mode == 2) ? a.bias[m0 + 128 * wm + 64 * hf + ml] : bcol;
                        if (a.act == 1) v = gelu_tanh(v);
                        else if (a.act == 2) v = v * gelu_parts(v).cdf;
                        wl[ml * 64 + (((nl >> 2) ^ (ml & 15)) << 2) + (nl & 3)] = v;
                    }
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            float* crow = crow0 + (long long)(64 * hf) * a.ldc;
#pragma unroll 4
            for (int c = lane; c < 64 * 16; c += 64) {
                const int ml = c >> 4, ch = c & 15;
                const float4 v = *reinterpret_cast<const float4*>(wl + ml * 64 + ((ch ^ (ml & 15)) << 2));
                *reinterpret_cast<float4*>(crow + (long long)ml * a.ldc + 4 * ch) = v;
            }
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int n = n0 + 64 * wn + 16 * j + cl;
        if (n >= a.N) continue;
        const float bcol = (a.bias_mode == 1) ? a.bias[n] : 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + 128 * wm + 16 * i + rq + r;
                if (m >= a.M) continue;
                TC* cp = Cb + (long long)m * a.ldc + n;
                float v = a.alpha * acc[i][j][r];
                if (a.beta != 0.f) v = fmaf(a.beta, ld(cp), v);
                v += (a.bias_mode == 2) ? a.bias[m] : bcol;
                if (a.act == 1) v = gelu_tanh(v);
                else if (a.act == 2) v = v * gelu_parts(v).cdf;
                st(cp, v);
            }
    }
}

// C[zo] = epi(alpha * sum_s ws[zo * S + s] + beta * C[zo]), fixed summation order (deterministic)
template <bool OUTF32>
__global__ __launch_bounds__(256) void gemm8_reduce(G8Args a) {
    const long long MN = (long long)a.M * a.N;
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    const int zo = blockIdx.y;
    if (i >= MN) return;
    const float* w = a.ws + (long long)zo * a.S * MN + i;
    float v = 0.f;
    for (int s = 0; s < a.S; ++s) v += w[s * MN];
    const int m = (int)(i / a.N), n = (int)(i - (long long)m * a.N);
    typedef typename std::conditional<OUTF32, float, __hip_bfloat16>::type TC;
    TC* cp = reinterpret_cast<TC*>(a.C) + (long long)zo * a.sC + (long long)m * a.ldc + n;
    v *= a.alpha;
    if (a.beta != 0.f) v = fmaf(a.beta, ld(cp), v);
    v += a.bias_mode == 1 ? a.bias[n] : (a.bias_mode == 2 ? a.bias[m] : 0.f);
    if (a.act == 1) v = gelu_tanh(v);
    else if (a.act == 2) v = v * gelu_parts(v).cdf;
    st(cp, v);
}

int g_sched = 0;   // 1: two-K-tiles-ahead staging (DEEP), 0: one tile ahead (vfm_gemm8_set_schedule)

template <bool AK, bool BKC, bool OUTF32, bool DEEP>
void launch8k(const G8Args& a, int nwg, int zo, hipStream_t st) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)gemm8_kernel<AK, BKC, OUTF32, DEEP>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BUF);
        attr = true;
    }
    hipLaunchKernelGGL((gemm8_kernel<AK, BKC, OUTF32, DEEP>), dim3(nwg, zo * a.S), dim3(THREADS), 2 * BUF, st, a);
}

template <bool AK, bool BKC, bool OUTF32>
int launch8(const G8Args& a, int batch, hipStream_t st) {
    const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    const int zo = a.reduce ? 1 : batch;
    if (g_sched) launch8k<AK, BKC, OUTF32, true>(a, nwg, zo, st);
    else launch8k<AK, BKC, OUTF32, false>(a, nwg, zo, st);
    if (a.ws) {
        const long long MN = (long long)a.M * a.N;
        hipLaunchKernelGGL(gemm8_reduce<OUTF32>, dim3((unsigned)((MN + 255) / 256), zo), dim3(256), 0, st, a);
    }
    return launch_status();
}

// fp32 -> NP bf16 pieces along the reduction dimension (NP = 3: [hi | mid | lo], NP = 2: [hi | lo]).
//   kcont = 1: src [R][K] (row stride lds_) -> dst [R][NP K]; kcont = 0: src [K][R] -> dst [NP K][R].
template <int NP>
__global__ void split_f32_kernel(const float* __restrict__ src, __hip_bfloat16* __restrict__ dst, int R, int K,
                                 long long lds_, long long sb, long long db, int kcont) {
    const long long idx4 = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    const long long total = (long long)R * K;
    if (idx4 >= total) return;
    const int z = blockIdx.y;
    const float* s = src + (long long)z * sb;
    __hip_bfloat16* d = dst + (long long)z * db;
    // 4 consecutive elements along the contiguous dimension
    long long r, c, inner;
    if (kcont) { r = idx4 / K; c = idx4 % K; inner = K; }
    else       { r = idx4 / R; c = idx4 % R; inner = R; }   // r = k row, c = column
    const float4 v = *reinterpret_cast<const float4*>(s + r * lds_ + c);
    uint32_t p01[NP], p23[NP];
    split_pieces<NP>(v.x, v.y, p01);
    split_pieces<NP>(v.z, v.w, p23);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        long long off;
        if (kcont) off = r * ((long long)NP * K) + (long long)p * K + c;
        else       off = ((long long)p * K + r) * inner + c;
        *reinterpret_cast<uint2*>(d + off) = make_uint2(p01[p], p23[p]);
    }
}

}  // namespace

extern "C" int vfm_split_f32(const float* src, void* dst, int R, int K, long long ld, long long sb, long long db,
                             int batch, int precision, int kcont, void* stream) {
    if (!src || !dst || R <= 0 || K <= 0 || batch <= 0 || batch > 65535) return VFM_ERR_ARGS;
    if (precision != VFM_F32 && precision != VFM_F32X3) return VFM_ERR_ARGS;
    const int inner = kcont ? K : R;
    if (inner % 4 || ld % 4 || sb % 4 || ((uintptr_t)src % 16) || ((uintptr_t)dst % 8)) return VFM_NO_KERNEL;
    const long long total4 = ((long long)R * K) / 4;
    dim3 grid((unsigned)((total4 + 255) / 256), batch);
    if (precision == VFM_F32)
        hipLaunchKernelGGL(split_f32_kernel<3>, grid, dim3(256), 0, (hipStream_t)stream, src, (__hip_bfloat16*)dst, R, K,
                           ld, sb, db, kcont);
    else
        hipLaunchKernelGGL(split_f32_kernel<2>, grid, dim3(256), 0, (hipStream_t)stream, src, (__hip_bfloat16*)dst, R, K,
                           ld, sb, db, kcont);
    return launch_status();
}

// pieces per fp32 operand (1: bf16 operands) of a precision code, 0 = invalid
static int pieces_of(int precision) {
    return precision == VFM_F32 ? 3 : precision == VFM_F32X3 ? 2 : precision == VFM_BF16 ? 1 : 0;
}

// product terms over np pieces and their packed piece indices (G8Args::T / pa / pb)
template <int NP>
static void pack_terms(int& T, int& pa, int& pb) {
    T = Terms<NP>::N;
    pa = pb = 0;
    for (int t = 0; t < T; ++t) {
        pa |= Terms<NP>::a(t) << (2 * t);
        pb |= Terms<NP>::b(t) << (2 * t);
    }
}
static void terms_of(int np, int& T, int& pa, int& pb) {
    if (np == 3) pack_terms<3>(T, pa, pb);
    else if (np == 2) pack_terms<2>(T, pa, pb);
    else pack_terms<1>(T, pa, pb);
}

extern "C" int vfm_gemm8(const void* A, const void* B, void* C, const float* bias, int precision, int out_dtype, int M,
                         int N, int K, int batch, int a_kcont, long long lda, long long sA, int b_kcont, long long ldb,
                         long long sB, long long ldc, long long sC, float alpha, float beta, int bias_mode, int act,
                         float* workspace, int kchunk, int reduce_batch, void* stream) {
    if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0 || batch <= 0 || batch > 65535) return VFM_ERR_ARGS;
    if (out_dtype != VFM_BF16 && out_dtype != VFM_F32) return VFM_NO_KERNEL;
    const int np = pieces_of(precision);
    if (!np) return VFM_ERR_ARGS;
    if (bias_mode < 0 || bias_mode > 2 || (bias_mode && !bias) || act < 0 || act > 2) return VFM_ERR_ARGS;
    if (K % BK) return VFM_NO_KERNEL;
    const int a_c = a_kcont ? K : M, b_c = b_kcont ? K : N;
    if (a_c % 8 || b_c % 8 || lda % 8 || ldb % 8 || sA % 8 || sB % 8) return VFM_NO_KERNEL;
    if (((uintptr_t)A | (uintptr_t)B) % 16) return VFM_NO_KERNEL;
    if (lda < (a_kcont ? (long long)np * K : M) || ldb < (b_kcont ? (long long)np * K : N) || ldc < N)
        return VFM_ERR_ARGS;
    const long long nwg = (long long)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    if (nwg > 0x7fffffffLL) return VFM_ERR_ARGS;
    G8Args a;
    a.Kp = K;
    terms_of(np, a.T, a.pa, a.pb);
    a.A = (const __hip_bfloat16*)A; a.B = (const __hip_bfloat16*)B; a.C = C; a.bias = bias;
    a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.sA = sA; a.sB = sB; a.sC = sC;
    a.M = M; a.N = N; a.K = K; a.alpha = alpha; a.beta = beta; a.bias_mode = bias_mode; a.act = act;
    // virtual K-tiles V per output; S = ceil(V / kchunk) splits (kchunk <= 0: one split)
    const int V = a.T * (reduce_batch ? batch : 1) * (K / BK);
    a.Z = batch;
    a.reduce = reduce_batch ? 1 : 0;
    a.kchunk = (kchunk <= 0 || kchunk > V) ? V : kchunk;
    a.S = (V + a.kchunk - 1) / a.kchunk;
    a.ws = (a.S > 1 || a.reduce) ? workspace : nullptr;
    if ((a.S > 1 || a.reduce) && !workspace) return VFM_ERR_ARGS;
    if ((long long)(a.reduce ? 1 : batch) * a.S > 65535) return VFM_ERR_ARGS;
    hipStream_t st = (hipStream_t)stream;
    const bool of32 = out_dtype == VFM_F32;
#define VFM_G8(AK, BK_) return of32 ? launch8<AK, BK_, true>(a, batch, st) : launch8<AK, BK_, false>(a, batch, st)
    if (a_kcont && b_kcont) VFM_G8(true, true);
    if (a_kcont && !b_kcont) VFM_G8(true, false);
    if (!a_kcont && b_kcont) VFM_G8(false, true);
    VFM_G8(false, false);
#undef VFM_G8
}

// K-tile staging schedule of vfm_gemm8 (A/B switch for microbenchmarks): 1 = two K-tiles ahead
// (default), 0 = one K-tile ahead. Returns the previous value.
extern "C" int vfm_gemm8_set_schedule(int deep) {
    const int prev = g_sched;
    g_sched = deep ? 1 : 0;
    return prev;
}

// fp32 workspace floats vfm_gemm8 needs for (precision, M, N, K, batch, kchunk, reduce_batch); 0 = none
extern "C" int vfm_gemm8_workspace_floats(int precision, int M, int N, int K, int batch, int kchunk, int reduce_batch) {
    const int np = pieces_of(precision);
    if (!np || M <= 0 || N <= 0 || K <= 0 || batch <= 0 || K % BK) return -1;
    int T, pa, pb;
    terms_of(np, T, pa, pb);
    const int V = T * (reduce_batch ? batch : 1) * (K / BK);
    const int kc = (kchunk <= 0 || kchunk > V) ? V : kchunk;
    const int S = (V + kc - 1) / kc;
    if (S <= 1 && !reduce_batch) return 0;
    const long long n = (long long)M * N * S * (reduce_batch ? 1 : batch);
    return n > 0x7fffffffLL ? -1 : (int)n;
}
