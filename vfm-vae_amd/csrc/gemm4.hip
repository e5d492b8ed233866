// 256 x 256 bf16 GEMM with one wave per SIMD: the frozen SigLIP2 tower's linears and the decoder's bf16
// 1x1 convolutions (C[z] = epi(alpha A[z] B[z] + beta C[z])).
//
// Why a second 256-tile kernel beside gemm8: gemm8 runs 8 waves (two per SIMD, 128 x 64 each, 256
// registers) in a ping-pong of 8 barriers per K-tile. Here the 4 waves of a workgroup each own a
// 128 x 128 block (8 x 8 v_mfma_f32_16x16x32_bf16 tiles), so a wave has the SIMD's whole 512-entry
// register file: 256 accumulator registers, a register stage of the next K-tile (64), the fragments
// of one k32 step (64), and one barrier per K-tile. Per K-tile a wave issues 128 MFMAs (2048 SIMD
// cycles) beside 32 fragment reads, 16 global loads and 16 LDS writes.
//
//   * operand tiles [256][64] (K-contiguous) or [64][256] (M/N-contiguous) go global -> registers
//     (buffer loads, one VGPR offset per chunk, the K-tile advance a scalar offset) -> LDS (two
//     64 KB stages); the K-tile t+2 loads are issued while K-tile t computes, their LDS write
//     during K-tile t+1;
//   * LDS images: K-contiguous [256 rows][64 k] with 128-B rows, chunk ^= (row >> 1) & 7
//     (ds_read_b128 fragments); MN-contiguous as two [64 k][128] halves, 256-B rows, the 4 x 4
//     chunk swizzle of the transposed reads (ds_read_b64_tr_b16) -- the images of gemm8.hip;
//   * the MFMA takes the B fragment as its first operand, so the accumulator of a 16 x 16 tile
//     holds, per lane, 4 CONSECUTIVE columns of one C row: the epilogue stores straight from the
//     accumulators (8-B bf16 / 16-B fp32 per lane), no LDS staging;
//   * XCD-aware bijective block -> tile remap with grouped tile order (as gemm8).
#include "vfm_common.h"

namespace {

using namespace vfm;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int BM = 256, BN = 256, BK = 64, THREADS = 256;
#ifndef G4_SCHED
#define G4_SCHED 1
#endif
constexpr int OPB = 256 * BK * 2;          // bytes of one operand tile image (32 KB)
constexpr int STAGE = 2 * OPB;             // A + B images of one K-tile (64 KB)

struct G4Args {
    const __hip_bfloat16* A;
    const __hip_bfloat16* B;
    void* C;
    const float* bias;
    long long lda, ldb, ldc, sA, sB, sC;
    int M, N, K;
    float alpha, beta;
    int bias_mode, act, out_f32;
    unsigned spanA, spanB;   // buffer-descriptor ranges in bytes (< 2^31, checked on the host)
};

__device__ __forceinline__ int kc_off(int row, int ch) { return row * 128 + 16 * (ch ^ ((row >> 1) & 7)); }
__device__ __forceinline__ int mc_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int mc_off(int row, int ch) { return row * 256 + 16 * (ch ^ mc_swz(row)); }

__device__ __forceinline__ float gelu_tanh(float x) {
    const float u = 0.7978845608028654f * fmaf(0.044715f * x, x * x, x);
    const float e = __builtin_amdgcn_exp2f(2.8853900817779268f * u);
    return 0.5f * x * (2.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f));
}

// 16x16x32 operand fragment of 16-row (or 16-column) block `blk` of an operand image, k32 step t:
// lane l carries row (col) l & 15, k = 32 t + 8 (l >> 4) .. + 7.
//   K-contiguous image [256][64]: blk 0..15;
//   MN-contiguous image: two [64][128] halves of 16 KB, blk 0..15 (half blk >> 3).
template <bool KCONT>
__device__ __forceinline__ bf16x8 frag(const unsigned char* img, int blk, int t, int lane) {
    if (KCONT) {
        return *reinterpret_cast<const bf16x8*>(img + kc_off(16 * blk + (lane & 15), 4 * t + (lane >> 4)));
    } else {
        const unsigned char* h = img + (blk >> 3) * (OPB / 2);
        const int b = blk & 7;
        const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
        const int ch = 2 * b + (p >> 1);
        const int row = 32 * t + 8 * g + q;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(h + mc_off(row, ch) + 8 * (p & 1)));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(h + mc_off(row + 4, ch) + 8 * (p & 1)));
        return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
}

// Per-thread chunks i = 0..7 of an operand tile: global byte offset (relative to the K-tile origin) and LDS byte
// offset (inside the operand image) of chunk 0, and the per-chunk steps -- uniform, so the global step rides in
// the scalar offset of the buffer load and the LDS step in the ds_write's immediate.
//   K-contiguous: row (tid >> 3) + 32 i, 16-B chunk tid & 7: global += 32 ld per i, LDS += 4096 per i.
//   MN-contiguous: k-row (tid >> 5) + 8 i, 16-B chunk tid & 31 of the 256 columns: global += 8 ld per i, LDS +=
//   2048 per i with the 4 x 4 swizzle's k-row bits alternating between even and odd i (lofs[0] / lofs[1]).
// No clamping: rows / columns past the operand read what follows (their outputs are never stored) or, past the
// buffer descriptor's range, zeros.
template <bool KCONT>
__device__ __forceinline__ void chunk_base(long long ld, int outer0, int tid, unsigned& gofs, int (&lofs)[2]) {
    if (KCONT) {
        const int row = tid >> 3, ch = tid & 7;
        gofs = (unsigned)(((long long)(outer0 + row) * ld + 8 * ch) * 2);
        lofs[0] = lofs[1] = kc_off(row, ch);
    } else {
        const int krow = tid >> 5, ch = tid & 31;
        gofs = (unsigned)(((long long)krow * ld + outer0 + 8 * ch) * 2);
        lofs[0] = (ch >> 4) * (OPB / 2) + mc_off(krow, ch & 15);
        lofs[1] = (ch >> 4) * (OPB / 2) + mc_off(krow + 8, ch & 15) - 2048;
    }
}

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef __bf16 b2 __attribute__((ext_vector_type(2)));
    const f2 x = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(x, b2));
}

// Epilogue through the wave's 32 KB of LDS: acc[i][j][r] = C[mw + 16 i + (lane & 15)][nw + 16 j + 4 (lane >> 4) + r].
// The block's rows go to LDS as row-major [rows][128] images -- STF = 0: bf16 (plain bf16 output: all 128 rows,
// 256-B rows); STF = 1: fp32 (two halves of 64 rows, 512-B rows; fp32 output, or bf16 output with an epilogue,
// which is applied to the fp32 sums before the one rounding) -- XOR-swizzled so the 8-B / 16-B writes in the
// accumulator layout and the 16-B row reads are conflict-free, and leave as whole 16-B row pieces.
template <bool STF, bool OUTF32>
__device__ __forceinline__ void epilogue(const G4Args& a, const f32x4 (&acc)[8][8], unsigned char* wl, int lane, int mw,
                                         int nw, int z, bool plain) {
    typedef typename std::conditional<OUTF32, float, __hip_bfloat16>::type TC;
    constexpr int H = STF ? 2 : 1, RH = 128 / H;                 // halves, rows per half
    constexpr int RB = STF ? 512 : 256;                          // bytes per image row
    constexpr int PPR = RB / 16;                                 // 16-B pieces per row
    constexpr int VPP = STF ? 4 : 8;                             // values per piece
    TC* Cz = reinterpret_cast<TC*>(a.C) + (long long)z * a.sC;
    const bool vec = (a.ldc % 8) == 0 && (a.sC % 8) == 0 && (reinterpret_cast<uintptr_t>(a.C) % 16) == 0;
#pragma unroll
    for (int h = 0; h < H; ++h) {
#pragma unroll
        for (int ii = 0; ii < 8 / H; ++ii) {
            const int i = h * (8 / H) + ii;
            const int ml = 16 * ii + (lane & 15);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int c = 4 * j + (lane >> 4);              // 4-value chunk of the row (0..31)
                const f32x4 v = acc[i][j];
                if (STF) {
                    *reinterpret_cast<f32x4*>(wl + ml * RB + 16 * (c ^ (ml & 15))) = v;
                } else {
                    *reinterpret_cast<uint2*>(wl + ml * RB + 8 * (c ^ ((ml & 15) << 1))) =
                        make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
                }
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
#pragma unroll 2
        for (int q = lane; q < RH * PPR; q += 64) {
            const int ml = q / PPR, p = q % PPR;
            const int m = mw + h * RH + ml;
            const uint4 raw = *reinterpret_cast<const uint4*>(wl + ml * RB + 16 * (p ^ (ml & 15)));
            const int n = nw + VPP * p;
            if (m >= a.M || n >= a.N) continue;
            TC* dst = Cz + (long long)m * a.ldc + n;
            const bool whole = n + VPP <= a.N && vec;
            if (!STF && whole) {                                 // plain bf16: the staged bytes as they are
                *reinterpret_cast<uint4*>(dst) = raw;
                continue;
            }
            float v[VPP];
            if (STF) {
                const float4 f = __builtin_bit_cast(float4, raw);
                v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
            } else {
                const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v[2 * e] = __uint_as_float(w[e] << 16);
                    v[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
                }
            }
            if (!plain) {
                const float brow = (a.bias_mode == 2) ? a.bias[m] : 0.f;
#pragma unroll
                for (int e = 0; e < VPP; ++e) {
                    const bool in = n + e < a.N;
                    float x = a.alpha * v[e];
                    if (a.beta != 0.f && in) x = fmaf(a.beta, ld(dst + e), x);
                    x += (a.bias_mode == 1) ? (in ? a.bias[n + e] : 0.f) : brow;
                    if (a.act == 1) x = gelu_tanh(x);
                    else if (a.act == 2) x = x * gelu_parts(x).cdf;
                    v[e] = x;
                }
            }
            if (whole) {
                if (OUTF32) {
                    *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
                } else {
                    *reinterpret_cast<uint2*>(dst) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
                }
            } else {
                for (int e = 0; e < VPP && n + e < a.N; ++e) st(dst + e, v[e]);
            }
        }
        if (H > 1) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
        }
    }
}

template <bool AK, bool BKC, bool OUTF32>
__global__ __launch_bounds__(THREADS, 1) void gemm4_kernel(G4Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.N + BN - 1) / BN;
    const int nwg = tiles_m * tiles_n;
    int m0, n0;
    {
        const int bid = blockIdx.x;
        const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
        const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
        constexpr int GROUP = 4;
        const int gsz = GROUP * tiles_n, grp = tile / gsz, rem = tile - grp * gsz;
        const int rows_g = min(GROUP, tiles_m - grp * GROUP);
        m0 = (grp * GROUP + rem % rows_g) * BM;
        n0 = (rem / rows_g) * BN;
    }
    const int z = blockIdx.y;
    const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, 0, (int)a.spanA, 0x00020000);
    const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, 0, (int)a.spanB, 0x00020000);
    unsigned gA, gB;
    int lA[2], lB[2];
    chunk_base<AK>(a.lda, m0, tid, gA, lA);
    chunk_base<BKC>(a.ldb, n0, tid, gB, lB);
    const long long zA = (long long)z * a.sA * 2, zB = (long long)z * a.sB * 2;
    const unsigned stA = (unsigned)((AK ? 32 : 8) * a.lda * 2), stB = (unsigned)((BKC ? 32 : 8) * a.ldb * 2);
    const int KT = a.K / BK;
    uint4 stg[16];
    auto gload = [&](int kt) {
        const unsigned sa = (unsigned)(zA + (AK ? (long long)kt * BK * 2 : (long long)kt * BK * a.lda * 2));
        const unsigned sb = (unsigned)(zB + (BKC ? (long long)kt * BK * 2 : (long long)kt * BK * a.ldb * 2));
#pragma unroll
        for (int i = 0; i < 8; ++i)
            stg[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rA, gA, sa + i * stA, 0));
#pragma unroll
        for (int i = 0; i < 8; ++i)
            stg[8 + i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rB, gB, sb + i * stB, 0));
    };
    auto swrite = [&](int buf) {
        unsigned char* base = lds + buf * STAGE;
#pragma unroll
        for (int i = 0; i < 8; ++i)
            *reinterpret_cast<uint4*>(base + lA[i & 1] + (AK ? 4096 : 2048) * i) = stg[i];
#pragma unroll
        for (int i = 0; i < 8; ++i)
            *reinterpret_cast<uint4*>(base + OPB + lB[i & 1] + (BKC ? 4096 : 2048) * i) = stg[8 + i];
    };

    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{};

    // A blocks of this wave: rows 128 wm + 16 bi -> image block 8 wm + bi (both layouts); same for B
    const int ablk = 8 * wm, bblk = 8 * wn;
    bf16x8 a0[8], b0[8], a1[8], b1[8];          // fragments of k32 step 0 / 1
    auto reads = [&](const unsigned char* buf, int t, bf16x8 (&af)[8], bf16x8 (&bf)[8]) {
#pragma unroll
        for (int i = 0; i < 8; ++i) af[i] = frag<AK>(buf, ablk + i, t, lane);
#pragma unroll
        for (int j = 0; j < 8; ++j) bf[j] = frag<BKC>(buf + OPB, bblk + j, t, lane);
    };
    auto mfmas = [&](const bf16x8 (&af)[8], const bf16x8 (&bf)[8]) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
    };
    // LDS reads per k32 step: a K-contiguous fragment is one ds_read_b128, a transposed one two ds_read_b64_tr
    constexpr int NRD = (AK ? 8 : 16) + (BKC ? 8 : 16);

    // Pipeline (one barrier per K-tile, placed mid-tile):
    //   step 0 of K-tile t: MFMAs on (a0, b0) = step 0 of t, beside the reads of step 1 of t (a1, b1), the LDS
    //     write of K-tile t+1 (register stage, loaded during K-tile t-1) and the loads of K-tile t+2;
    //   lgkmcnt(0) + barrier: K-tile t+1 is in LDS for every wave, and every wave's reads of K-tile t-1's
    //     buffer are done (the next step 0 overwrites it);
    //   step 1 of K-tile t: MFMAs on (a1, b1) beside the reads of step 0 of K-tile t+1 (a0, b0).
    // K-tiles past the end are clamped (reloaded; written to the buffer nobody reads any more).
    gload(0);
    swrite(0);
    gload(1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    reads(lds, 0, a0, b0);
    for (int kt = 0; kt < KT; ++kt) {
        const int cur = kt & 1, nxt = cur ^ 1;
        reads(lds + cur * STAGE, 1, a1, b1);
        mfmas(a0, b0);
        swrite(nxt);
        gload(min(kt + 2, KT - 1));
        if (G4_SCHED) {
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);         // MFMA
                __builtin_amdgcn_sched_group_barrier(0x100, NRD / 16, 0);  // DS read
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);         // DS write
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);         // VMEM read
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        reads(lds + nxt * STAGE, 0, a0, b0);
        mfmas(a1, b1);
        if (G4_SCHED) {
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                __builtin_amdgcn_sched_group_barrier(0x100, NRD / 16, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
            }
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();               // every wave's LDS reads are done: the epilogue reuses LDS

    const bool plain = a.beta == 0.f && a.bias_mode == 0 && a.act == 0 && a.alpha == 1.f;
    unsigned char* wl = lds + wave * 32768;
    const int mw = m0 + 128 * wm, nw = n0 + 128 * wn;
    if (!OUTF32 && plain) epilogue<false, false>(a, acc, wl, lane, mw, nw, z, true);
    else epilogue<true, OUTF32>(a, acc, wl, lane, mw, nw, z, plain);
}

template <bool AK, bool BKC, bool OUTF32>
void launch4(const G4Args& a, int batch, hipStream_t st) {
    static bool attr[MAXDEV] = {};
    const int dv_attr = cur_dev();
    if (!attr[dv_attr]) {
        (void)hipFuncSetAttribute((const void*)gemm4_kernel<AK, BKC, OUTF32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  2 * STAGE);
        attr[dv_attr] = true;
    }
    const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    VFM_LAUNCH((gemm4_kernel<AK, BKC, OUTF32>), dim3(nwg, batch), dim3(THREADS), 2 * STAGE, st, a);
}

long long span4(int kcont, long long outer, long long kdim, long long ld, long long sb, int batch) {
    const long long rows = kcont ? outer : kdim;
    const long long cols = kcont ? kdim : outer;
    const long long e = (rows - 1) * ld + cols + (long long)(batch - 1) * sb;
    const long long bytes = e * 2;
    return bytes >= (1LL << 31) ? -1 : bytes;
}

}  // namespace

// bf16 operands: C[z] (M x N, ldc, batch stride sC) = epi(alpha A[z] B[z] + beta C[z]) with A [M, K]
// (a_kcont: K-contiguous rows of stride lda, else M-contiguous rows of K) and B [K, N] (b_kcont: B is
// given as N rows of K, stride ldb; else K rows of N). bias_mode 0 none / 1 per column / 2 per row;
// act 0 none / 1 tanh-GELU / 2 erf-GELU. Returns VFM_NO_KERNEL for shapes it does not take (K % 64,
// unaligned operands, > 2 GiB spans).
extern "C" int vfm_gemm4(const void* A, const void* B, void* C, const float* bias, int out_dtype, int M, int N, int K,
                         int batch, int a_kcont, long long lda, long long sA, int b_kcont, long long ldb, long long sB,
                         long long ldc, long long sC, float alpha, float beta, int bias_mode, int act, void* stream) {
    if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0 || batch <= 0 || batch > 65535) return VFM_ERR_ARGS;
    if (out_dtype != VFM_BF16 && out_dtype != VFM_F32) return VFM_NO_KERNEL;
    if (bias_mode < 0 || bias_mode > 2 || (bias_mode && !bias) || act < 0 || act > 2) return VFM_ERR_ARGS;
    if (K % BK) return VFM_NO_KERNEL;
    const int a_c = a_kcont ? K : M, b_c = b_kcont ? K : N;
    if (a_c % 8 || b_c % 8 || lda % 8 || ldb % 8 || sA % 8 || sB % 8) return VFM_NO_KERNEL;
    if (((uintptr_t)A | (uintptr_t)B) % 16) return VFM_NO_KERNEL;
    if (lda < (a_kcont ? (long long)K : M) || ldb < (b_kcont ? (long long)K : N) || ldc < N) return VFM_ERR_ARGS;
    const long long nwg = (long long)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    if (nwg > 0x7fffffffLL) return VFM_ERR_ARGS;
    const long long spA = span4(a_kcont, M, K, lda, sA, batch);
    const long long spB = span4(b_kcont, N, K, ldb, sB, batch);
    if (spA < 0 || spB < 0) return VFM_NO_KERNEL;
    G4Args a{};
    a.A = (const __hip_bfloat16*)A; a.B = (const __hip_bfloat16*)B; a.C = C; a.bias = bias;
    a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.sA = sA; a.sB = sB; a.sC = sC;
    a.M = M; a.N = N; a.K = K; a.alpha = alpha; a.beta = beta; a.bias_mode = bias_mode; a.act = act;
    a.spanA = (unsigned)spA; a.spanB = (unsigned)spB;
    a.out_f32 = out_dtype == VFM_F32;
    hipStream_t st = (hipStream_t)stream;
    const bool of32 = out_dtype == VFM_F32;
#define VFM_G4(AK, BK_) of32 ? launch4<AK, BK_, true>(a, batch, st) : launch4<AK, BK_, false>(a, batch, st)
    if (a_kcont && b_kcont) VFM_G4(true, true);
    else if (a_kcont && !b_kcont) VFM_G4(true, false);
    else if (!a_kcont && b_kcont) VFM_G4(false, true);
    else VFM_G4(false, false);
#undef VFM_G4
    return launch_status();
}
