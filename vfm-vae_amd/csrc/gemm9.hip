// 256 x 256 bf16 GEMM, one wave per SIMD, both operands staged by LDS-DMA: the hot path's bf16
// products (the frozen SigLIP2 tower's QKV / O / fc1 / fc2 linears, the decoder's bf16 1x1
// convolutions): C[z] = epi(alpha A[z] B[z] + beta C[z]).
//
// Why this structure (the third 256-tile kernel of the tree): hipBLASLt's fastest gfx950 kernel for
// these shapes is a 256-thread workgroup whose 4 waves each own a 128 x 128 block, with both operand
// tiles moved global -> LDS by LDS-DMA, two K-tiles in flight and two barriers per 64-deep K-tile
// (its code object's name and instruction mix: DirectToLds A/B, prefetch depth 2, wave tile 8 x 8 of
// v_mfma_f32_16x16x32_bf16). gemm4 (register staging, removed in round 6) lost its K-loop to the compiler serialising the
// staged loads behind the MFMA chain; gemm8 (8 waves of 128 x 64) spends twice the fragment reads per
// MFMA and 8 barriers per K-tile. Here, per K-tile and wave: 128 MFMAs, 32 fragment reads (one per
// MFMA in the two read phases), 16 LDS-DMA issues (one per ~5 MFMAs), 2 barriers:
//
//   phase 1: MFMAs on k-half 0 of K-tile t (fragments in VGPRs since the previous iteration) beside the
//            fragment reads of k-half 1 of t;
//   barrier B1 (after lgkmcnt(0)): every wave has read all of buffer t & 1;
//   phase 2: the rest of k-half 0 and most of k-half 1 beside the 16 LDS-DMA of K-tile t + 2 into
//            buffer t & 1;
//   vmcnt(16) + barrier B2: K-tile t + 1 (issued one iteration earlier) has landed for every wave;
//   phase 3: the last MFMAs of k-half 1 beside the fragment reads of k-half 0 of K-tile t + 1.
//
// The order of every MFMA, fragment read and DMA issue is pinned with sched_barrier(0) (the compiler
// inserts the counted lgkmcnt waits of the fragment reads itself); the DMAs are inline asm so that the
// waitcnt pass does not drain them before every ds_read, and only the counted waits above retire them.
// LDS images (two 64 KB stages, A then B): K-contiguous operands [256 rows][64 k] with 128-B rows and
// chunk ^= (row >> 1) & 7 (ds_read_b128 fragments); M/N-contiguous ones two [64 k][128] halves with
// 256-B rows and the 4 x 4 chunk swizzle of the transposed reads (ds_read_b64_tr_b16) -- the images of
// gemm8.hip, swizzled on the DMA source address (the destination is lane-linear).
// The MFMA takes the B fragment first, so a lane's accumulator holds 4 consecutive columns of one C
// row; the epilogue pairs column blocks with v_permlane16_swap and stores 16 B per lane straight from
// the accumulators (no LDS round trip).
#include <type_traits>

#include "vfm_common.h"

namespace {

using namespace vfm;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned v4u32 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BM = 256, BN = 256, BK = 64, THREADS = 256;
constexpr int OPB = 256 * BK * 2;          // one operand image (32 KB)
constexpr int STAGE = 2 * OPB;             // A + B of one K-tile (64 KB)
constexpr int LDS9P = 2 * STAGE + 8192;    // persistent form: + 4 epilogue slots of 2 KB

struct G9Args {
    const __hip_bfloat16* A;
    const __hip_bfloat16* B;
    void* C;
    const float* bias;
    long long lda, ldb, ldc, sA, sB, sC;
    int M, N, K;
    float alpha, beta;
    int bias_mode, act;
    long long spanA, spanB, spanC;    // operand / output spans in bytes (the one-tile-per-workgroup form: < 2^31)
    // batch-reduced split-K (persistent form): the K-tiles of all Z batches form one reduction of V = Z KTz
    // K-tiles cut into S chunks of kchunk; item (tile, chunk s) writes its fp32 partial to C[s] (the
    // workspace, sC = M N), gemm9_reduce sums the S partials in a fixed order
    int reduce, S, kchunk, KTz;
    // batched K-split (f32x6 pieces form): item batch index zz = z bs + s, chunk s of batch z's K-tiles; the
    // partial of (z, s) goes to C[zz] (the workspace), gemm9_reduce_batched sums each batch's bs partials
    int bs;
    // ConvNeXt-MLP GELU epilogues (EPI 4 / 5, bf16 C; see the epilogue): second output C2 (g), aux input H
    // (h, C's layout), per-(batch, row) scale rscale [Z][M] (null: 1), bias per row, and per-row partial sums
    // rs0 / rs1 [Z][2 tiles_n][M] of the backward (rs0 may be null)
    void* C2;
    const __hip_bfloat16* H;
    const float* rscale;
    float* rs0;
    float* rs1;
    // fp32-equivalent products (NP = 3, csrc/gemm8.hip's f32x6): fp32 operands as three exact bf16 pieces, T = 6
    // product terms per real K-tile run back to back as "virtual" K-tiles (term-fastest), term t reading piece
    // (pa >> 2t) & 3 of A at psA elements per piece and (pb >> 2t) & 3 of B at psB; T = 1 for bf16 operands
    int T, pa, pb;
    long long psA, psB;
};

__device__ __forceinline__ int kc_off(int row, int ch) { return row * 128 + 16 * (ch ^ ((row >> 1) & 7)); }
__device__ __forceinline__ int mc_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int mc_off(int row, int ch) { return row * 256 + 16 * (ch ^ mc_swz(row)); }

__device__ __forceinline__ float gelu_tanh(float x) {
    const float u = 0.7978845608028654f * fmaf(0.044715f * x, x * x, x);
    const float e = __builtin_amdgcn_exp2f(2.8853900817779268f * u);
    return 0.5f * x * (2.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f));
}

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    typedef __bf16 b2 __attribute__((ext_vector_type(2)));
    const f2 x = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(x, b2));
}

// One LDS-DMA instruction (buffer_load_dwordx4 ... offen lds): lane l's 16 B from rsrc + voff + soff land
// at M0 + 16 l. M0 and soff are SALU values (no VALU -> SGPR hand-off before the load).
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rsrc, unsigned voff, unsigned soff, unsigned m0) {
    asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(rsrc),
                 "s"(soff), "s"(m0)
                 : "memory");
}

// The same with the per-lane offset voff0 + su formed inside the statement (su: the slot's wave-uniform step):
// the compiler cannot hoist the 8 slot offsets of an operand out of the K-loop into 8 live VGPRs.
__device__ __forceinline__ void dma16s(__amdgpu_buffer_rsrc_t rsrc, unsigned voff0, unsigned su, unsigned m0) {
    unsigned t;
    asm volatile("v_add_u32 %0, %1, %2\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %3, 0 offen lds"
                 : "=&v"(t)
                 : "v"(voff0), "s"(su), "s"(rsrc), "s"(m0)
                 : "memory");
}

// dma16s with the LDS destination formed in M0 itself: m0 = mb + mo (two SGPR operands, no separate add)
__device__ __forceinline__ void dma16m(__amdgpu_buffer_rsrc_t rsrc, unsigned voff0, unsigned su, unsigned mb,
                                       unsigned mo) {
    unsigned t;
    asm volatile("v_add_u32 %0, %1, %2\n\ts_add_u32 m0, %4, %5\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %3, 0 offen lds"
                 : "=&v"(t)
                 : "v"(voff0), "s"(su), "s"(rsrc), "s"(mb), "s"(mo)
                 : "memory", "scc");
}

// The dword form (4 B per lane: 256 B per wave), for the epilogue's bias values.
__device__ __forceinline__ void dma4(__amdgpu_buffer_rsrc_t rsrc, unsigned voff, unsigned m0) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dword %0, %1, 0 offen lds" ::"v"(voff), "s"(rsrc), "s"(m0)
                 : "memory");
}

// Per-lane byte offset (from the operand's K-tile origin) of DMA slot u (0..7) of a 256-wide operand tile
// starting at outer0; destination byte u * 4096 + 16 tid of the operand image. Rows / columns past
// outer_n read a valid element whose product is never stored.
template <bool KCONT>
__device__ __forceinline__ unsigned dma_voff(long long ld, int outer0, int outer_n, int u, int tid) {
    if (KCONT) {
        const int row = 32 * u + (tid >> 3), chs = (tid & 7) ^ ((row >> 1) & 7);
        const int o = min(outer0 + row, outer_n - 1);
        return (unsigned)(((long long)o * ld + 8 * chs) * 2);
    } else {
        const int h = u >> 2, row = 16 * (u & 3) + (tid >> 4), chs = (tid & 15) ^ mc_swz(row);
        int o = outer0 + 128 * h + 8 * chs;
        if (o >= outer_n) o = 0;                       // (outer_n % 8 == 0): a valid chunk, result unused
        return (unsigned)(((long long)row * ld + o) * 2);
    }
}

// 16x16x32 fragment of 16-row block blk (0..15) of an operand image, k32 step t: lane l carries row
// (column) l & 15, k = 32 t + 8 (l >> 4) .. + 7.
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

// acc += x y on the matrix core with the accumulator pinned to AGPRs: the builtin's form lets the register
// allocator split the 256 accumulator registers between the two files and shuffle them every K-tile
// (hundreds of v_accvgpr moves per K-tile, which is also what held gemm4's loop back)
__device__ __forceinline__ void mfma_acc(f32x4& c, const bf16x8& x, const bf16x8& y) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(x), "v"(y));
}

// acc = x y (the first K-tile of an output tile: the accumulator is defined by the MFMA, no zeroing pass and no
// loop-carried zeros for the register allocator to juggle)
__device__ __forceinline__ void mfma_acc0(f32x4& c, const bf16x8& x, const bf16x8& y) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(x), "v"(y));
}

#define SB() __builtin_amdgcn_sched_barrier(0)
#define VMCNT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
template <int N>
__device__ __forceinline__ void vmcnt_const() {
    static_assert(N >= 0 && N <= 63, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// operand DMAs of a K-tile moved from phase 2 into phase 3 of the persistent kernel (A/B builds; 0: none)
#ifndef G9_P3
#define G9_P3 0
#endif
// MFMAs in phase 1 (k-half 0, beside the k-half-1 fragment reads) and phase 3 (k-half 1, beside the next K-tile's
// k-half-0 reads) of the persistent kernel; phase 2 (the DMA window between the barriers) takes the rest
#ifndef G9_PH1
#define G9_PH1 26
#endif
#ifndef G9_PH3
#define G9_PH3 21
#endif

template <bool AK, bool BKC, bool OUTF32>
__global__ __launch_bounds__(THREADS, 1) void gemm9_kernel(G9Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.N + BN - 1) / BN;
    const int nwg = tiles_m * tiles_n;
    int m0, n0;
    {
        // XCD-aware bijective remap, then grouped order (GROUP tile-rows per column sweep), as gemm8
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
    unsigned voA[8], voB[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        voA[u] = dma_voff<AK>(a.lda, m0, a.M, u, tid);
        voB[u] = dma_voff<BKC>(a.ldb, n0, a.N, u, tid);
    }
    const unsigned m0A = (unsigned)(size_t)(lds_void*)lds + (unsigned)wave * 1024u;
    const unsigned zA = (unsigned)(z * a.sA * 2), zB = (unsigned)(z * a.sB * 2);
    const unsigned dkA = (unsigned)(AK ? BK * 2 : BK * a.lda * 2), dkB = (unsigned)(BKC ? BK * 2 : BK * a.ldb * 2);
    const int KT = a.K / BK;

    // DMA slot g (0..7 A, 8..15 B) of K-tile kt into buffer buf; past the last K-tile the descriptors have no
    // records (the DMA writes zeros into a buffer nobody reads any more and moves no memory), so every K-tile
    // runs the same body
    const __amdgpu_buffer_rsrc_t nA = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, 0, 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t nB = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, 0, 0, 0x00020000);
    auto dma = [&](int g, int buf, int kt) __attribute__((always_inline)) {
        const bool live = kt < KT;
        if (g < 8) dma16(live ? rA : nA, voA[g], zA + (unsigned)kt * dkA, m0A + buf * STAGE + g * 4096);
        else dma16(live ? rB : nB, voB[g - 8], zB + (unsigned)kt * dkB, m0A + buf * STAGE + OPB + (g - 8) * 4096);
    };

    f32x4 acc[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{};
    bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
    // fragment read r (0..15) of k-half h from buffer buf, in the order A0 B0 A1..A7 B1..B7: the MFMAs of a
    // k-half walk j (B block) outer, i (A block) inner, so the first MFMA needs reads 0 and 1 only
    auto rd = [&](int h, int r, int buf) __attribute__((always_inline)) {
        const unsigned char* base = lds + buf * STAGE;
        const bool isb = (r == 1) || r >= 9;
        const int idx = r == 0 ? 0 : r == 1 ? 0 : r <= 8 ? r - 1 : r - 8;
        if (!isb) {
            const bf16x8 v = frag<AK>(base, 8 * wm + idx, h, lane);
            if (h == 0) fa0[idx] = v; else fa1[idx] = v;
        } else {
            const bf16x8 v = frag<BKC>(base + OPB, 8 * wn + idx, h, lane);
            if (h == 0) fb0[idx] = v; else fb1[idx] = v;
        }
    };
    // MFMA q (0..63) of k-half h: B block j = q / 8, A block i = q % 8
    auto mf = [&](int h, int q) __attribute__((always_inline)) {
        const int j = q >> 3, i = q & 7;
        mfma_acc(acc[i][j], h ? fb1[j] : fb0[j], h ? fa1[i] : fa0[i]);
    };

    // prologue: K-tiles 0 and 1 in flight (1 as a null DMA when K has one tile), K-tile 0 landed, k-half 0
    // fragments of K-tile 0 read
#pragma unroll
    for (int g = 0; g < 16; ++g) dma(g, 0, 0);
#pragma unroll
    for (int g = 0; g < 16; ++g) dma(g, 1, 1);
    VMCNT(16);
    __builtin_amdgcn_s_barrier();
    SB();
#pragma unroll
    for (int r = 0; r < 16; ++r) rd(0, r, 0);
    SB();

    // one K-tile per iteration (the last one's phase 3 reads a buffer that holds no K-tile: unused)
    for (int t = 0; t < KT; ++t) {
        const int cur = t & 1;
        // phase 1: 26 MFMAs of k-half 0 beside the 16 reads of k-half 1
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            mf(0, q);
            SB();
            rd(1, q, cur);
            SB();
        }
#pragma unroll
        for (int q = 16; q < 26; ++q) mf(0, q);
        SB();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        SB();
        // phase 2: 38 MFMAs of k-half 0 + 43 of k-half 1 beside the 16 DMA of K-tile t + 2 (every 5th)
#pragma unroll
        for (int s = 0; s < 81; ++s) {
            if (s < 38) mf(0, 26 + s);
            else mf(1, s - 38);
            SB();
            if ((s % 5) == 4 && s / 5 < 16) {
                dma(s / 5, cur, t + 2);
                SB();
            }
        }
        VMCNT(16);
        __builtin_amdgcn_s_barrier();
        SB();
        // phase 3: 21 MFMAs of k-half 1 beside the 16 reads of k-half 0 of K-tile t + 1
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            mf(1, 43 + q);
            SB();
            rd(0, q, cur ^ 1);
            SB();
        }
#pragma unroll
        for (int q = 59; q < 64; ++q) mf(1, q);
        SB();
    }
    VMCNT(0);                                  // the null DMAs of the last two iterations
    // the asm MFMAs are opaque to the hazard recognizer: wait out the last results (XDL write -> VALU read)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");

    // epilogue straight from the accumulators: acc[i][j][r] = C[mw + 16 i + (l & 15)][nw + 16 j + 4 (l >> 4) + r]
    const int mw = m0 + 128 * wm, nw = n0 + 128 * wn;
    const int l15 = lane & 15, row4 = lane >> 4;
    typedef typename std::conditional<OUTF32, float, __hip_bfloat16>::type TC;
    TC* Cz = reinterpret_cast<TC*>(a.C) + (long long)z * a.sC;
    const bool plain = a.beta == 0.f && a.bias_mode == 0 && a.act == 0 && a.alpha == 1.f;
    // epilogue value of column n of row m (the generic form; plain products skip it)
    auto epi = [&](float x, int m, bool mok, int n, const TC* crow) __attribute__((always_inline)) {
        const bool in = mok && n < a.N;
        x *= a.alpha;
        if (a.beta != 0.f && in) x = fmaf(a.beta, ld(crow + n), x);
        x += a.bias_mode == 1 ? (n < a.N ? a.bias[n] : 0.f) : (a.bias_mode == 2 && mok ? a.bias[m] : 0.f);
        if (a.act == 1) x = gelu_tanh(x);
        else if (a.act == 2) x = x * gelu_parts(x).cdf;
        return x;
    };
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int m = mw + 16 * i + l15;
        const bool mok = m < a.M;
        TC* crow = Cz + (long long)(mok ? m : 0) * a.ldc;
#pragma unroll
        for (int jp = 0; jp < 4; ++jp) {
            const int j0 = 2 * jp, j1 = j0 + 1;
            f32x4 v0 = acc[i][j0], v1 = acc[i][j1];
            if (!plain) {
                const int n0c = nw + 16 * j0 + 4 * row4, n1c = n0c + 16;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v0[r] = epi(v0[r], m, mok, n0c + r, crow);
                    v1[r] = epi(v1[r], m, mok, n1c + r, crow);
                }
            }
            if (OUTF32) {
                const int n0c = nw + 16 * j0 + 4 * row4;
                float* cf = reinterpret_cast<float*>(crow);
                if (mok && n0c < a.N) *reinterpret_cast<f32x4*>(cf + n0c) = v0;
                if (mok && n0c + 16 < a.N) *reinterpret_cast<f32x4*>(cf + n0c + 16) = v1;
            } else {
                const uint32_t a0 = pack_bf16x2(v0[0], v0[1]), a1 = pack_bf16x2(v0[2], v0[3]);
                const uint32_t b0 = pack_bf16x2(v1[0], v1[1]), b1 = pack_bf16x2(v1[2], v1[3]);
                // rows (16-lane groups) 1 and 3 of (a0, a1) <-> rows 0 and 2 of (b0, b1): each lane then holds 8
                // consecutive columns (a0 a1 b0 b1) of block j0 (rows 0, 2) or j1 (rows 1, 3)
                const auto s0 = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
                const auto s1 = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
                const int n = nw + 16 * (j0 + (row4 & 1)) + 8 * (row4 >> 1);
                if (mok && n < a.N)
                    *reinterpret_cast<uint4*>(reinterpret_cast<__hip_bfloat16*>(crow) + n) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
            }
        }
    }
}

// Persistent form: one workgroup per CU walks items (z, tile) = blockIdx.x, + gridDim.x, ...; the K-tiles of
// consecutive items form one stream, so the DMA of the next item's first two K-tiles is issued during the
// current item's last two (no prologue per item) and the epilogue's stores leave while the next item's first
// K-tile computes. The stores are buffer stores with an out-of-range offset for the lanes outside C (the
// hardware drops them), so every wave issues exactly NST of them and the counted vmcnt waits stay exact:
// at B2 of an item's first K-tile the stores are younger than the DMA waited for.
__device__ __forceinline__ void item_tile(int item, int nwg, int total, int tiles_m, int tiles_n, int& z, int& m0,
                                          int& n0) {
    // XCD-aware bijective remap over all items (blocks b and b + 8 share an XCD; with gridDim.x % 8 == 0 the
    // items a workgroup walks stay on its XCD), then grouped order inside the output batch
    const int xcd = item & 7, q8 = total >> 3, r8 = total & 7;
    const int g = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (item >> 3);
    z = g / nwg;
    const int tile = g - z * nwg;
    constexpr int GROUP = 4;
    const int gsz = GROUP * tiles_n, grp = tile / gsz, rem = tile - grp * gsz;
    const int rows_g = min(GROUP, tiles_m - grp * GROUP);
    m0 = (grp * GROUP + rem % rows_g) * BM;
    n0 = (rem / rows_g) * BN;
}

// EPI 0: plain C = A B; EPI 1 / 2 / 3: C = act(alpha A B + bias), act = none / tanh-GELU / erf-GELU, with the
// item's 256 bias values (per column or per
// row) moved into one of 4 LDS slots by a dword LDS-DMA that rides with every K-tile's 16 operand DMAs (the
// slot of the cursor's item, so the counted waits cover it and it has landed before the item's epilogue)
// ConvNeXt-MLP GELU epilogues (reference networks/utils/convnext_utils.py:135-142: pwconv1 -> GELU ->
// pwconv2 with the modulation scale s[b, o] and bias b1[o] of channel o = GEMM row; the roundings of the
// separate scale_bias_gelu kernels, csrc/decoder.hip gelu_fwd / gelu_bwd):
//   EPI 4 (forward):  h = bf16(acc) -> C (when non-null); g = bf16(GELU(h s + b1)) -> C2;
//   EPI 5 (backward): dg = bf16(acc); dz = dg GELU'(h s + b1) with h read from H; dh = bf16(dz s) -> C; per-row
//                     sums of dz h and dz over the wave's 128 columns -> rs0 / rs1 at [z][2 tn + wn][m].
// Row values (b1, s) come from the item's LDS slot; every wave issues a fixed number of buffer stores
// (out-of-range lanes and a null output: offsets past the descriptor's records, dropped), which the
// counted waits of the next item's first K-tile rely on.
template <int EPI>
__device__ __forceinline__ void gelu_epilogue9(const G9Args& a, const f32x4 (&acc)[8][8], const float* bsl,
                                               __amdgpu_buffer_rsrc_t rC, int z, int m0, int n0, int wm, int wn,
                                               int l15, int row4, int tiles_n) {
    auto rsrc2 = [&](const void* base, long long off, long long span) __attribute__((always_inline)) {
        const long long left = base ? span - off : 0;
        return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)base + (base ? off : 0)), 0,
                                                 (int)(left > 0 ? (left < 0x7fffffffLL ? left : 0x7fffffffLL) : 0),
                                                 0x00020000);
    };
    const int mw = m0 + 128 * wm, nw = n0 + 128 * wn;
    const bool hasS = a.rscale != nullptr;
    const long long zoff = (long long)z * a.sC * 2;
    const __amdgpu_buffer_rsrc_t rC2 = rsrc2(a.C2, zoff, a.spanC);
    const __amdgpu_buffer_rsrc_t rH = rsrc2(a.H, zoff, a.spanC);
    const long long nparts = 2LL * tiles_n;
    const long long pbase = ((long long)z * nparts + 2 * (n0 / BN) + wn) * a.M;
    const __amdgpu_buffer_rsrc_t rP0 = rsrc2(a.rs0, pbase * 4, (long long)a.M * 4 * nparts * (z + 1));
    const __amdgpu_buffer_rsrc_t rP1 = rsrc2(a.rs1, pbase * 4, (long long)a.M * 4 * nparts * (z + 1));
    // H prefetch one row block ahead (EPI 5): the lane's 4 + 4 columns of blocks j0, j1 for each column pair
    uint2 hn[4][2];
    // (unconditional loads: rows / columns past C read garbage of the same slice or zeros past its end -- the
    // masked dz ignores them -- and no select in the address lets the compiler sink a load into a branch)
    auto load_h = [&](int i, uint2 (&hv)[4][2]) __attribute__((always_inline)) {
        const unsigned ob = (unsigned)((mw + 16 * i + l15) * a.ldc + nw + 4 * row4) * 2u;
#pragma unroll
        for (int jp = 0; jp < 4; ++jp) {
            hv[jp][0] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rH, ob + 64u * jp, 0, 0));
            hv[jp][1] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rH, ob + 64u * jp + 32u, 0, 0));
        }
    };
    if (EPI == 5) load_h(0, hn);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int ml = 128 * wm + 16 * i + l15;
        const int m = m0 + ml;
        const bool mok = m < a.M;
        const float b1v = bsl[ml], scv = hasS ? bsl[256 + ml] : 1.f;
        uint2 hc[4][2];
        if (EPI == 5) {
#pragma unroll
            for (int jp = 0; jp < 4; ++jp) {
                hc[jp][0] = hn[jp][0];
                hc[jp][1] = hn[jp][1];
            }
            if (i < 7) load_h(i + 1, hn);
        }
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int jp = 0; jp < 4; ++jp) {
            const int j0 = 2 * jp, j1 = j0 + 1;
            const int n0c = nw + 16 * j0 + 4 * row4;
            const f32x4 v0 = acc[i][j0], v1 = acc[i][j1];
            uint32_t pa[2], pb[2], qa[2], qb[2];        // bf16 pairs of blocks j0 (a) / j1 (b): C, C2 outputs
            if (EPI == 4) {
                float h0[4], h1[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    h0[r] = __builtin_bit_cast(float, (uint32_t)__builtin_bit_cast(unsigned short, __float2bfloat16(v0[r])) << 16);
                    h1[r] = __builtin_bit_cast(float, (uint32_t)__builtin_bit_cast(unsigned short, __float2bfloat16(v1[r])) << 16);
                }
                float g0[4], g1[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float z0 = fmaf(h0[r], scv, b1v), z1 = fmaf(h1[r], scv, b1v);
                    g0[r] = z0 * gelu_parts(z0).cdf;
                    g1[r] = z1 * gelu_parts(z1).cdf;
                }
                pa[0] = pack_bf16x2(h0[0], h0[1]); pa[1] = pack_bf16x2(h0[2], h0[3]);
                pb[0] = pack_bf16x2(h1[0], h1[1]); pb[1] = pack_bf16x2(h1[2], h1[3]);
                qa[0] = pack_bf16x2(g0[0], g0[1]); qa[1] = pack_bf16x2(g0[2], g0[3]);
                qb[0] = pack_bf16x2(g1[0], g1[1]); qb[1] = pack_bf16x2(g1[2], g1[3]);
            } else {
                float d0[4], d1[4];
                const uint32_t hw[4] = {hc[jp][0].x, hc[jp][0].y, hc[jp][1].x, hc[jp][1].y};
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float dg0 = __builtin_bit_cast(float, (uint32_t)__builtin_bit_cast(unsigned short, __float2bfloat16(v0[r])) << 16);
                    const float dg1 = __builtin_bit_cast(float, (uint32_t)__builtin_bit_cast(unsigned short, __float2bfloat16(v1[r])) << 16);
                    const uint32_t w0 = hw[r >> 1], w1 = hw[2 + (r >> 1)];
                    const float hv0 = __builtin_bit_cast(float, (r & 1) ? (w0 & 0xffff0000u) : (w0 << 16));
                    const float hv1 = __builtin_bit_cast(float, (r & 1) ? (w1 & 0xffff0000u) : (w1 << 16));
                    const GeluParts gp0 = gelu_parts(fmaf(hv0, scv, b1v)), gp1 = gelu_parts(fmaf(hv1, scv, b1v));
                    float dz0 = dg0 * (gp0.cdf + gp0.zpdf), dz1 = dg1 * (gp1.cdf + gp1.zpdf);
                    if (!mok || n0c + r >= a.N) dz0 = 0.f;
                    if (!mok || n0c + 16 + r >= a.N) dz1 = 0.f;
                    s0 = fmaf(dz0, hv0, s0);
                    s1 += dz0;
                    s0 = fmaf(dz1, hv1, s0);
                    s1 += dz1;
                    d0[r] = dz0 * scv;
                    d1[r] = dz1 * scv;
                }
                pa[0] = pack_bf16x2(d0[0], d0[1]); pa[1] = pack_bf16x2(d0[2], d0[3]);
                pb[0] = pack_bf16x2(d1[0], d1[1]); pb[1] = pack_bf16x2(d1[2], d1[3]);
            }
            const int n = nw + 16 * (j0 + (row4 & 1)) + 8 * (row4 >> 1);
            const unsigned o = (mok && n < a.N) ? (unsigned)(((long long)m * a.ldc + n) * 2) : 0x80000000u;
            {
                const auto x0 = __builtin_amdgcn_permlane16_swap(pa[0], pb[0], false, false);
                const auto x1 = __builtin_amdgcn_permlane16_swap(pa[1], pb[1], false, false);
                const v4u32 d = {x0[0], x1[0], x0[1], x1[1]};
                __builtin_amdgcn_raw_buffer_store_b128(d, rC, o, 0, 0);
            }
            if (EPI == 4) {
                const auto x0 = __builtin_amdgcn_permlane16_swap(qa[0], qb[0], false, false);
                const auto x1 = __builtin_amdgcn_permlane16_swap(qa[1], qb[1], false, false);
                const v4u32 d = {x0[0], x1[0], x0[1], x1[1]};
                __builtin_amdgcn_raw_buffer_store_b128(d, rC2, o, 0, 0);
            }
        }
        if (EPI == 5) {
            // the 4 lanes of a row (l >> 4 = 0..3): xor 16, 32 (fixed order, identical on every lane)
            s0 += __shfl_xor(s0, 16);
            s1 += __shfl_xor(s1, 16);
            s0 += __shfl_xor(s0, 32);
            s1 += __shfl_xor(s1, 32);
            const unsigned po = (row4 == 0 && mok) ? (unsigned)((long long)m * 4) : 0x80000000u;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, s0), rP0, po, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, s1), rP1, po, 0, 0);
        }
        SB();
    }
}

// K range of an item: its batch's KT K-tiles, or (reduce) chunk s = z of the batch-concatenated reduction
__device__ __forceinline__ void item_k_range(const G9Args& a, int z, int KT, int& v0, int& n) {
    if (a.reduce) {
        const int V = a.KTz * a.reduce * a.T;            // virtual K-tiles (kchunk: a multiple of T)
        v0 = z * a.kchunk;
        n = min(V, v0 + a.kchunk) - v0;
    } else if (a.bs > 1) {                             // batched split: chunk z % bs of the batch's K-tiles
        const int V = KT * a.T;
        v0 = (z % a.bs) * a.kchunk;
        n = min(V, v0 + a.kchunk) - v0;
    } else {
        v0 = 0;
        n = KT * a.T;
    }
}

template <bool AK, bool BKC, bool OUTF32, int EPI, int NP = 1>
__global__ __launch_bounds__(THREADS, 1) void gemm9p_kernel(G9Args a, int total) {
    constexpr int NP_T = NP == 3 ? 6 : NP == 2 ? 3 : 1;     // product terms per real K-tile (a.T)
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1, wn = wave & 1;
    const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.N + BN - 1) / BN;
    const int nwg = tiles_m * tiles_n;
    const int G = gridDim.x;
    const int KT = a.K / BK;
    const unsigned m0A = (unsigned)(size_t)(lds_void*)lds + (unsigned)wave * 1024u;
    const unsigned dkA = (unsigned)(AK ? BK * 2 : BK * a.lda * 2), dkB = (unsigned)(BKC ? BK * 2 : BK * a.ldb * 2);

    // DMA cursor: the item and K-tile of the next stream position to issue. Per-lane offsets are relative to the
    // operand tile's K-tile origin and the same for every item and K-tile; the origin itself moves the buffer
    // descriptor's base (SALU), whose record count is the operand's remaining span, so rows / columns past the
    // operand read in-bounds garbage or zeros that no stored output depends on, and nothing past its end.
    // slot u of an operand: voff(u) = voff(0) + a wave-uniform step (the swizzle chunk does not depend on u)
    const unsigned voA0 = dma_voff<AK>(a.lda, 0, 0x7fffffff, 0, tid), voB0 = dma_voff<BKC>(a.ldb, 0, 0x7fffffff, 0, tid);
    auto ustep = [&](bool kc, long long ld, int u) __attribute__((always_inline)) {
        return (unsigned)((kc ? 32LL * u * ld : 16LL * (u & 3) * ld + 128 * (u >> 2)) * 2);
    };
    int d_item = blockIdx.x, d_kt = 0, d_k = 0;   // d_k: the cursor item's index among this workgroup's items
    int d_KT = KT, d_v0 = 0, d_z = 0;             // the cursor item's K-tiles, first reduction K-tile, batch
    int d_term = 0, d_kk = 0;                     // (NP = 3) the cursor's product term and real K-tile
    long long offA = 0, offB = 0;                 // byte offsets of the cursor item's tile origin in A / B
    long long offS = 0, offR = 0;                 // byte offsets of the cursor item's bias values / row scales
    auto setup_dma = [&](int item) __attribute__((always_inline)) {
        int z, m0, n0;
        item_tile(item, nwg, total, tiles_m, tiles_n, z, m0, n0);
        offA = (AK ? (long long)m0 * a.lda : (long long)m0) * 2;
        offB = (BKC ? (long long)n0 * a.ldb : (long long)n0) * 2;
        d_z = a.bs > 1 ? z / a.bs : z;
        item_k_range(a, z, KT, d_v0, d_KT);
        offS = (long long)(a.bias_mode == 1 ? n0 : m0) * 4;
        offR = ((long long)z * a.M + m0) * 4;
    };
    auto rsrc = [&](const void* base, long long off, long long span) __attribute__((always_inline)) {
        // 64-bit base, record count clamped to 31 bits: a tile's accesses from its origin stay far below that
        const long long left = span - off;
        return __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)base + off), 0,
                                                 (int)(left > 0 ? (left < 0x7fffffffLL ? left : 0x7fffffffLL) : 0),
                                                 0x00020000);
    };
    __amdgpu_buffer_rsrc_t rA = rsrc(a.A, 0, a.spanA), rB = rsrc(a.B, 0, a.spanB), rS = rA;
    // epilogue slot of an item (2 KB): [0, 1 KB) its 256 bias values (per column or per row, zeros without a
    // bias), [1 KB, 2 KB) its 256 row scales (EPI 4 / 5, rscale of the item's batch)
    const long long spanS = EPI && a.bias ? (long long)(a.bias_mode == 1 ? a.N : a.M) * 4 : 0;
    const long long spanR = EPI >= 4 && a.rscale ? (long long)a.M * 4 * (a.reduce ? 1 : 1) : 0;
    __amdgpu_buffer_rsrc_t rR = rA;
    const unsigned sl0 = (unsigned)(size_t)(lds_void*)lds + 2 * STAGE + (unsigned)wave * 256u;
    const unsigned voS = (unsigned)tid * 4u;          // wave w: values 64 w .. 64 w + 63 of the slot
    auto dma = [&](int g, int buf) __attribute__((always_inline)) {
        const unsigned mb = m0A + (unsigned)buf * STAGE;
        if (g < 8) dma16m(rA, voA0, ustep(AK, a.lda, g), mb, (unsigned)(g * 4096));
        else if (g < 16) dma16m(rB, voB0, ustep(BKC, a.ldb, g - 8), mb, (unsigned)(OPB + (g - 8) * 4096));
        else if (g == 16) dma4(rS, voS, sl0 + (unsigned)(d_k & 3) * 2048u);          // the cursor item's bias
        else dma4(rR, voS, sl0 + (unsigned)(d_k & 3) * 2048u + 1024u);               // and row scales (EPI 4 / 5)
    };
    // descriptors of the cursor's position (after setup_dma / a K-tile step)
    // (past the workgroup's last item: no records, the DMA writes zeros into a buffer nobody reads again)
    // The operand descriptors of the cursor as (64-bit address, record count) in SGPRs: rebuilt in full at an
    // item's first K-tile (and per K-tile of a batch-reduced product, whose K-tiles cross batches), else
    // advanced by one K-tile's step in SALU asm (a 64-bit add and a saturating subtract per operand instead of
    // the multiplies, compares and selects of a full rebuild in every K-tile)
    unsigned aLo = 0, aHi = 0, aN = 0, bLo = 0, bHi = 0, bN = 0;
    auto clamp31 = [](long long left) __attribute__((always_inline)) {
        return (unsigned)(left > 0 ? (left < 0x7fffffffLL ? left : 0x7fffffffLL) : 0);
    };
    auto mk = [](unsigned lo, unsigned hi, unsigned n) __attribute__((always_inline)) {
        return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), 0, (int)n, 0x00020000);
    };
    auto point = [&]() __attribute__((always_inline)) {
        const bool live = d_item < total;
        int zt = d_z, kk = NP > 1 ? d_kk + (a.bs > 1 ? d_v0 / NP_T : 0) : d_kt;
        if (a.reduce) {                         // reduction K-tile v -> (batch, K-tile of that batch)
            const int v = NP > 1 ? d_v0 / NP_T + d_kk : d_v0 + d_kt;
            zt = v / a.KTz;
            kk = v - zt * a.KTz;
        }
        long long pofa = 0, pofb = 0;           // the term's piece planes
        if (NP > 1) {
            pofa = ((a.pa >> (2 * d_term)) & 3) * a.psA;
            pofb = ((a.pb >> (2 * d_term)) & 3) * a.psB;
        }
        const long long cA = offA + (zt * a.sA + (long long)kk * (dkA / 2) + pofa) * 2;
        const long long cB = offB + (zt * a.sB + (long long)kk * (dkB / 2) + pofb) * 2;
        const unsigned long long pA = (unsigned long long)((const char*)a.A + cA);
        const unsigned long long pB = (unsigned long long)((const char*)a.B + cB);
        aLo = __builtin_amdgcn_readfirstlane((unsigned)pA);
        aHi = __builtin_amdgcn_readfirstlane((unsigned)(pA >> 32));
        aN = __builtin_amdgcn_readfirstlane(live ? clamp31(a.spanA - cA) : 0u);
        bLo = __builtin_amdgcn_readfirstlane((unsigned)pB);
        bHi = __builtin_amdgcn_readfirstlane((unsigned)(pB >> 32));
        bN = __builtin_amdgcn_readfirstlane(live ? clamp31(a.spanB - cB) : 0u);
        rA = mk(aLo, aHi, aN);
        rB = mk(bLo, bHi, bN);
        if (EPI) rS = rsrc(a.bias, offS, live ? spanS : 0);
        if (EPI >= 4) rR = rsrc(a.rscale, offR, (live && spanR) ? (long long)d_z * a.M * 4 + spanR : 0);
    };
    auto step = [&]() __attribute__((always_inline)) {
        asm volatile("s_add_u32 %0, %0, %6\n\ts_addc_u32 %1, %1, 0\n\ts_sub_u32 %2, %2, %6\n\ts_cselect_b32 %2, 0, %2\n\t"
                     "s_add_u32 %3, %3, %7\n\ts_addc_u32 %4, %4, 0\n\ts_sub_u32 %5, %5, %7\n\ts_cselect_b32 %5, 0, %5"
                     : "+s"(aLo), "+s"(aHi), "+s"(aN), "+s"(bLo), "+s"(bHi), "+s"(bN)
                     : "s"(dkA), "s"(dkB)
                     : "scc");
        rA = mk(aLo, aHi, aN);
        rB = mk(bLo, bHi, bN);
    };
    auto advance = [&]() __attribute__((always_inline)) {
        if (++d_kt == d_KT) {
            d_kt = 0;
            d_term = 0;
            d_kk = 0;
            d_item += G;
            ++d_k;
            if (d_item < total) setup_dma(d_item);
            point();
        } else if (NP > 1) {                    // next term of the real K-tile, or the next real K-tile
            if (++d_term == a.T) {
                d_term = 0;
                ++d_kk;
            }
            point();
        } else if (a.reduce) {
            point();
        } else {
            step();
        }
    };

    f32x4 acc[8][8];
    bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
    // lane index as the fragment addresses see it: re-made opaque in every K-tile, so the M/N-contiguous
    // images' per-block addresses (lane-dependent XOR swizzle) are formed next to their reads instead of
    // being hoisted out of the K-loop into dozens of live VGPRs
    int flane = lane;
    auto rd = [&](int h, int r, int buf) __attribute__((always_inline)) {
        const unsigned char* base = lds + buf * STAGE;
        const bool isb = (r == 1) || r >= 9;
        const int idx = r == 0 ? 0 : r == 1 ? 0 : r <= 8 ? r - 1 : r - 8;
        if (!isb) {
            const bf16x8 v = frag<AK>(base, 8 * wm + idx, h, AK ? lane : flane);
            if (h == 0) fa0[idx] = v; else fa1[idx] = v;
        } else {
            const bf16x8 v = frag<BKC>(base + OPB, 8 * wn + idx, h, BKC ? lane : flane);
            if (h == 0) fb0[idx] = v; else fb1[idx] = v;
        }
    };
    auto mf = [&](int h, int q, bool first) __attribute__((always_inline)) {
        const int j = q >> 3, i = q & 7;
        if (first && h == 0) mfma_acc0(acc[i][j], fb0[j], fa0[i]);
        else mfma_acc(acc[i][j], h ? fb1[j] : fb0[j], h ? fa1[i] : fa0[i]);
    };

    // C through a buffer descriptor: out-of-range lanes store to an offset past its records (dropped)
    typedef typename std::conditional<OUTF32, float, __hip_bfloat16>::type TC;
    constexpr int ES = sizeof(TC);

    // prologue: stream positions 0 and 1 in flight, 0 landed, k-half 0 fragments of position 0 read
    setup_dma(d_item);
    point();
    constexpr int NG = EPI >= 4 ? 18 : EPI ? 17 : 16;    // DMA instructions per K-tile and wave
    constexpr int D2 = 16 - G9_P3;                        // operand DMAs in phase 2 (the rest in phase 3)
    constexpr int PH2 = 128 - G9_PH1 - G9_PH3;            // MFMAs between the two barriers
    constexpr int PH1 = G9_PH1, PH3 = G9_PH3;
    constexpr int SP = PH2 / D2;                          // MFMAs per phase-2 DMA
    static_assert(PH1 >= 16 && PH3 >= 16 && PH1 <= 64 && PH3 <= 64 && SP >= 1, "gemm9 phase split");
#pragma unroll
    for (int g = 0; g < NG; ++g) dma(g, 0);
    advance();
#pragma unroll
    for (int g = 0; g < NG; ++g) dma(g, 1);
    advance();
    if (EPI >= 4) VMCNT(18);
    else if (EPI) VMCNT(17);
    else VMCNT(16);
    __builtin_amdgcn_s_barrier();
    SB();
#pragma unroll
    for (int r = 0; r < 16; ++r) rd(0, r, 0);
    SB();

    int p = 0;                                  // stream position (buffer p & 1)
    int item_k = 0;                             // index of the item among this workgroup's items (bias slot)
    for (int item = blockIdx.x; item < total; item += G) {
        const bool stores_young = item != (int)blockIdx.x;
        // one K-tile (first: the item's first, whose k-half-0 MFMAs define the accumulators)
        auto ktile = [&](int t, auto first_c) __attribute__((always_inline)) {
            constexpr bool first = decltype(first_c)::value;
            const int cur = p & 1;
            if (!AK || !BKC) asm volatile("" : "+v"(flane));
            // phase 1: PH1 MFMAs of k-half 0 beside the 16 reads of k-half 1
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                mf(0, q, first);
                SB();
                rd(1, q, cur);
                SB();
            }
#pragma unroll
            for (int q = 16; q < PH1; ++q) mf(0, q, first);
            SB();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            SB();
            // phase 2: 64 - PH1 MFMAs of k-half 0 + 64 - PH3 of k-half 1 beside D2 of the 16 operand DMAs of position
            // p + 2 (every SP-th MFMA); the other P3 ride in phase 3 (G9_P3, default 0: all 16 here)
#pragma unroll
            for (int s = 0; s < PH2; ++s) {
                if (s < 64 - PH1) mf(0, PH1 + s, first);
                else mf(1, s - (64 - PH1), false);
                SB();
                if ((s % SP) == SP - 1 && s / SP < D2) {
                    dma(s / SP, cur);
                    SB();
                }
                if (NG > 16 && s == PH2 - 1) {   // the slot DMAs (EPI > 0) after the operands'
                    dma(16, cur);
                    if (NG > 17) dma(17, cur);
                    SB();
                }
            }
            if (G9_P3 == 0) {
                advance();
                SB();
            }
            // position p + 1 landed; younger than it: this iteration's DMA and, in an item's first K-tile, the
            // previous item's stores
            // (fp32 C: 64 stores + 16 DMA younger than the awaited ones exceed vmcnt's 63; waiting for 63 still
            // retires every older operation)
            // (with G9_P3 > 0 only D2 of this iteration's operand DMAs are younger than position p + 1's)
            if (EPI >= 4) {                     // 64 (h, g) / 48 (dh, row sums) stores: past 63 with the DMA
                if (t == 0 && stores_young) VMCNT(63);
                else vmcnt_const<D2 + 2>();
            } else if (EPI) {
                if (t == 0 && stores_young) {
                    if (OUTF32) VMCNT(63);
                    else vmcnt_const<D2 + 33>();
                } else {
                    vmcnt_const<D2 + 1>();
                }
            } else {
                if (t == 0 && stores_young) {
                    if (OUTF32) VMCNT(63);
                    else vmcnt_const<D2 + 32>();
                } else {
                    vmcnt_const<D2>();
                }
            }
            __builtin_amdgcn_s_barrier();
            SB();
            // phase 3: 21 MFMAs of k-half 1 beside the 16 reads of k-half 0 of position p + 1 (past the stream's
            // end: reads of a buffer that holds nothing, unused)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                mf(1, 64 - PH3 + q, false);
                SB();
                rd(0, q, cur ^ 1);
                SB();
                if (G9_P3 > 0 && (q % (16 / (G9_P3 > 0 ? G9_P3 : 1))) == 1 && q / (16 / (G9_P3 > 0 ? G9_P3 : 1)) < G9_P3) {
                    dma(D2 + q / (16 / (G9_P3 > 0 ? G9_P3 : 1)), cur);
                    SB();
                }
            }
#pragma unroll
            for (int q = 64 - PH3 + 16; q < 64; ++q) mf(1, q, false);
            SB();
            if (G9_P3 > 0) {
                advance();
                SB();
            }
            ++p;
        };
        ktile(0, std::true_type{});
        int iKT, iv0;
        {
            int z_, m0_, n0_;
            item_tile(item, nwg, total, tiles_m, tiles_n, z_, m0_, n0_);
            item_k_range(a, z_, KT, iv0, iKT);
        }
        for (int t = 1; t < iKT; ++t) ktile(t, std::false_type{});
        // epilogue of this item; acc[i][j][r] = C[mw + 16 i + (l & 15)][nw + 16 j + 4 (l >> 4) + r]
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");     // XDL write -> VALU read of the asm MFMAs
        // lane-derived epilogue values from an opaque lane index: formed here, not hoisted into registers that
        // stay live through the K-loop
        int elane = lane;
        asm volatile("" : "+v"(elane));
        const int l15 = elane & 15, row4 = elane >> 4;
        int z, m0, n0;
        item_tile(item, nwg, total, tiles_m, tiles_n, z, m0, n0);
        const int mw = m0 + 128 * wm, nw = n0 + 128 * wn;
        // the output batch's slice through its own descriptor (64-bit base): tile offsets stay 32-bit
        const __amdgpu_buffer_rsrc_t rC = rsrc(a.C, z * a.sC * ES, a.C ? a.spanC : 0);   // (null C: no records)
        const unsigned zc = 0u;
        const float* bsl = reinterpret_cast<const float*>(lds + 2 * STAGE + (item_k & 3) * 2048);
        auto act = [&](float x) __attribute__((always_inline)) {
            if (EPI == 2) x = gelu_tanh(x);
            else if (EPI == 3) x = x * gelu_parts(x).cdf;
            return x;
        };
        // the slot holds the item's 256 bias values (zeros without a bias): per column or per row, selected
        // by scalar factors (no per-element branches)
        const float fcol = a.bias_mode == 1 ? 1.f : 0.f, frow = a.bias_mode == 2 ? 1.f : 0.f;
        if (EPI >= 4) {
            gelu_epilogue9<EPI>(a, acc, bsl, rC, z, m0, n0, wm, wn, l15, row4, tiles_n);
            ++item_k;
            SB();
            continue;
        }
#pragma unroll
        for (int jp = 0; jp < 4; ++jp) {
            const int j0 = 2 * jp, j1 = j0 + 1;
            const int c0 = 128 * wn + 16 * j0 + 4 * row4;          // tile-local column of v0[0] (v1: + 16)
            f32x4 bc0 = {}, bc1 = {};
            if (EPI) {
                bc0 = *reinterpret_cast<const f32x4*>(bsl + c0) * fcol;
                bc1 = *reinterpret_cast<const f32x4*>(bsl + c0 + 16) * fcol;
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int m = mw + 16 * i + l15;
                const bool mok = m < a.M;
                f32x4 v0 = acc[i][j0], v1 = acc[i][j1];
                if (EPI) {
                    const float br = bsl[128 * wm + 16 * i + l15] * frow;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        v0[r] = act(fmaf(a.alpha, v0[r], bc0[r] + br));
                        v1[r] = act(fmaf(a.alpha, v1[r], bc1[r] + br));
                    }
                }
                if (OUTF32) {
                    const int n0c = nw + 16 * j0 + 4 * row4;
                    const unsigned o0 = (mok && n0c < a.N) ? (unsigned)(((long long)m * a.ldc + n0c) * ES) : 0x80000000u;
                    const unsigned o1 = (mok && n0c + 16 < a.N) ? (unsigned)(((long long)m * a.ldc + n0c + 16) * ES) : 0x80000000u;
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, v0), rC, o0, zc, 0);
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, v1), rC, o1, zc, 0);
                } else {
                    const uint32_t a0 = pack_bf16x2(v0[0], v0[1]), a1 = pack_bf16x2(v0[2], v0[3]);
                    const uint32_t b0 = pack_bf16x2(v1[0], v1[1]), b1 = pack_bf16x2(v1[2], v1[3]);
                    // rows (16-lane groups) 1 and 3 of (a0, a1) <-> rows 0 and 2 of (b0, b1): each lane then holds 8
                    // consecutive columns (a0 a1 b0 b1) of block j0 (rows 0, 2) or j1 (rows 1, 3)
                    const auto s0 = __builtin_amdgcn_permlane16_swap(a0, b0, false, false);
                    const auto s1 = __builtin_amdgcn_permlane16_swap(a1, b1, false, false);
                    const int n = nw + 16 * (j0 + (row4 & 1)) + 8 * (row4 >> 1);
                    const unsigned o = (mok && n < a.N) ? (unsigned)(((long long)m * a.ldc + n) * ES) : 0x80000000u;
                    const v4u32 d = {s0[0], s1[0], s0[1], s1[1]};
                    __builtin_amdgcn_raw_buffer_store_b128(d, rC, o, zc, 0);
                }
                SB();                           // one block pair at a time (no hoisting of all 256 AGPR reads)
            }
        }
        ++item_k;
        SB();
    }
    VMCNT(0);                                   // the null DMAs past the stream's end land before the LDS is freed
}

// C = alpha sum_s ws[s] (fixed order), fp32 or bf16 C (row stride ldc): the batch-reduced split-K's combine
template <bool OUTF32>
__global__ __launch_bounds__(256) void gemm9_reduce(const float* __restrict__ ws, void* C, int M, int N, long long ldc,
                                                    int S, float alpha) {
    const long long MN = (long long)M * N;
    for (long long i4 = ((long long)blockIdx.x * 256 + threadIdx.x) * 4; i4 < MN; i4 += (long long)gridDim.x * 1024) {
        f32x4 v = *reinterpret_cast<const f32x4*>(ws + i4);
        for (int k = 1; k < S; ++k) v += *reinterpret_cast<const f32x4*>(ws + k * MN + i4);
        v *= alpha;
        const int m = (int)(i4 / N), n = (int)(i4 - (long long)m * N);
        if (OUTF32) {
            *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(C) + m * ldc + n) = v;
        } else {
            const uint2 b = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
            *reinterpret_cast<uint2*>(reinterpret_cast<__hip_bfloat16*>(C) + m * ldc + n) = b;
        }
    }
}

// C[z] = alpha sum_s ws[z S + s] (fixed order) for each batch z: the batched K-split's combine (fp32 C, row
// stride ldc, batch stride sC)
__global__ __launch_bounds__(256) void gemm9_reduce_batched(const float* __restrict__ ws, float* C, int M, int N,
                                                            long long ldc, long long sC, int S, float alpha) {
    const long long MN = (long long)M * N;
    const int z = blockIdx.y;
    const float* w = ws + (long long)z * S * MN;
    for (long long i4 = ((long long)blockIdx.x * 256 + threadIdx.x) * 4; i4 < MN; i4 += (long long)gridDim.x * 1024) {
        f32x4 v = *reinterpret_cast<const f32x4*>(w + i4);
        for (int k = 1; k < S; ++k) v += *reinterpret_cast<const f32x4*>(w + k * MN + i4);
        v *= alpha;
        const int m = (int)(i4 / N), n = (int)(i4 - (long long)m * N);
        *reinterpret_cast<f32x4*>(C + z * sC + m * ldc + n) = v;
    }
}

int g_persistent = 1;            // vfm_gemm9_set_mode: 1 persistent (default), 0 one workgroup per tile


// fp32-equivalent (NP = 3) products: fp32 C, plain or bias epilogue, persistent form
template <bool AK, bool BKC>
void launch9_pieces(const G9Args& a, int batch, hipStream_t st) {
    static bool attr[MAXDEV] = {};
    const int dv_attr = cur_dev();
    if (!attr[dv_attr]) {
        (void)hipFuncSetAttribute((const void*)gemm9p_kernel<AK, BKC, true, 0, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS9P);
        (void)hipFuncSetAttribute((const void*)gemm9p_kernel<AK, BKC, true, 1, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS9P);
        attr[dv_attr] = true;
    }
    const int cus = device_cus(cur_dev());
    const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    const long long total = (long long)nwg * batch;
    const int grid = (int)std::min<long long>(total, cus);
    const bool plain = a.bias_mode == 0 && a.alpha == 1.f;
    if (plain)
        VFM_LAUNCH((gemm9p_kernel<AK, BKC, true, 0, 3>), dim3(grid), dim3(THREADS), LDS9P, st, a, (int)total);
    else
        VFM_LAUNCH((gemm9p_kernel<AK, BKC, true, 1, 3>), dim3(grid), dim3(THREADS), LDS9P, st, a, (int)total);
}

template <bool AK, bool BKC, bool OUTF32>
void launch9(const G9Args& a, int batch, hipStream_t st) {
    static bool attr[MAXDEV] = {};
    const int dv_attr = cur_dev();
    if (!attr[dv_attr]) {
        (void)hipFuncSetAttribute((const void*)gemm9_kernel<AK, BKC, OUTF32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  2 * STAGE);
        attr[dv_attr] = true;
    }
    const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    const bool plain = a.beta == 0.f && a.bias_mode == 0 && a.act == 0 && a.alpha == 1.f;
    if (g_persistent && a.beta == 0.f) {
        static bool attrp[MAXDEV] = {};
        const int dv_attrp = cur_dev();
        if (!attrp[dv_attrp]) {
            (void)hipFuncSetAttribute((const void*)gemm9p_kernel<AK, BKC, OUTF32, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS9P);
            (void)hipFuncSetAttribute((const void*)gemm9p_kernel<AK, BKC, OUTF32, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS9P);
            (void)hipFuncSetAttribute((const void*)gemm9p_kernel<AK, BKC, OUTF32, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS9P);
            (void)hipFuncSetAttribute((const void*)gemm9p_kernel<AK, BKC, OUTF32, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS9P);
            attrp[dv_attrp] = true;
        }
        const int cus = device_cus(cur_dev());
        const long long total = (long long)nwg * (a.reduce ? a.S : batch);
        const int grid = (int)std::min<long long>(total, cus);
        if (plain)
            VFM_LAUNCH((gemm9p_kernel<AK, BKC, OUTF32, 0>), dim3(grid), dim3(THREADS), LDS9P, st, a, (int)total);
        else if (a.act == 0)
            VFM_LAUNCH((gemm9p_kernel<AK, BKC, OUTF32, 1>), dim3(grid), dim3(THREADS), LDS9P, st, a, (int)total);
        else if (a.act == 1)
            VFM_LAUNCH((gemm9p_kernel<AK, BKC, OUTF32, 2>), dim3(grid), dim3(THREADS), LDS9P, st, a, (int)total);
        else
            VFM_LAUNCH((gemm9p_kernel<AK, BKC, OUTF32, 3>), dim3(grid), dim3(THREADS), LDS9P, st, a, (int)total);
        return;
    }
    VFM_LAUNCH((gemm9_kernel<AK, BKC, OUTF32>), dim3(nwg, batch), dim3(THREADS), 2 * STAGE, st, a);
}

long long span9(int kcont, long long outer, long long kdim, long long ld, long long sb, int batch) {
    const long long rows = kcont ? outer : kdim;
    const long long cols = kcont ? kdim : outer;
    const long long e = (rows - 1) * ld + cols + (long long)(batch - 1) * sb;
    return e * 2;
}

}  // namespace

// bf16 operands: C[z] (M x N, ldc, batch stride sC) = epi(alpha A[z] B[z] + beta C[z]) with A [M, K]
// (a_kcont: K-contiguous rows of stride lda, else M-contiguous rows of K) and B [K, N] (b_kcont: B is
// given as N rows of K, stride ldb; else K rows of N). bias_mode 0 none / 1 per column / 2 per row;
// act 0 none / 1 tanh-GELU / 2 erf-GELU; out_dtype VFM_BF16 or VFM_F32. Returns VFM_NO_KERNEL for shapes
// it does not take (K % 64, N % 8, unaligned operands, > 2 GiB spans).
static int gemm9_impl(const void* A, const void* B, void* C, const float* bias, int out_dtype, int M, int N, int K,
                      int batch, int a_kcont, long long lda, long long sA, int b_kcont, long long ldb, long long sB,
                      long long ldc, long long sC, float alpha, float beta, int bias_mode, int act, float* workspace,
                      int splits, int reduce_batch, void* stream) {
    if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0 || batch <= 0 || batch > 65535) return VFM_ERR_ARGS;
    if (out_dtype != VFM_BF16 && out_dtype != VFM_F32) return VFM_NO_KERNEL;
    if (bias_mode < 0 || bias_mode > 2 || (bias_mode && !bias) || act < 0 || act > 2) return VFM_ERR_ARGS;
    if (K % BK || N % 8) return VFM_NO_KERNEL;
    const int a_c = a_kcont ? K : M, b_c = b_kcont ? K : N;
    if (a_c % 8 || b_c % 8 || lda % 8 || ldb % 8 || sA % 8 || sB % 8 || ldc % 8 || sC % 8) return VFM_NO_KERNEL;
    if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) % 16) return VFM_NO_KERNEL;
    if (lda < (a_kcont ? (long long)K : M) || ldb < (b_kcont ? (long long)K : N) || ldc < N) return VFM_ERR_ARGS;
    const long long nwg = (long long)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    if (nwg > 0x7fffffffLL) return VFM_ERR_ARGS;
    // spans in bytes; the persistent form moves 64-bit descriptor bases and needs only one batch element's
    // tile offsets below 2^31, the one-workgroup-per-tile form the whole operand
    const long long spA = span9(a_kcont, M, K, lda, sA, batch), spB = span9(b_kcont, N, K, ldb, sB, batch);
    const long long spA1 = span9(a_kcont, M, K, lda, 0, 1), spB1 = span9(b_kcont, N, K, ldb, 0, 1);
    if (spA1 >= (1LL << 31) || spB1 >= (1LL << 31)) return VFM_NO_KERNEL;
    if (!g_persistent && (spA >= (1LL << 31) || spB >= (1LL << 31))) return VFM_NO_KERNEL;
    G9Args a{};
    a.T = 1;
    a.A = (const __hip_bfloat16*)A; a.B = (const __hip_bfloat16*)B; a.C = C; a.bias = bias;
    a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.sA = sA; a.sB = sB; a.sC = sC;
    a.M = M; a.N = N; a.K = K; a.alpha = alpha; a.beta = beta; a.bias_mode = bias_mode; a.act = act;
    a.spanA = spA; a.spanB = spB;
    hipStream_t st = (hipStream_t)stream;
    const bool of32 = out_dtype == VFM_F32;
    if (reduce_batch || splits > 1) {
        // batch-reduced (and / or K-split) product: fp32 partials of S chunks into the workspace, then the
        // fixed-order combine into C (plain epilogue, alpha only)
        if (!workspace || beta != 0.f || bias_mode || act || !g_persistent) return VFM_NO_KERNEL;
        if (!reduce_batch && batch != 1) return VFM_NO_KERNEL;
        const int KTz = K / BK, V = KTz * batch;
        const int S = std::max(1, std::min(splits, V));
        a.reduce = batch;
        a.KTz = KTz;
        a.kchunk = (V + S - 1) / S;
        a.S = (V + a.kchunk - 1) / a.kchunk;
        const long long MN = (long long)M * N;
        if (MN * 4 >= (1LL << 31) || MN % 4) return VFM_NO_KERNEL;
        G9Args p = a;
        p.C = workspace; p.ldc = N; p.sC = MN; p.alpha = 1.f;
        p.spanC = MN * a.S * 4;
        p.bias = nullptr; p.bias_mode = 0; p.act = 0;
#define VFM_G9R(AK, BK_) launch9<AK, BK_, true>(p, 1, st)
        if (a_kcont && b_kcont) VFM_G9R(true, true);
        else if (a_kcont && !b_kcont) VFM_G9R(true, false);
        else if (!a_kcont && b_kcont) VFM_G9R(false, true);
        else VFM_G9R(false, false);
#undef VFM_G9R
        const int blocks = (int)std::min<long long>((MN / 4 + 255) / 256, 4096);
        if (of32) VFM_LAUNCH(gemm9_reduce<true>, dim3(blocks), dim3(256), 0, st, workspace, C, M, N, ldc, a.S, alpha);
        else VFM_LAUNCH(gemm9_reduce<false>, dim3(blocks), dim3(256), 0, st, workspace, C, M, N, ldc, a.S, alpha);
        return launch_status();
    }
    {
        const int es = of32 ? 4 : 2;
        const long long spC1 = ((long long)(M - 1) * ldc + N) * es;
        const long long spC = spC1 + (long long)(batch - 1) * sC * es;
        if (spC1 >= (1LL << 31) || nwg * (long long)batch > 0x7fffffffLL) return VFM_NO_KERNEL;
        if (!g_persistent && spC >= (1LL << 31)) return VFM_NO_KERNEL;
        a.spanC = spC;
    }
#define VFM_G9(AK, BK_) of32 ? launch9<AK, BK_, true>(a, batch, st) : launch9<AK, BK_, false>(a, batch, st)
    if (a_kcont && b_kcont) VFM_G9(true, true);
    else if (a_kcont && !b_kcont) VFM_G9(true, false);
    else if (!a_kcont && b_kcont) VFM_G9(false, true);
    else VFM_G9(false, false);
#undef VFM_G9
    return launch_status();
}

// bf16 operands: C[z] (M x N, ldc, batch stride sC) = epi(alpha A[z] B[z] + beta C[z]) with A [M, K]
// (a_kcont: K-contiguous rows of stride lda, else M-contiguous rows of K) and B [K, N] (b_kcont: B is
// given as N rows of K, stride ldb; else K rows of N). bias_mode 0 none / 1 per column / 2 per row;
// act 0 none / 1 tanh-GELU / 2 erf-GELU; out_dtype VFM_BF16 or VFM_F32. Returns VFM_NO_KERNEL for shapes
// it does not take (K % 64, N % 8, unaligned operands, > 2 GiB spans).
extern "C" int vfm_gemm9(const void* A, const void* B, void* C, const float* bias, int out_dtype, int M, int N, int K,
                         int batch, int a_kcont, long long lda, long long sA, int b_kcont, long long ldb, long long sB,
                         long long ldc, long long sC, float alpha, float beta, int bias_mode, int act, void* stream) {
    return gemm9_impl(A, B, C, bias, out_dtype, M, N, K, batch, a_kcont, lda, sA, b_kcont, ldb, sB, ldc, sC, alpha,
                      beta, bias_mode, act, nullptr, 1, 0, stream);
}

// vfm_gemm9 with K splits and / or the batch reduction C = alpha sum_z A[z] B[z] (reduce_batch; C is [M, N]):
// S = min(splits, Z K/64) chunks of the batch-concatenated reduction, fp32 partials in `workspace`
// (vfm_gemm9_workspace_floats), combined in a fixed order. Plain products only (beta 0, no bias / act).
extern "C" int vfm_gemm9_ex(const void* A, const void* B, void* C, int out_dtype, int M, int N, int K, int batch,
                            int a_kcont, long long lda, long long sA, int b_kcont, long long ldb, long long sB,
                            long long ldc, float alpha, float* workspace, int splits, int reduce_batch, void* stream) {
    return gemm9_impl(A, B, C, nullptr, out_dtype, M, N, K, batch, a_kcont, lda, sA, b_kcont, ldb, sB, ldc, 0, alpha,
                      0.f, 0, 0, workspace, splits, reduce_batch, stream);
}

// fp32 workspace floats vfm_gemm9_ex needs (M N S); -1 when the shapes are not covered
extern "C" long long vfm_gemm9_workspace_floats(int M, int N, int K, int batch, int splits, int reduce_batch) {
    if (M <= 0 || N <= 0 || K <= 0 || batch <= 0 || K % BK) return -1;
    if (!reduce_batch && batch > 1) {                  // the batched K-split of vfm_gemm9_pieces: [batch][S][M][N]
        const int KTz = K / BK;
        const int S0 = std::max(1, std::min(splits, KTz));
        const int kc = (KTz + S0 - 1) / S0;
        return (long long)M * N * batch * ((KTz + kc - 1) / kc);
    }
    const int V = (K / BK) * (reduce_batch ? batch : 1);
    const int S0 = std::max(1, std::min(splits, V));
    const int kc = (V + S0 - 1) / S0;
    const int S = (V + kc - 1) / kc;
    return (long long)M * N * S;
}

// ConvNeXt-MLP 1x1 GEMMs with the GELU epilogues (gelu_epilogue9), bf16 operands and outputs, on the persistent
// kernel: C[z] = W[M, K] X[z][K, N] with W K-contiguous (lda), X N-contiguous (ldb, batch stride sB);
// mode 1: C = h (may be null), C2 = g = GELU(h s + b1); mode 2: C = dh from acc = dg and H = h,
// rsum0 (may be null) / rsum1 = [batch][vfm_gemm9_gelu_parts(N)][M] partial sums.
// rscale [batch][M] (null: 1), bias [M] (null: 0). C, C2, H share (ldc, sC).
extern "C" int vfm_gemm9_gelu(const void* W, const void* X, void* C, void* C2, const void* H, const float* rscale,
                              const float* bias, float* rsum0, float* rsum1, int mode, int M, int N, int K, int batch,
                              long long lda, long long ldb, long long sB, long long ldc, long long sC, void* stream) {
    if (!W || !X || M <= 0 || N <= 0 || K <= 0 || batch <= 0 || batch > 65535) return VFM_ERR_ARGS;
    if (mode == 1 ? !C2 : (mode == 2 ? (!C || !H || !rsum1) : true)) return VFM_ERR_ARGS;
    if (K % BK || K % 8 || N % 8 || M % 8 || lda % 8 || ldb % 8 || sB % 8 || ldc % 8 || sC % 8) return VFM_NO_KERNEL;
    if (((uintptr_t)W | (uintptr_t)X | (uintptr_t)C | (uintptr_t)C2 | (uintptr_t)H) % 16) return VFM_NO_KERNEL;
    if (lda < K || ldb < N || ldc < N) return VFM_ERR_ARGS;
    if (span9(1, M, K, lda, 0, 1) >= (1LL << 31) || span9(0, N, K, ldb, 0, 1) >= (1LL << 31) ||
        ((long long)(M - 1) * ldc + N) * 2 >= (1LL << 31))
        return VFM_NO_KERNEL;
    const long long nwg = (long long)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    if (nwg * batch > 0x7fffffffLL) return VFM_ERR_ARGS;
    G9Args a{};
    a.T = 1;
    a.A = (const __hip_bfloat16*)W; a.B = (const __hip_bfloat16*)X; a.C = C; a.C2 = C2;
    a.H = (const __hip_bfloat16*)H; a.rscale = rscale; a.bias = bias; a.rs0 = rsum0; a.rs1 = rsum1;
    a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.sA = 0; a.sB = sB; a.sC = sC;
    a.M = M; a.N = N; a.K = K; a.alpha = 1.f; a.beta = 0.f; a.bias_mode = 0; a.act = 0;
    a.spanA = span9(1, M, K, lda, 0, 1);
    a.spanB = span9(0, N, K, ldb, sB, batch);
    a.spanC = ((long long)(M - 1) * ldc + N + (long long)(batch - 1) * sC) * 2;
    hipStream_t st = (hipStream_t)stream;
    static bool attr[MAXDEV] = {};
    const int dv_attr = cur_dev();
    if (!attr[dv_attr]) {
        (void)hipFuncSetAttribute((const void*)gemm9p_kernel<true, false, false, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS9P);
        (void)hipFuncSetAttribute((const void*)gemm9p_kernel<true, false, false, 5>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS9P);
        attr[dv_attr] = true;
    }
    const int cus = device_cus(cur_dev());
    const long long total = nwg * batch;
    const int grid = (int)std::min<long long>(total, cus);
    if (mode == 1)
        VFM_LAUNCH((gemm9p_kernel<true, false, false, 4>), dim3(grid), dim3(THREADS), LDS9P, st, a, (int)total);
    else
        VFM_LAUNCH((gemm9p_kernel<true, false, false, 5>), dim3(grid), dim3(THREADS), LDS9P, st, a, (int)total);
    return launch_status();
}

// fp32 operands given as their three exact bf16 pieces (vfm_split_f32; csrc/gemm8.hip's f32x6 contract): C[z]
// (fp32, M x N) = alpha sum_t A_pa(t)[z] B_pb(t)[z] + bias over the six product terms of order >= 2^-16, on the
// persistent gemm9 kernel (the terms of a real K-tile as consecutive virtual K-tiles). psA / psB: elements
// between an operand's pieces (0: the stacked layouts, pieces along K). Plain or bias epilogues only (no split,
// beta 0, no activation); VFM_NO_KERNEL for what it does not take.
extern "C" int vfm_gemm9_pieces(const void* A, const void* B, float* C, const float* bias, int M, int N, int K,
                                int batch, int a_kcont, long long lda, long long sA, long long psA, int b_kcont,
                                long long ldb, long long sB, long long psB, long long ldc, long long sC, float alpha,
                                int bias_mode, float* workspace, int splits, int reduce_batch, void* stream) {
    if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0 || batch <= 0 || batch > 65535) return VFM_ERR_ARGS;
    if (bias_mode < 0 || bias_mode > 2 || (bias_mode && !bias) || psA < 0 || psB < 0) return VFM_ERR_ARGS;
    if (K % BK || N % 8) return VFM_NO_KERNEL;
    const int a_c = a_kcont ? K : M, b_c = b_kcont ? K : N;
    if (a_c % 8 || b_c % 8 || lda % 8 || ldb % 8 || sA % 8 || sB % 8 || ldc % 8 || sC % 8 || psA % 8 || psB % 8)
        return VFM_NO_KERNEL;
    if (((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) % 16) return VFM_NO_KERNEL;
    const int kra = (a_kcont && !psA) ? 3 * K : K, krb = (b_kcont && !psB) ? 3 * K : K;
    if (lda < (a_kcont ? (long long)kra : M) || ldb < (b_kcont ? (long long)krb : N) || ldc < N) return VFM_ERR_ARGS;
    const long long nwg = (long long)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    if (nwg * batch > 0x7fffffffLL || !g_persistent) return VFM_NO_KERNEL;
    G9Args a{};
    a.T = 6;
    for (int t = 0; t < 6; ++t) {
        a.pa |= Terms<3>::a(t) << (2 * t);
        a.pb |= Terms<3>::b(t) << (2 * t);
    }
    a.psA = psA ? psA : (a_kcont ? (long long)K : (long long)K * lda);
    a.psB = psB ? psB : (b_kcont ? (long long)K : (long long)K * ldb);
    // spans: one batch element's piece-0 extent plus the two further planes (the tile offsets of one batch
    // element below 2^31: the descriptor bases move per tile, as in vfm_gemm9)
    const long long spA1 = span9(a_kcont, M, K, lda, 0, 1) + 2 * a.psA * 2;
    const long long spB1 = span9(b_kcont, N, K, ldb, 0, 1) + 2 * a.psB * 2;
    if (spA1 >= (1LL << 31) || spB1 >= (1LL << 31)) return VFM_NO_KERNEL;
    a.spanA = span9(a_kcont, M, K, lda, sA, batch) + 2 * a.psA * 2;
    a.spanB = span9(b_kcont, N, K, ldb, sB, batch) + 2 * a.psB * 2;
    const long long spC1 = ((long long)(M - 1) * ldc + N) * 4;
    if (spC1 >= (1LL << 31)) return VFM_NO_KERNEL;
    a.spanC = spC1 + (long long)(batch - 1) * sC * 4;
    a.A = (const __hip_bfloat16*)A; a.B = (const __hip_bfloat16*)B; a.C = C; a.bias = bias;
    a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.sA = sA; a.sB = sB; a.sC = sC;
    a.M = M; a.N = N; a.K = K; a.alpha = alpha; a.beta = 0.f; a.bias_mode = bias_mode; a.act = 0;
    hipStream_t st = (hipStream_t)stream;
    auto go = [&](const G9Args& g, int items_batch) {
        if (a_kcont && b_kcont) launch9_pieces<true, true>(g, items_batch, st);
        else if (a_kcont) launch9_pieces<true, false>(g, items_batch, st);
        else if (b_kcont) launch9_pieces<false, true>(g, items_batch, st);
        else launch9_pieces<false, false>(g, items_batch, st);
    };
    if (reduce_batch || splits > 1) {
        // K-split and / or batch-reduced product (vfm_gemm9_ex's scheme): S chunks of whole real K-tiles of the
        // batch-concatenated reduction (each chunk its six terms per real K-tile) into fp32 partials, then the
        // fixed-order combine
        if (!workspace || bias_mode) return VFM_NO_KERNEL;
        if (!reduce_batch && batch != 1) {
            // batched K-split: bs chunks of each batch's real K-tiles, partials [batch][bs][M][N] in the workspace
            const int KTz = K / BK;
            const int S0 = std::max(1, std::min(splits, KTz));
            const int kcr = (KTz + S0 - 1) / S0;
            a.bs = (KTz + kcr - 1) / kcr;
            a.kchunk = kcr * a.T;
            const long long MN = (long long)M * N;
            if (MN * 4 >= (1LL << 31) || MN % 4 || (long long)batch * a.bs > 65535) return VFM_NO_KERNEL;
            G9Args p = a;
            p.C = workspace; p.ldc = N; p.sC = MN; p.alpha = 1.f;
            p.spanC = MN * (long long)batch * a.bs * 4;
            p.bias = nullptr; p.bias_mode = 0;
            go(p, batch * a.bs);
            const int blocks = (int)std::min<long long>((MN / 4 + 255) / 256, 1024);
            VFM_LAUNCH(gemm9_reduce_batched, dim3(blocks, batch), dim3(256), 0, st, workspace, C, M, N, ldc, sC, a.bs,
                       alpha);
            return launch_status();
        }
        const int KTz = K / BK, V = KTz * batch;
        const int S0 = std::max(1, std::min(splits, V));
        const int kcr = (V + S0 - 1) / S0;
        a.reduce = batch;
        a.KTz = KTz;
        a.kchunk = kcr * a.T;
        a.S = (V + kcr - 1) / kcr;
        const long long MN = (long long)M * N;
        if (MN * 4 >= (1LL << 31) || MN % 4) return VFM_NO_KERNEL;
        G9Args p = a;
        p.C = workspace; p.ldc = N; p.sC = MN; p.alpha = 1.f;
        p.spanC = MN * a.S * 4;
        p.bias = nullptr; p.bias_mode = 0;
        go(p, a.S);
        const int blocks = (int)std::min<long long>((MN / 4 + 255) / 256, 4096);
        VFM_LAUNCH(gemm9_reduce<true>, dim3(blocks), dim3(256), 0, st, workspace, C, M, N, ldc, a.S, alpha);
        return launch_status();
    }
    go(a, batch);
    return launch_status();
}

// Partial-sum slots per (batch, row) of vfm_gemm9_gelu mode 2 for N columns.
extern "C" int vfm_gemm9_gelu_parts(int N) { return N <= 0 ? -1 : 2 * ((N + BN - 1) / BN); }

// Kernel form of vfm_gemm9 (A/B switch for microbenchmarks): 1 = persistent (one workgroup per CU walking the
// output tiles, default), 0 = one workgroup per output tile. Returns the previous setting.
extern "C" int vfm_gemm9_set_mode(int persistent) {
    const int prev = g_persistent;
    g_persistent = persistent ? 1 : 0;
    return prev;
}
