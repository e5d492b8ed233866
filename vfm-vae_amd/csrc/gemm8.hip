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
//     wave-column's 64. A half-tile is 16 KB = 2 LDS-DMA (buffer_load_dwordx4 ... lds) per thread;
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
//     through LDS (8 KB per wave of the consumed buffer) with 16-B row stores;
//   * operands read through buffer descriptors: the 8 per-lane DMA offsets of a tile are computed
//     once, the K-tile advance is a scalar offset (no per-lane address arithmetic in the K-loop).
#include <cstdlib>

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
    // (pa >> 2t) & 3 of A and (pb >> 2t) & 3 of B (T = 1, pa = pb = 0 for bf16 operands). Piece p of
    // an operand starts p * psA (psB) elements after piece 0: Kp (K-contiguous [R][hi | mid | lo]),
    // Kp * ld (MN-contiguous [hi ; mid ; lo][R]) or the element count of a whole tensor (planar
    // pieces [NP][tensor], one split of an activation shared by its forward and backward products)
    int T, Kp, pa, pb;
    long long psA, psB;
    // microbenchmark stamps (null in production): per block, s_memrealtime (100 MHz) at entry, after the first
    // K-tile's wait, then per item: main loop done, epilogue stores issued, stores drained
    long long* stamps;
    // operand spans in bytes from A / B (buffer-descriptor ranges; < 2^31, checked on the host)
    unsigned spanA, spanB;
    // ConvNeXt-MLP GELU epilogues (EPI = 1 / 2, bf16 C; see gelu_epilogue): second output C2 (g),
    // aux input H (h, C's layout), per-(batch, row) scale [Z][M], bias per row, and per-row partial
    // sums [Z][4 tiles_n][M] of the backward
    void* C2;
    const __hip_bfloat16* H;
    const float* rscale;
    float* rs0;
    float* rs1;
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

// One LDS-DMA instruction through a buffer descriptor (buffer_load_dwordx4 ... offen lds: lane l's
// 16 B from rsrc + voff + soff land at M0 + 16 l). The per-lane byte offsets of a tile's 8 DMA slots
// are computed once per tile (dma_voff) and the K-tile advance is the scalar soff, so the K-loop
// issues its loads with no per-lane address arithmetic and no generic->LDS pointer conversion.
// Issued from inline asm so that hipcc's waitcnt pass does not see an LDS write in flight and drain
// it with vmcnt(0) before every ds_read; the counted waits below are the only ones. M0 is written in
// the same statement; the s_nops cover the readfirstlane -> soffset and M0 -> LDS-DMA hazards.
__device__ __forceinline__ void bdma16(__amdgpu_buffer_rsrc_t rsrc, unsigned voff, unsigned soff, unsigned m0) {
    asm volatile("s_nop 4\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(rsrc),
                 "s"(soff), "s"(m0)
                 : "memory");
}

// Per-lane byte offset (relative to the operand's K-tile origin) of DMA slot u of the half-tile
// (q, ISA) of a tile starting at outer0: K-contiguous images [128 rows][64 k] (chunk ^= (row>>1)&7),
// MN-contiguous ones [64 k][128] (gemm.hip's 4x4 chunk swizzle); rows beyond outer_n are clamped /
// redirected to a valid chunk whose result is unused.
template <bool KCONT, bool ISA>
__device__ __forceinline__ unsigned dma_voff(long long ld, int outer0, int outer_n, int q, int u, int tid) {
    const int ci = tid + 512 * u;
    if (KCONT) {
        const int row = ci >> 3, chs = (ci & 7) ^ ((row >> 1) & 7);
        const int o = min(outer0 + (ISA ? a_outer(row, q) : b_outer(row, q)), outer_n - 1);
        return (unsigned)(((long long)o * ld + 8 * chs) * 2);
    } else {
        const int row = ci >> 4, chs = (ci & 15) ^ mc_swz(row);
        int o = outer0 + (ISA ? a_outer(8 * chs, q) : b_outer(8 * chs, q));
        if (o >= outer_n) o = 0;                       // (outer_n % 8 == 0): a valid chunk, result unused
        return (unsigned)(((long long)row * ld + o) * 2);
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

__device__ __forceinline__ unsigned short bf16_bits(float v) {
    return __builtin_bit_cast(unsigned short, __float2bfloat16(v));
}
__device__ __forceinline__ float bf16_val(unsigned short b) { return __uint_as_float((uint32_t)b << 16); }

// Work item of the grid: one 256 x 256 output tile of one output batch and K split (y = batch * S +
// split): block (blockIdx.x, blockIdx.y).
struct Item {
    int m0, n0, tn, z, v0, KT, y;
};

// acc rows of quarter hf (rows 32 hf .. 32 hf + 31 of the wave block): a select on the wave-uniform
// quarter index, so the quarter loops of the epilogues stay rolled (one copy of their code: the
// unrolled forms were ~7k instructions per kernel and the epilogue ran out of instruction cache,
// ~13 us per tile).
__device__ __forceinline__ float acc_q(const f32x4 (&acc)[8][4], int hf, int ii, int j, int r) {
    const float v0 = acc[ii][j][r], v1 = acc[2 + ii][j][r], v2 = acc[4 + ii][j][r], v3 = acc[6 + ii][j][r];
    return hf == 0 ? v0 : hf == 1 ? v1 : hf == 2 ? v2 : v3;
}

// Stage quarter hf of the wave's 128 x 64 fp32 block into its 8 KB of LDS: 16-B chunk c (4 columns)
// of row ml at chunk c ^ (ml & 15) (conflict-free writes in the accumulator layout and row reads).
__device__ __forceinline__ void stage_quarter(float* wl, const f32x4 (&acc)[8][4], int hf, int lane) {
    const int cl = lane & 15, rq = 4 * (lane >> 4);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ml = 16 * ii + rq + r, nl = 16 * j + cl;
                wl[ml * 64 + (((nl >> 2) ^ (ml & 15)) << 2) + (nl & 3)] = acc_q(acc, hf, ii, j, r);
            }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// GELU epilogues of the ConvNeXt MLP's 1x1 GEMMs (reference networks/utils/convnext_utils.py:
// 135-142: pwconv1 -> GELU -> pwconv2, with the modulation scale s[b, o] and bias b1[o] of the
// channel o = GEMM row; the same roundings as the separate scale_bias_gelu kernels, csrc/decoder.hip
// gelu_fwd / gelu_bwd):
//   EPI 1 (forward):  h = bf16(acc) -> C (if non-null); g = bf16(GELU(h s + b1)) -> C2;
//   EPI 2 (backward): dg = bf16(acc); dz = dg GELU'(h s + b1) with h from H; dh = bf16(dz s) -> C;
//                     per-row sums of dz h and dz over this wave's 64 columns -> rs0 / rs1 at
//                     [z][4 tn + wn][m] (the host sums the 4 tiles_n partials: fixed order).
// The wave's 128 x 64 fp32 block goes through its 8 KB of LDS in four 32-row quarters; each lane then
// walks 8-column row chunks in a rolled loop (16-B global loads / stores of h, g, dh; the row scale
// and bias loaded once per chunk), which keeps the epilogue's registers out of the accumulator's way
// (the element-wise form of this epilogue spilled ~300 VGPRs).
template <int EPI>
__device__ __forceinline__ void gelu_epilogue(const G8Args& a, f32x4 (&acc)[8][4], float* wl, int lane, int wm,
                                              int wn, int m0, int n0, int z, int tn) {
    const int mw = m0 + 128 * wm, nw = n0 + 64 * wn;           // this wave's 128 x 64 block
    const long long zo = (long long)z * a.sC;
    __hip_bfloat16* Cb = reinterpret_cast<__hip_bfloat16*>(a.C);
    __hip_bfloat16* C2b = reinterpret_cast<__hip_bfloat16*>(a.C2);
    const float* sc_row = a.rscale ? a.rscale + (long long)z * a.M : nullptr;
    const bool vec = (a.ldc % 8) == 0 && (a.sC % 8) == 0 &&
                     ((reinterpret_cast<uintptr_t>(a.C) | reinterpret_cast<uintptr_t>(a.C2) |
                       reinterpret_cast<uintptr_t>(a.H)) % 16) == 0;
    const long long pbase = ((long long)z * (4LL * ((a.N + BN - 1) / BN)) + 4 * tn + wn) * a.M;
#pragma unroll 1
    for (int hf = 0; hf < 4; ++hf) {
        stage_quarter(wl, acc, hf, lane);
        // item c: row ml = c >> 3 of the quarter, columns 8 (c & 7) .. + 7; 8 lanes share a row
#pragma unroll 1
        for (int c = lane; c < 32 * 8; c += 64) {
            const int ml = c >> 3, q = c & 7;
            const int m = mw + 32 * hf + ml, n = nw + 8 * q;
            const float4 v0 = *reinterpret_cast<const float4*>(wl + ml * 64 + (((2 * q) ^ (ml & 15)) << 2));
            const float4 v1 = *reinterpret_cast<const float4*>(wl + ml * 64 + (((2 * q + 1) ^ (ml & 15)) << 2));
            float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
            const bool mok = m < a.M;
            const int mr = mok ? m : a.M - 1;
            const float sc = sc_row ? sc_row[mr] : 1.f;
            const float bi = a.bias ? a.bias[mr] : 0.f;
            const long long off = zo + (long long)mr * a.ldc + n;
            const bool full = mok && vec && n + 8 <= a.N;
            float s0 = 0.f, s1 = 0.f;
            if (EPI == 1) {
                unsigned short hb[8], gb[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    hb[k] = bf16_bits(v[k]);
                    const float zz = fmaf(bf16_val(hb[k]), sc, bi);
                    gb[k] = bf16_bits(zz * gelu_parts(zz).cdf);
                }
                if (full) {
                    if (Cb) *reinterpret_cast<uint4*>(Cb + off) = *reinterpret_cast<const uint4*>(hb);
                    *reinterpret_cast<uint4*>(C2b + off) = *reinterpret_cast<const uint4*>(gb);
                } else if (mok) {
                    for (int k = 0; k < 8 && n + k < a.N; ++k) {
                        if (Cb) Cb[off + k] = __builtin_bit_cast(__hip_bfloat16, hb[k]);
                        C2b[off + k] = __builtin_bit_cast(__hip_bfloat16, gb[k]);
                    }
                }
            } else {
                unsigned short hb[8], db[8];
                if (full) {
                    *reinterpret_cast<uint4*>(hb) = *reinterpret_cast<const uint4*>(a.H + off);
                } else {
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        hb[k] = (mok && n + k < a.N) ? __builtin_bit_cast(unsigned short, a.H[off + k]) : 0;
                }
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const float hv = bf16_val(hb[k]);
                    const GeluParts gp = gelu_parts(fmaf(hv, sc, bi));
                    float dz = bf16_val(bf16_bits(v[k])) * (gp.cdf + gp.zpdf);
                    if (!full && (!mok || n + k >= a.N)) dz = 0.f;
                    s0 = fmaf(dz, hv, s0);
                    s1 += dz;
                    db[k] = bf16_bits(dz * sc);
                }
                if (full) {
                    *reinterpret_cast<uint4*>(Cb + off) = *reinterpret_cast<const uint4*>(db);
                } else if (mok) {
                    for (int k = 0; k < 8 && n + k < a.N; ++k) Cb[off + k] = __builtin_bit_cast(__hip_bfloat16, db[k]);
                }
                // the 8 lanes of this row: xor 1, 2, 4 (fixed order, identical on every lane)
                s0 += __shfl_xor(s0, 1);
                s1 += __shfl_xor(s1, 1);
                s0 += __shfl_xor(s0, 2);
                s1 += __shfl_xor(s1, 2);
                s0 += __shfl_xor(s0, 4);
                s1 += __shfl_xor(s1, 4);
                if (q == 0 && mok) {
                    if (a.rs0) a.rs0[pbase + m] = s0;
                    a.rs1[pbase + m] = s1;
                }
            }
        }
    }
}

// Epilogue of one item (everything but the GELU forms): acc -> C = act(alpha acc + beta C + bias), or
// the raw split-K partial. The wave's 128 x 64 fp32 block goes through its 8 KB of the consumed LDS
// buffer in four 32-row quarters; each lane then walks 8-column row chunks (16-B / 32-B stores where
// the chunk is whole and aligned, guarded element stores at the edges). Both loops are rolled.
template <bool OUTF32>
__device__ __forceinline__ void store_tile(const G8Args& a, f32x4 (&acc)[8][4], float* wl, int lane, int wm, int wn,
                                           const Item& it) {
    typedef typename std::conditional<OUTF32, float, __hip_bfloat16>::type TC;
    const int mw = it.m0 + 128 * wm, nw = it.n0 + 64 * wn;
    const bool part = a.ws != nullptr;
    float* wsb = part ? a.ws + (long long)it.y * a.M * a.N : nullptr;
    TC* Cb = reinterpret_cast<TC*>(a.C) + (long long)it.z * a.sC;
    const bool cvec = OUTF32 ? ((a.ldc % 4) == 0 && (a.sC % 4) == 0 && (reinterpret_cast<uintptr_t>(a.C) % 16) == 0)
                             : ((a.ldc % 8) == 0 && (a.sC % 8) == 0 && (reinterpret_cast<uintptr_t>(a.C) % 16) == 0);
    const bool wvec = (a.N % 4) == 0;
    const bool plain = a.beta == 0.f && a.bias_mode == 0 && a.act == 0 && a.alpha == 1.f;
#pragma unroll 1
    for (int hf = 0; hf < 4; ++hf) {
        stage_quarter(wl, acc, hf, lane);
#pragma unroll 1
        for (int c = lane; c < 32 * 8; c += 64) {
            const int ml = c >> 3, q = c & 7;
            const int m = mw + 32 * hf + ml, n = nw + 8 * q;
            if (m >= a.M || n >= a.N) continue;
            const float4 v0 = *reinterpret_cast<const float4*>(wl + ml * 64 + (((2 * q) ^ (ml & 15)) << 2));
            const float4 v1 = *reinterpret_cast<const float4*>(wl + ml * 64 + (((2 * q + 1) ^ (ml & 15)) << 2));
            float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
            const bool whole = n + 8 <= a.N;
            if (part) {
                float* d = wsb + (long long)m * a.N + n;
                if (whole && wvec) {
                    *reinterpret_cast<float4*>(d) = v0;
                    *reinterpret_cast<float4*>(d + 4) = v1;
                } else {
                    for (int k = 0; k < 8 && n + k < a.N; ++k) d[k] = v[k];
                }
                continue;
            }
            TC* d = Cb + (long long)m * a.ldc + n;
            if (!plain) {
                const float brow = (a.bias_mode == 2) ? a.bias[m] : 0.f;
#pragma unroll 1
                for (int k = 0; k < 8; ++k) {
                    const bool in = whole || n + k < a.N;
                    float x = a.alpha * v[k];
                    if (a.beta != 0.f && in) x = fmaf(a.beta, ld(d + k), x);
                    x += (a.bias_mode == 1) ? (in ? a.bias[n + k] : 0.f) : brow;
                    if (a.act == 1) x = gelu_tanh(x);
                    else if (a.act == 2) x = x * gelu_parts(x).cdf;
                    v[k] = x;
                }
            }
            if (whole && cvec) {
                if (OUTF32) {
                    float* df = reinterpret_cast<float*>(d);
                    *reinterpret_cast<float4*>(df) = make_float4(v[0], v[1], v[2], v[3]);
                    *reinterpret_cast<float4*>(df + 4) = make_float4(v[4], v[5], v[6], v[7]);
                } else {
                    unsigned short b[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) b[k] = bf16_bits(v[k]);
                    *reinterpret_cast<uint4*>(d) = *reinterpret_cast<const uint4*>(b);
                }
            } else {
                for (int k = 0; k < 8 && n + k < a.N; ++k) st(d + k, v[k]);
            }
        }
    }
}

template <bool AK, bool BKC, bool OUTF32, bool DEEP, int EPI = 0>
__global__ __launch_bounds__(THREADS, 1) void gemm8_kernel(G8Args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 2, wn = wave & 3;
    const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.N + BN - 1) / BN;
    const int nwg = tiles_m * tiles_n;
    const int KTz = a.Kp / BK;                         // K-tiles per batch and piece
    const int VT = a.reduce ? a.Z * KTz : KTz;         // virtual K-tiles of one product term
    const int V = a.T * VT;                            // virtual K-tiles of one output

    Item it;
    {
        const int y = blockIdx.y, bid = blockIdx.x;
        // XCD-aware bijective remap, then grouped order: consecutive tiles (the ~32 an XCD runs at
        // once) cover GROUP tile-rows x 32/GROUP tile-columns, so the XCD's L2 holds GROUP A panels +
        // 32/GROUP B panels instead of 1 + 32
        const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
        const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
        constexpr int GROUP = 4;
        const int gsz = GROUP * tiles_n, grp = tile / gsz, rem = tile - grp * gsz;
        const int rows_g = min(GROUP, tiles_m - grp * GROUP);
        const int tm = grp * GROUP + rem % rows_g;
        it.tn = rem / rows_g;
        it.m0 = tm * BM;
        it.n0 = it.tn * BN;
        it.z = a.reduce ? 0 : y / a.S;
        it.v0 = (y - it.z * a.S) * a.kchunk;
        it.KT = min(V, it.v0 + a.kchunk) - it.v0;      // >= 1 by construction of S on the host
        it.y = y;
    }
    const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)a.A, 0, (int)a.spanA, 0x00020000);
    const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)a.B, 0, (int)a.spanB, 0x00020000);
    // per-lane byte offsets of the 8 DMA slots (half-tile h = 0 A_lo, 1 B_lo, 2 B_hi, 3 A_hi; slot u)
    unsigned vo[8];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        vo[0 + u] = dma_voff<AK, true>(a.lda, it.m0, a.M, 0, u, tid);
        vo[2 + u] = dma_voff<BKC, false>(a.ldb, it.n0, a.N, 0, u, tid);
        vo[4 + u] = dma_voff<BKC, false>(a.ldb, it.n0, a.N, 1, u, tid);
        vo[6 + u] = dma_voff<AK, true>(a.lda, it.m0, a.M, 1, u, tid);
    }
    const unsigned lds0 =
        __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_void*)lds + (unsigned)wave * 64 * 16);
    // virtual K-tile iterator, term-fastest (v = T * real K-tile + term): the T piece products of one real
    // K-tile run back to back, so the piece tiles a term re-reads (hi of A for three terms, ...) are still
    // in L2 from the term before -- one HBM read of each piece instead of one per term. Then batch zt
    // (batch-reduced products) and K-tile kk of the batch.
    int term, zt, kk;
    {
        const int v = it.v0;
        const int rest = v / a.T;
        term = v - rest * a.T;
        zt = a.reduce ? rest / KTz : it.z;
        kk = a.reduce ? rest - (rest / KTz) * KTz : rest;
    }
    // scalar byte offsets of the current K-tile inside A / B
    auto soffs = [&](unsigned& sa, unsigned& sb) {
        const long long ka = (long long)kk * BK, kb = ka;
        const long long pofa = ((a.pa >> (2 * term)) & 3) * a.psA, pofb = ((a.pb >> (2 * term)) & 3) * a.psB;
        sa = __builtin_amdgcn_readfirstlane((unsigned)((zt * a.sA + (AK ? ka : ka * a.lda) + pofa) * 2));
        sb = __builtin_amdgcn_readfirstlane((unsigned)((zt * a.sB + (BKC ? kb : kb * a.ldb) + pofb) * 2));
    };
    auto advance = [&]() {                               // branch-free: selects on wave-uniform values
        const bool w0 = ++term == a.T;
        term = w0 ? 0 : term;
        const bool w1 = w0 && ++kk == KTz;
        kk = w1 ? 0 : kk;
        zt += (a.reduce && w1) ? 1 : 0;
    };
    auto issue = [&](unsigned sa, unsigned sb, int bsel, int h) {
        const unsigned m0 = lds0 + bsel * BUF + (h == 0 ? OFF_ALO : h == 1 ? OFF_BLO : h == 2 ? OFF_BHI : OFF_AHI);
        const bool isa = (h == 0 || h == 3);
#pragma unroll
        for (int u = 0; u < 2; ++u) bdma16(isa ? rA : rB, vo[2 * h + u], isa ? sa : sb, m0 + u * 512 * 16);
    };
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};
    bf16x8 af[4][2], bl[2][2], bh[2][2];        // A quadrant rows; B_lo / B_hi columns (both kept)
    // phase p multiplies quadrant (qm, qn) with the fragments read in this or an earlier phase
    // (A_lo + B_lo at p0, B_hi at p1, A_hi at p2)
    auto phase_math = [&](int p) {
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

    const long long t_entry = a.stamps ? (long long)__builtin_amdgcn_s_memrealtime() : 0;
    const int KT = it.KT;
    unsigned sa1 = 0, sb1 = 0;                  // offsets of K-tile t + 1
    {
        unsigned sa, sb;
        soffs(sa, sb);
        issue(sa, sb, 0, 0);
        issue(sa, sb, 0, 1);
        issue(sa, sb, 0, 2);
        issue(sa, sb, 0, 3);
        if (DEEP && KT > 1) {
            advance();
            soffs(sa1, sb1);
            issue(sa1, sb1, 1, 0);
            issue(sa1, sb1, 1, 1);
        }
    }
    if (DEEP && KT > 1) VMCNT(8);               // A_lo(0), B_lo(0) landed; B_hi(0), A_hi(0), A_lo(1), B_lo(1) in flight
    else VMCNT(4);                              // A_lo, B_lo of the first K-tile
    __builtin_amdgcn_s_barrier();
    long long* stamp = (a.stamps && tid == 0) ? a.stamps + (long long)(blockIdx.y * gridDim.x + blockIdx.x) * 16 : nullptr;
    if (stamp) {
        stamp[0] = t_entry;
        stamp[1] = (long long)__builtin_amdgcn_s_memrealtime();
    }
    // ping-pong: the wm = 1 wave-row runs one barrier behind (2 barriers per phase), so one
    // wave-row's 16 MFMAs overlap the other's DMA issue + fragment reads (see the header)
    if (wm == 1) __builtin_amdgcn_s_barrier();
    if (DEEP) {
        // Two K-tiles ahead: the fragments of a half-tile live in VGPRs after their phase, so its LDS
        // slot is restaged for K-tile t+2 two or more phases later (WAR with the rows one barrier
        // apart). Phase p of K-tile t issues p0: B_hi(t+1), p1: A_hi(t+1) (buffer (t+1)&1), p2:
        // A_lo(t+2), p3: B_lo(t+2) (buffer t&1); the counted waits leave 4 half-tiles (8 DMA) in
        // flight, so each half-tile is issued 5-6 phases before its read (2-4 in the other schedule).
        for (int t = 0; t < KT; ++t) {
            const unsigned char* buf = lds + (t & 1) * BUF;
            const bool n1 = t + 1 < KT, n2 = t + 2 < KT;
            unsigned sa2 = 0, sb2 = 0;
            if (n2) {
                advance();
                soffs(sa2, sb2);
            }
            // p0: issue B_hi(t+1); read A_lo(t), B_lo(t); wait for B_hi(t)
            if (n1) issue(sa1, sb1, (t + 1) & 1, 2);
            phase_reads(buf, 0);
            if (n1) VMCNT(8);
            else VMCNT(2);
            phase_math(0);
            // p1: issue A_hi(t+1); read B_hi(t); wait for A_hi(t)
            if (n1) issue(sa1, sb1, (t + 1) & 1, 3);
            phase_reads(buf, 1);
            if (n1) VMCNT(8);
            else VMCNT(0);
            phase_math(1);
            // p2: issue A_lo(t+2); read A_hi(t)
            if (n2) issue(sa2, sb2, t & 1, 0);
            phase_reads(buf, 2);
            phase_math(2);
            // p3: issue B_lo(t+2); wait for A_lo(t+1), B_lo(t+1)
            if (n2) issue(sa2, sb2, t & 1, 1);
            if (n1) {
                if (n2) VMCNT(8);
                else VMCNT(4);
            }
            phase_math(3);
            sa1 = sa2;
            sb1 = sb2;
        }
    } else {
        for (int t = 0; t < KT; ++t) {
            const unsigned char* buf = lds + (t & 1) * BUF;
            const bool nxt = t + 1 < KT;
            unsigned sa = 0, sb = 0;
            if (nxt) {
                advance();
                soffs(sa, sb);
            }
            const int nb = (t + 1) & 1;
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                if (nxt) issue(sa, sb, nb, p);
                phase_reads(buf, p);
                // wait for the NEXT phase's half-tile (see the header), then the phase barrier
                if (nxt) {
                    if (p == 0 || p == 1 || p == 3) VMCNT(4);
                } else {
                    if (p == 0) VMCNT(2);
                    else if (p == 1) VMCNT(0);
                }
                phase_math(p);
            }
        }
    }
    if (wm == 0) __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (stamp) stamp[2] = (long long)__builtin_amdgcn_s_memrealtime();
    // epilogue through this wave's 8 KB of the buffer the last K-tile was read from;
    // acc[i][j][r] = C[m0 + 128wm + 16i + 4(l>>4) + r][n0 + 64wn + 16j + (l&15)]
    unsigned char* wl = lds + ((it.KT - 1) & 1) * BUF + wave * (BUF / 8);
    if (EPI) gelu_epilogue<EPI>(a, acc, reinterpret_cast<float*>(wl), lane, wm, wn, it.m0, it.n0, it.z, it.tn);
    else store_tile<OUTF32>(a, acc, reinterpret_cast<float*>(wl), lane, wm, wn, it);
    if (stamp) {
        stamp[3] = (long long)__builtin_amdgcn_s_memrealtime();     // stores issued
        VMCNT(0);
        stamp[4] = (long long)__builtin_amdgcn_s_memrealtime();     // stores drained
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

long long* g_stamps = nullptr;   // microbenchmark stamp buffer (vfm_gemm8_set_stamps)
int g_deep = 0;                  // K-tile staging: 1 = two K-tiles ahead, 0 = one (vfm_gemm8_set_schedule)

template <bool AK, bool BKC, bool OUTF32, bool DEEP, int EPI>
void launch8d(const G8Args& a, int nwg, int ny, hipStream_t st) {
    static bool attr[MAXDEV] = {};
    const int dv_attr = cur_dev();
    if (!attr[dv_attr]) {
        (void)hipFuncSetAttribute((const void*)gemm8_kernel<AK, BKC, OUTF32, DEEP, EPI>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BUF);
        attr[dv_attr] = true;
    }
    VFM_LAUNCH((gemm8_kernel<AK, BKC, OUTF32, DEEP, EPI>), dim3(nwg, ny), dim3(THREADS), 2 * BUF, st, a);
}

template <bool AK, bool BKC, bool OUTF32, int EPI = 0>
void launch8k(const G8Args& a, int nwg, int ny, hipStream_t st) {
    if (g_deep) launch8d<AK, BKC, OUTF32, true, EPI>(a, nwg, ny, st);
    else launch8d<AK, BKC, OUTF32, false, EPI>(a, nwg, ny, st);
}

template <bool AK, bool BKC, bool OUTF32>
int launch8(const G8Args& a, int batch, hipStream_t st) {
    const int nwg = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
    const int zo = a.reduce ? 1 : batch;
    launch8k<AK, BKC, OUTF32>(a, nwg, zo * a.S, st);
    if (a.ws) {
        const long long MN = (long long)a.M * a.N;
        VFM_LAUNCH(gemm8_reduce<OUTF32>, dim3((unsigned)((MN + 255) / 256), zo), dim3(256), 0, st, a);
    }
    return launch_status();
}

// Bytes an operand spans from its base: rows x ld (+ batch stride), as the buffer descriptor range;
// -1 when it does not fit the 32-bit offsets of the DMA (2 GiB).
static long long span_bytes(int kcont, long long outer, long long kdim, long long ld, long long sb, int batch) {
    const long long rows = kcont ? outer : kdim;
    const long long cols = kcont ? kdim : outer;
    const long long e = (rows - 1) * ld + cols + (long long)(batch - 1) * sb;
    const long long bytes = e * 2;
    return bytes >= (1LL << 31) ? -1 : bytes;
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

// The planar form (R = 1, kcont: dst = [NP][n] pieces of a contiguous n-element tensor, n % 8 == 0):
// 8 elements per thread, two 16-B loads and one 16-B store per piece, no index division.
template <int NP>
__global__ __launch_bounds__(256) void split_planar_kernel(const float* __restrict__ src,
                                                           __hip_bfloat16* __restrict__ dst, long long n) {
    for (long long i8 = ((long long)blockIdx.x * 256 + threadIdx.x) * 8; i8 < n; i8 += (long long)gridDim.x * 256 * 8) {
        const float4 a = *reinterpret_cast<const float4*>(src + i8);
        const float4 b = *reinterpret_cast<const float4*>(src + i8 + 4);
        uint32_t q[4][NP];
        split_pieces<NP>(a.x, a.y, q[0]);
        split_pieces<NP>(a.z, a.w, q[1]);
        split_pieces<NP>(b.x, b.y, q[2]);
        split_pieces<NP>(b.z, b.w, q[3]);
#pragma unroll
        for (int p = 0; p < NP; ++p)
            *reinterpret_cast<uint4*>(dst + (long long)p * n + i8) = make_uint4(q[0][p], q[1][p], q[2][p], q[3][p]);
    }
}

}  // namespace

extern "C" int vfm_split_f32(const float* src, void* dst, int R, int K, long long ld, long long sb, long long db,
                             int batch, int precision, int kcont, void* stream) {
    if (!src || !dst || R <= 0 || K <= 0 || batch <= 0 || batch > 65535) return VFM_ERR_ARGS;
    if (precision != VFM_F32 && precision != VFM_F32X3) return VFM_ERR_ARGS;
    const int inner = kcont ? K : R;
    if (inner % 4 || ld % 4 || sb % 4 || ((uintptr_t)src % 16) || ((uintptr_t)dst % 8)) return VFM_NO_KERNEL;
    static const bool planar8 = [] {                       // VFM_SPLIT_PLANAR8=0: the generic split kernel
        const char* e = getenv("VFM_SPLIT_PLANAR8");
        return !(e && e[0] == '0');
    }();
    if (planar8 && R == 1 && kcont && batch == 1 && K % 8 == 0 && (uintptr_t)dst % 16 == 0) {
        // planar pieces of one contiguous tensor (gemm_hip._planar)
        const long long blocks = std::min<long long>(((long long)K / 8 + 255) / 256, 4096);
        if (precision == VFM_F32)
            VFM_LAUNCH(split_planar_kernel<3>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, src,
                       (__hip_bfloat16*)dst, (long long)K);
        else
            VFM_LAUNCH(split_planar_kernel<2>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, src,
                       (__hip_bfloat16*)dst, (long long)K);
        return launch_status();
    }
    const long long total4 = ((long long)R * K) / 4;
    dim3 grid((unsigned)((total4 + 255) / 256), batch);
    if (precision == VFM_F32)
        VFM_LAUNCH(split_f32_kernel<3>, grid, dim3(256), 0, (hipStream_t)stream, src, (__hip_bfloat16*)dst, R, K,
                           ld, sb, db, kcont);
    else
        VFM_LAUNCH(split_f32_kernel<2>, grid, dim3(256), 0, (hipStream_t)stream, src, (__hip_bfloat16*)dst, R, K,
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

// Bytes an operand with np pieces spans: the stacked layouts (ps = 0: pieces along K) or planar
// pieces ps elements apart; -1 when the buffer descriptor cannot cover it (>= 2^31 bytes).
static long long piece_span(int kcont, long long outer, int K, int np, long long ld, long long sb, int batch,
                            long long ps) {
    if (ps == 0) return span_bytes(kcont, outer, (long long)np * K, ld, sb, batch);
    const long long one = span_bytes(kcont, outer, K, ld, sb, batch);
    if (one < 0) return -1;
    const long long bytes = one + (long long)(np - 1) * ps * 2;
    return bytes >= (1LL << 31) ? -1 : bytes;
}

static int gemm8_impl(const void* A, const void* B, void* C, const float* bias, int precision, int out_dtype, int M,
                      int N, int K, int batch, int a_kcont, long long lda, long long sA, long long psA, int b_kcont,
                      long long ldb, long long sB, long long psB, long long ldc, long long sC, float alpha, float beta,
                      int bias_mode, int act, float* workspace, int kchunk, int reduce_batch, void* stream) {
    if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0 || batch <= 0 || batch > 65535) return VFM_ERR_ARGS;
    if (out_dtype != VFM_BF16 && out_dtype != VFM_F32) return VFM_NO_KERNEL;
    const int np = pieces_of(precision);
    if (!np) return VFM_ERR_ARGS;
    if (bias_mode < 0 || bias_mode > 2 || (bias_mode && !bias) || act < 0 || act > 2) return VFM_ERR_ARGS;
    if (psA < 0 || psB < 0) return VFM_ERR_ARGS;
    if (K % BK) return VFM_NO_KERNEL;
    const int a_c = a_kcont ? K : M, b_c = b_kcont ? K : N;
    if (a_c % 8 || b_c % 8 || lda % 8 || ldb % 8 || sA % 8 || sB % 8 || psA % 8 || psB % 8) return VFM_NO_KERNEL;
    if (((uintptr_t)A | (uintptr_t)B) % 16) return VFM_NO_KERNEL;
    // stacked pieces (ps = 0) lie along K inside a K-contiguous row: the row holds np K
    const int kra = (a_kcont && !psA) ? np * K : K, krb = (b_kcont && !psB) ? np * K : K;
    if (lda < (a_kcont ? (long long)kra : M) || ldb < (b_kcont ? (long long)krb : N) || ldc < N) return VFM_ERR_ARGS;
    const long long nwg = (long long)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    if (nwg > 0x7fffffffLL) return VFM_ERR_ARGS;
    const long long spA = piece_span(a_kcont, M, K, np, lda, sA, batch, psA);
    const long long spB = piece_span(b_kcont, N, K, np, ldb, sB, batch, psB);
    if (spA < 0 || spB < 0) return VFM_NO_KERNEL;
    G8Args a{};
    a.stamps = g_stamps;
    a.spanA = (unsigned)spA;
    a.spanB = (unsigned)spB;
    a.Kp = K;
    a.psA = psA ? psA : (a_kcont ? (long long)K : (long long)K * lda);
    a.psB = psB ? psB : (b_kcont ? (long long)K : (long long)K * ldb);
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

extern "C" int vfm_gemm8(const void* A, const void* B, void* C, const float* bias, int precision, int out_dtype, int M,
                         int N, int K, int batch, int a_kcont, long long lda, long long sA, int b_kcont, long long ldb,
                         long long sB, long long ldc, long long sC, float alpha, float beta, int bias_mode, int act,
                         float* workspace, int kchunk, int reduce_batch, void* stream) {
    return gemm8_impl(A, B, C, bias, precision, out_dtype, M, N, K, batch, a_kcont, lda, sA, 0, b_kcont, ldb, sB, 0,
                      ldc, sC, alpha, beta, bias_mode, act, workspace, kchunk, reduce_batch, stream);
}

// vfm_gemm8 with explicit piece strides (elements; 0 = the stacked layouts of vfm_split_f32): planar
// pieces [NP][tensor] of an fp32 tensor (vfm_split_f32 with R = 1 over the whole tensor) addressed
// through any strided view of it, so one split serves every product the tensor enters.
extern "C" int vfm_gemm8_pieces(const void* A, const void* B, void* C, const float* bias, int precision, int out_dtype,
                                int M, int N, int K, int batch, int a_kcont, long long lda, long long sA, long long psA,
                                int b_kcont, long long ldb, long long sB, long long psB, long long ldc, long long sC,
                                float alpha, float beta, int bias_mode, int act, float* workspace, int kchunk,
                                int reduce_batch, void* stream) {
    return gemm8_impl(A, B, C, bias, precision, out_dtype, M, N, K, batch, a_kcont, lda, sA, psA, b_kcont, ldb, sB,
                      psB, ldc, sC, alpha, beta, bias_mode, act, workspace, kchunk, reduce_batch, stream);
}

// ConvNeXt-MLP 1x1 GEMMs with the GELU epilogues (gelu_epilogue above), bf16 operands and outputs:
//   C[z] = W[M, K] X[z][K, N] with W K-contiguous (lda), X N-contiguous (ldb, batch stride sB);
//   mode 1: C = h (may be null), C2 = g = GELU(h s + b1); mode 2: C = dh from acc = dg and H = h,
//   rsum0 (may be null) / rsum1 = [batch][vfm_gemm8_gelu_parts(N)][M] partial sums.
// rscale [batch][M] (null: 1), bias [M] (null: 0). C, C2, H share (ldc, sC).
extern "C" int vfm_gemm8_gelu(const void* W, const void* X, void* C, void* C2, const void* H, const float* rscale,
                              const float* bias, float* rsum0, float* rsum1, int mode, int M, int N, int K, int batch,
                              long long lda, long long ldb, long long sB, long long ldc, long long sC, void* stream) {
    if (!W || !X || M <= 0 || N <= 0 || K <= 0 || batch <= 0 || batch > 65535) return VFM_ERR_ARGS;
    if (mode == 1 ? !C2 : (mode == 2 ? (!C || !H || !rsum1) : true)) return VFM_ERR_ARGS;
    if (K % BK || K % 8 || N % 8 || lda % 8 || ldb % 8 || sB % 8 || ldc % 8 || sC % 8) return VFM_NO_KERNEL;
    if (((uintptr_t)W | (uintptr_t)X) % 16) return VFM_NO_KERNEL;
    if (lda < K || ldb < N || ldc < N) return VFM_ERR_ARGS;
    const long long spA = span_bytes(1, M, K, lda, 0, 1), spB = span_bytes(0, N, K, ldb, sB, batch);
    if (spA < 0 || spB < 0) return VFM_NO_KERNEL;
    G8Args a{};
    a.spanA = (unsigned)spA;
    a.spanB = (unsigned)spB;
    a.A = (const __hip_bfloat16*)W; a.B = (const __hip_bfloat16*)X; a.C = C; a.C2 = C2;
    a.H = (const __hip_bfloat16*)H; a.rscale = rscale; a.bias = bias; a.rs0 = rsum0; a.rs1 = rsum1;
    a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.sA = 0; a.sB = sB; a.sC = sC;
    a.M = M; a.N = N; a.K = K; a.alpha = 1.f; a.beta = 0.f; a.bias_mode = 0; a.act = 0;
    a.Kp = K; a.T = 1; a.pa = a.pb = 0; a.psA = K; a.psB = (long long)K * ldb;
    a.Z = batch; a.reduce = 0; a.kchunk = K / BK; a.S = 1; a.ws = nullptr;
    a.stamps = g_stamps;
    const long long nwg = (long long)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    if (nwg > 0x7fffffffLL) return VFM_ERR_ARGS;
    hipStream_t st = (hipStream_t)stream;
    if (mode == 1) launch8k<true, false, false, 1>(a, (int)nwg, batch, st);
    else launch8k<true, false, false, 2>(a, (int)nwg, batch, st);
    return launch_status();
}

// Microbenchmarks only: device buffer of 16 int64 per block (s_memrealtime stamps, see G8Args::stamps)
// for the following vfm_gemm8 / vfm_gemm8_gelu launches; null turns the stamps off.
extern "C" int vfm_gemm8_set_stamps(long long* buf) {
    g_stamps = buf;
    return VFM_OK;
}

// K-tile staging schedule of vfm_gemm8 / vfm_gemm8_gelu (A/B switch for microbenchmarks): 1 = half-tile
// slots restaged two K-tiles ahead, 0 = one K-tile ahead (default: 8192^3 1284 vs 1120 TF/s, SigLIP2
// qkv 879 vs 805, profiles/r3_k_gemm8_shapes.txt). Returns the previous value.
extern "C" int vfm_gemm8_set_schedule(int deep) {
    const int prev = g_deep;
    g_deep = deep ? 1 : 0;
    return prev;
}

// Partial-sum slots per (batch, row) of vfm_gemm8_gelu mode 2 for N columns.
extern "C" int vfm_gemm8_gelu_parts(int N) { return N <= 0 ? -1 : 4 * ((N + BN - 1) / BN); }

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
