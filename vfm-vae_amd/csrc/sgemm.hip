// Exact-fp32 GEMM on the fp32-input MFMA (v_mfma_f32_32x32x2_f32): the fp32 products the reference
// runs with TF32 off (training/training_loop.py:504-505) whose shapes the bf16-piece kernels serve
// badly -- the D heads' batch-folded 1-D convolutions (reference networks/discriminator.py:39-42,
// :116-142, SpectralConv1d k = 1 / 9 over [B, 384, 196] DINO tokens) and the decoder's narrow fp32 1x1
// convolutions of the 4^2 .. 16^2 blocks (reference networks/utils/convnext_utils.py:36-57 and :135-138,
// gigagan_utils.py:53-185, generator.py:726-783: per-sample planes of 16 .. 256 pixels). No operand split
// (the f32x6 forms need a split pass per tensor and six products), one product per multiply-add, each
// output a k-ordered chain of fmaf (the MFMA's exact-fp32 numerics): the reference's precision class.
//
//   C[z] = epi( alpha * A[z] . B[z] + beta * C[z] )       A: M x K, B: K x N, fp32
//   epi: + bias (per column or per row), then GELU (tanh / erf) -- the vfm_gemm contract.
//
// Tile BM x BN x 32 (BM, BN in {64, 128}), 4 waves (2 x 2), each wave (BM/2) x (BN/2) as 32 x 32 blocks.
// Both operands staged in LDS as [k][outer] fp32 images, so every MFMA operand is one ds_read_b32 of 32
// consecutive floats per half-wave (lane l: A[m = l & 31][k = l >> 5], B[k = l >> 5][n = l & 31]):
//   * K-contiguous global operand (rows = outer, 16-B chunks along k): transposed on the way in by four
//     ds_write_b32 per chunk into rows of S = BM + 1 floats (S = 1 mod 8: the 32 lanes of a half-wave --
//     4 outer rows x 8 k-chunks -- hit 32 distinct banks);
//   * MN-contiguous global operand (rows = k, 16-B chunks along outer): one ds_write_b128 per chunk into
//     rows of S = BM + 4 floats.
// The next K-tile is loaded into registers while the current one is multiplied (written to LDS after
// the barrier). The fp32 MFMA runs at 1/16 of the bf16 rate (64 FLOP/clk/SIMD): per K-tile a wave issues
// 16 x TI x TJ MFMAs (64 cycles each) against 2 x 16 LDS reads and <= 16 LDS writes, so the loop is
// MFMA-bound with the staging in its shadow and two workgroups per CU.
//
// Reductions longer than one workgroup's share: the virtual K-tiles of an output tile -- the K-tiles of
// one batch item, or of every batch item when reduce_batch (C = alpha sum_z A[z] B[z]: the weight
// gradients) -- are cut into `splits` chunks; each chunk writes an fp32 partial tile to the workspace
// and sgemm_reduce sums them in a fixed order (deterministic) before the epilogue.
// Batch folding (lgp > 0, the vfm_gemm_fold layout): B[z] MN-contiguous [K][P], C[z] [M][P] with
// P = 2^lgp columns per sample, run as ONE product over N = batch * P columns (column n -> sample
// n >> lgp): the 4 x 4 / 8 x 8 planes fill whole 64- / 128-wide tiles.
#include "vfm_common.h"

#include <type_traits>

namespace {

using namespace vfm;

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BK = 32, NT = 256;

struct SgArgs {
    const float* A;
    const float* B;
    float* C;
    const float* bias;
    float* ws;                 // partials [J][M][N] (null: direct epilogue)
    long long lda, ldb, ldc, sA, sB, sC;
    int M, N, K, batch, splits, reduce, lgp;
    int kt;                    // K-tiles per batch item
    int tpc;                   // virtual K-tiles per split chunk
    int tiles_m, tiles_n;
    float alpha, beta;
    int bias_mode, act;        // bias 0 none / 1 per column / 2 per row; act 0 none / 1 gelu tanh / 2 gelu erf
    int va, vb;                // operand staged with 16-B loads (contiguous extent, leading dims, base: 16-B units)
};

__device__ __forceinline__ float gelu_tanh_f(float x) {
    const float u = 0.7978845608028654f * fmaf(0.044715f * x, x * x, x);
    const float e = __builtin_amdgcn_exp2f(2.8853900817779268f * u);
    const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
    return 0.5f * x * (1.f + t);
}

__device__ __forceinline__ float epilogue(const SgArgs& a, float v, int m, int n, float cold) {
    v *= a.alpha;
    if (a.beta != 0.f) v = fmaf(a.beta, cold, v);
    if (a.bias_mode == 1) v += a.bias[a.lgp ? (n & ((1 << a.lgp) - 1)) : n];
    else if (a.bias_mode == 2) v += a.bias[m];
    if (a.act == 1) v = gelu_tanh_f(v);
    else if (a.act == 2) v = v * gelu_parts(v).cdf;
    return v;
}

// One operand tile (O outer x 32 k) global -> registers -> LDS image [2][O][16]: half hh = k / 16, outer row,
// s = k % 16 contiguous, the four 16-B slots of a row XOR-swizzled by (row >> 2) & 3, and 16 pad floats before
// half 1 (so the two halves of a row land on disjoint banks). The MFMA k-step s (0..15) pairs k = s (lanes 0-31)
// with k = 16 + s (lanes 32-63) -- the same permutation of the K-tile for both operands -- so a lane's fragments
// of 4 consecutive k-steps are ONE ds_read_b128 (the 16 lanes of each b128 lane group hit 16 distinct 16-B slots
// of the 256-B bank row).
//   K-contiguous operand (global rows = outer, 16-B chunks along k): one chunk = one ds_write_b128;
//   MN-contiguous operand (global rows = k, chunks along outer): the 32 lanes of a half-wave take the 32 k of
//     one chunk column, so the chunk's four ds_write_b32 (one per outer row) hit 32 distinct banks.
template <bool KCONT, int O, int NTH>
struct Stage {
    static constexpr int HALF = O * 16 + 16;                   // floats of half 0 (+ pad)
    static constexpr int FLOATS = 2 * HALF;
    static constexpr int CHUNKS = O * BK / 4;                  // 16-B chunks per tile
    static constexpr int PER = CHUNKS / NTH;
    static_assert(PER * NTH == CHUNKS, "chunks per thread");
    float4 r[PER];

    // chunk c of the tile -> (outer row offset, k offset)
    __device__ __forceinline__ static void chunk(int c, int& row, int& kk) {
        if (KCONT) { row = c >> 3; kk = (c & 7) * 4; }         // 8 chunks per outer row (128 B)
        else       { kk = c & 31; row = (c >> 5) * 4; }        // lanes along k, 4 outer per chunk
    }

    // base: the operand of this batch item; outer0 / k0: tile origin; bounds outer_n / K.
    // Folded (lgp): outer index o -> item o >> lgp at stride sb, column o & (2^lgp - 1) (MN-contiguous only).
    __device__ __forceinline__ void load(const float* base, long long ld, int outer0, int k0, int outer_n, int K,
                                         int tid, int lgp, long long sb, int vec) {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            int row, kk;
            chunk(tid + NTH * u, row, kk);
            const int o = outer0 + row, k = k0 + kk;
            if (vec) {
                long long off;
                if (KCONT) off = (long long)o * ld + k;
                else if (lgp) off = (long long)(o >> lgp) * sb + (long long)k * ld + (o & ((1 << lgp) - 1));
                else off = (long long)k * ld + o;
                // branch-free bounds: an out-of-range chunk loads the operand's first chunk and is zeroed
                const bool ok = o < outer_n && k < K;
                const float4 v = *reinterpret_cast<const float4*>(base + (ok ? off : 0LL));
                r[u] = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
            } else {
                // contiguous extent / leading dim not in 16-B units (the equivariance decodes' 3 x 3 planes):
                // four bounds-checked scalar loads
                float e[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int oi = KCONT ? o : o + i, ki = KCONT ? k + i : k;
                    long long off;
                    if (KCONT) off = (long long)oi * ld + ki;
                    else if (lgp) off = (long long)(oi >> lgp) * sb + (long long)ki * ld + (oi & ((1 << lgp) - 1));
                    else off = (long long)ki * ld + oi;
                    e[i] = (oi < outer_n && ki < K) ? base[off] : 0.f;
                }
                r[u] = make_float4(e[0], e[1], e[2], e[3]);
            }
        }
    }

    __device__ __forceinline__ static int at(int row, int kk) {       // float index of (row, k) in the image
        const int ss = kk & 15;
        return (kk >> 4) * HALF + row * 16 + 4 * ((ss >> 2) ^ ((row >> 2) & 3)) + (ss & 3);
    }

    __device__ __forceinline__ void store(float* img, int tid) const {
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            int row, kk;
            chunk(tid + NTH * u, row, kk);
            if (KCONT) {
                *reinterpret_cast<float4*>(img + at(row, kk)) = r[u];
            } else {
                img[at(row, kk)] = r[u].x;
                img[at(row + 1, kk)] = r[u].y;
                img[at(row + 2, kk)] = r[u].z;
                img[at(row + 3, kk)] = r[u].w;
            }
        }
    }

    // fragments of k-steps 4q .. 4q + 3 of the lane's row (orow + (lane & 31)) of the image
    __device__ __forceinline__ static float4 quad(const float* img, int lane, int orow, int q) {
        const int row = orow + (lane & 31);
        return *reinterpret_cast<const float4*>(img + (lane >> 5) * HALF + row * 16 + 4 * (q ^ ((row >> 2) & 3)));
    }
};

// virtual K-tile t of the chunk -> (batch item, k0)
__device__ __forceinline__ void vtile(const SgArgs& a, int zfix, int t, int& z, int& k0) {
    if (a.reduce) { z = t / a.kt; k0 = (t - z * a.kt) * BK; }
    else          { z = zfix; k0 = t * BK; }
}

// KW wave groups (KW x 256 threads): group g multiplies k-step quads [g 4/KW, (g + 1) 4/KW) of every K-tile
// into its own accumulators, summed through LDS (fixed order) before the epilogue -- KW = 2 puts two waves of
// one output tile on every SIMD, for the grids whose tiles would otherwise leave one wave per SIMD.
template <bool AK, bool BKC, int BM, int BN, int KW>
__global__ __launch_bounds__(NT * KW, 2 / KW) void sgemm_kernel(SgArgs a) {
    constexpr int WM = 2, WN = 2, TI = BM / WM / 32, TJ = BN / WN / 32, NTH = NT * KW, QG = 4 / KW;
    typedef Stage<AK, BM, NTH> SA;
    typedef Stage<BKC, BN, NTH> SB;
    // two stages: the K-tile being multiplied and the next one being stored
    constexpr int STAGE = SA::FLOATS + SB::FLOATS;
    __shared__ __attribute__((aligned(16))) float lds[2 * STAGE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int kg = wave >> 2, wm = wave & 1, wn = (wave >> 1) & 1;
    // XCD-aware tile order: workgroups b, b + 8, ... share an XCD (and its L2); give them consecutive
    // tiles, m fastest, so the M-tiles reading one B column panel run on one L2
    const int ntile = a.tiles_m * a.tiles_n;
    int tile = blockIdx.x;
    if ((ntile & 7) == 0) tile = (blockIdx.x & 7) * (ntile >> 3) + (blockIdx.x >> 3);
    const int tm = tile % a.tiles_m, tn = tile / a.tiles_m;
    const int m0 = tm * BM, n0 = tn * BN;
    const int split = blockIdx.y % a.splits, zfix = blockIdx.y / a.splits;
    const int vt_total = a.reduce ? a.batch * a.kt : a.kt;
    const int t0 = split * a.tpc, t1 = min(vt_total, t0 + a.tpc);

    SA sa[2];                  // register sets of K-tiles t + 1 / t + 2 (two-deep global prefetch)
    SB sb[2];
    f32x16 acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) acc[i][j] = f32x16{};

    const long long sBb = a.lgp ? 0LL : a.sB;
    auto load = [&](int t, SA& ra, SB& rb) {
        int z, k0;
        vtile(a, zfix, t, z, k0);
        ra.load(a.A + z * a.sA, a.lda, m0, k0, a.M, a.K, tid, 0, 0, a.va);
        rb.load(a.B + z * sBb, a.ldb, n0, k0, a.N, a.K, tid, a.lgp, a.sB, a.vb);
    };
    const int ao = (BM / WM) * wm, bo = (BN / WN) * wn, qb = kg * QG;
    // the MFMAs of one K-tile from an LDS stage, fragments one quad of k-steps ahead (the b128 reads of quad
    // q + 1 issued before the MFMAs of quad q)
    auto compute = [&](const float* cur) {
        float4 fa[2][TI], fb[2][TJ];
#pragma unroll
        for (int i = 0; i < TI; ++i) fa[0][i] = SA::quad(cur, lane, ao + 32 * i, qb);
#pragma unroll
        for (int j = 0; j < TJ; ++j) fb[0][j] = SB::quad(cur + SA::FLOATS, lane, bo + 32 * j, qb);
#pragma unroll
        for (int q = 0; q < QG; ++q) {
            if (q + 1 < QG) {
#pragma unroll
                for (int i = 0; i < TI; ++i) fa[(q + 1) & 1][i] = SA::quad(cur, lane, ao + 32 * i, qb + q + 1);
#pragma unroll
                for (int j = 0; j < TJ; ++j) fb[(q + 1) & 1][j] = SB::quad(cur + SA::FLOATS, lane, bo + 32 * j, qb + q + 1);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int i = 0; i < TI; ++i)
#pragma unroll
                    for (int j = 0; j < TJ; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[q & 1][i][e], fb[q & 1][j][e], acc[i][j],
                                                                        0, 0, 0);
        }
    };
    // K-tile t (local index u = t - t0) lives in LDS stage u & 1 and, before that, in register set u & 1.
    // Iteration u: issue the loads of tile u + 2 into set u & 1 (tile u left it at iteration u - 1), multiply
    // stage u & 1, store set (u + 1) & 1 (tile u + 1, loaded at the start of iteration u - 1: two K-tiles of
    // MFMAs to land) into stage (u + 1) & 1 (last read in iteration u - 1), ONE barrier.
    const int nt = t1 - t0;
    if (nt > 0) {
        load(t0, sa[0], sb[0]);
        if (nt > 1) load(t0 + 1, sa[1], sb[1]);
        sa[0].store(lds, tid);
        sb[0].store(lds + SA::FLOATS, tid);
        __syncthreads();
    }
    auto iter = [&](int u, auto par) {
        constexpr int P = decltype(par)::value;
        if (u + 2 < nt) load(t0 + u + 2, sa[P], sb[P]);
        compute(lds + P * STAGE);
        if (u + 1 < nt) {
            sa[P ^ 1].store(lds + (P ^ 1) * STAGE, tid);
            sb[P ^ 1].store(lds + (P ^ 1) * STAGE + SA::FLOATS, tid);
        }
        __syncthreads();
    };
    for (int u = 0; u < nt; u += 2) {
        iter(u, std::integral_constant<int, 0>());
        if (u + 1 < nt) iter(u + 1, std::integral_constant<int, 1>());
    }

    if (KW > 1) {
        // the other groups' accumulators through LDS (the loop ended on a barrier): lane-contiguous slots
        static_assert(KW == 1 || (KW - 1) * 4 * TI * TJ * 16 * 64 <= 2 * STAGE, "reduction buffer");
        float* red = lds + ((kg - 1) * 4 + (wave & 3)) * (TI * TJ * 16 * 64) + lane;
        if (kg > 0) {
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int j = 0; j < TJ; ++j)
#pragma unroll
                    for (int e = 0; e < 16; ++e) red[((i * TJ + j) * 16 + e) * 64] = acc[i][j][e];
        }
        __syncthreads();
        if (kg > 0) return;
#pragma unroll
        for (int g = 1; g < KW; ++g) {
            const float* rp = lds + ((g - 1) * 4 + wave) * (TI * TJ * 16 * 64) + lane;
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int j = 0; j < TJ; ++j)
#pragma unroll
                    for (int e = 0; e < 16; ++e) acc[i][j][e] += rp[((i * TJ + j) * 16 + e) * 64];
        }
    }

    const int r = lane & 31, hh = lane >> 5;
    // acc[i][j][e] = C[m][n]: m = m0 + (BM/2) wm + 32 i + (e & 3) + 8 (e >> 2) + 4 hh, n = n0 + (BN/2) wn + 32 j + r
    if (a.ws) {
        const int jslot = a.reduce ? split : zfix * a.splits + split;
        float* w = a.ws + (long long)jslot * a.M * a.N;
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
            const int n = n0 + (BN / WN) * wn + 32 * j + r;
            if (n >= a.N) continue;
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int m = m0 + (BM / WM) * wm + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * hh;
                    if (m < a.M) w[(long long)m * a.N + n] = acc[i][j][e];
                }
        }
        return;
    }
    float* Cb = a.C + (a.lgp ? 0LL : (long long)zfix * a.sC);
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
        const int n = n0 + (BN / WN) * wn + 32 * j + r;
        if (n >= a.N) continue;
        float* Cn = a.lgp ? Cb + (long long)(n >> a.lgp) * a.sC + (n & ((1 << a.lgp) - 1)) : Cb + n;
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int m = m0 + (BM / WM) * wm + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * hh;
                if (m >= a.M) continue;
                float* cp = Cn + (long long)m * a.ldc;
                *cp = epilogue(a, acc[i][j][e], m, n, a.beta != 0.f ? *cp : 0.f);
            }
    }
}

// C = epi(sum_j ws[j]) for j < J (fixed order), over the (z, m, n) outputs; four columns per thread.
__global__ void sgemm_reduce(SgArgs a, int J) {
    const long long MN = (long long)a.M * a.N;
    const long long q = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    const int zc = blockIdx.y;
    if (q >= MN) return;
    const float* w = a.ws + (long long)zc * J * MN + q;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    const int cnt = (int)min(4LL, MN - q);
    if ((a.N & 3) == 0) {                      // rows of whole float4s (q is a multiple of 4)
        for (int j = 0; j < J; ++j) {
            const float4 v = *reinterpret_cast<const float4*>(w + (long long)j * MN);
            s[0] += v.x; s[1] += v.y; s[2] += v.z; s[3] += v.w;
        }
    } else {
        for (int j = 0; j < J; ++j)
            for (int c = 0; c < cnt; ++c) s[c] += w[(long long)j * MN + c];
    }
    for (int c = 0; c < cnt; ++c) {
        const long long qi = q + c;
        const int mi = (int)(qi / a.N), ni = (int)(qi - (long long)mi * a.N);
        float* cp = a.C + (long long)zc * a.sC + (long long)mi * a.ldc + ni;
        *cp = epilogue(a, s[c], mi, ni, a.beta != 0.f ? *cp : 0.f);
    }
}

template <bool AK, bool BKC, int BM, int BN, int KW>
int launch(const SgArgs& a, int gy, hipStream_t st) {
    const int ntile = a.tiles_m * a.tiles_n;
    VFM_LAUNCH((sgemm_kernel<AK, BKC, BM, BN, KW>), dim3(ntile, gy), dim3(NT * KW), 0, st, a);
    return launch_status();
}

template <int BM, int BN, int KW>
int launch_layout(const SgArgs& a, int gy, int ak, int bk, hipStream_t st) {
    if (ak && bk) return launch<true, true, BM, BN, KW>(a, gy, st);
    if (ak) return launch<true, false, BM, BN, KW>(a, gy, st);
    if (bk) return launch<false, true, BM, BN, KW>(a, gy, st);
    return launch<false, false, BM, BN, KW>(a, gy, st);
}

// tile code: bits 0-1: 0 = 128 x 128, 1 = 128 x 64, 2 = 64 x 128, 3 = 64 x 64; bit 2: two wave groups (KW = 2)
inline int tile_bm(int code) { return (code & 2) ? 64 : 128; }
inline int tile_bn(int code) { return (code & 1) ? 64 : 128; }

// Heuristic tile when the caller passes tile < 0: the largest tile whose grid still covers the chip
// (~256 CUs x 2 workgroups) at the given batch and splits; narrow outputs take the 64-wide forms.
int pick_tile(int M, int N, int batch_tiles) {
    int best = 3;
    for (int code = 0; code < 4; ++code) {
        const int bm = tile_bm(code), bn = tile_bn(code);
        if ((bm == 128 && M <= 64) || (bn == 128 && N <= 64)) continue;
        const long long tiles = (long long)((M + bm - 1) / bm) * ((N + bn - 1) / bn) * batch_tiles;
        if (tiles >= 256) return code;
        best = code;
    }
    return best;
}

}  // namespace

extern "C" long long vfm_sgemm_workspace_floats(int M, int N, int batch, int splits, int reduce_batch) {
    if (splits < 1) splits = 1;
    if (splits == 1 && !reduce_batch) return 0;
    return (long long)M * N * (reduce_batch ? splits : (long long)batch * splits);
}

extern "C" int vfm_sgemm(const float* A, const float* B, float* C, const float* bias, int M, int N, int K, int batch,
                         int a_kcont, long long lda, long long sA, int b_kcont, long long ldb, long long sB,
                         long long ldc, long long sC, float alpha, float beta, int bias_mode, int act, int lgp,
                         float* workspace, int splits, int reduce_batch, int tile, void* stream) {
    if (!A || !B || !C || M <= 0 || N <= 0 || K <= 0 || batch <= 0) return VFM_ERR_ARGS;
    if (bias_mode < 0 || bias_mode > 2 || (bias_mode && !bias) || act < 0 || act > 2) return VFM_ERR_ARGS;
    if (splits < 1) splits = 1;
    if (lgp && (b_kcont || reduce_batch || lgp < 2 || lgp > 20)) return VFM_ERR_ARGS;
    const int P = lgp ? (1 << lgp) : N;
    // 16-B loads where every contiguous extent, leading dim and batch stride is in 16-B units and the base is
    // 16-B aligned; otherwise bounds-checked scalar loads
    const int a_c = a_kcont ? K : M, b_c = b_kcont ? K : P;
    const int va = !(a_c % 4 || lda % 4 || sA % 4 || ((uintptr_t)A % 16));
    const int vb = !(b_c % 4 || ldb % 4 || sB % 4 || ((uintptr_t)B % 16));
    if (lda < a_c || ldb < b_c || ldc < P) return VFM_ERR_ARGS;
    const long long Nf = lgp ? (long long)batch * P : N;
    if (lgp && (Nf != N)) return VFM_ERR_ARGS;
    const bool use_ws = splits > 1 || reduce_batch;
    if (use_ws && (!workspace || lgp)) return VFM_ERR_ARGS;
    const int kt = (K + BK - 1) / BK;
    const int vt = reduce_batch ? batch * kt : kt;
    if (splits > vt) splits = vt;
    SgArgs a;
    a.A = A; a.B = B; a.C = C; a.bias = bias;
    a.lda = lda; a.ldb = ldb; a.ldc = ldc; a.sA = sA; a.sB = sB; a.sC = sC;
    a.M = M; a.N = N; a.K = K; a.batch = batch; a.reduce = reduce_batch ? 1 : 0; a.lgp = lgp;
    a.kt = kt;
    a.tpc = (vt + splits - 1) / splits;
    a.splits = (vt + a.tpc - 1) / a.tpc;           // no empty chunk
    a.alpha = alpha; a.beta = beta; a.bias_mode = bias_mode; a.act = act;
    a.ws = use_ws ? workspace : nullptr;
    a.va = va; a.vb = vb;
    const int zgrid = (reduce_batch || lgp) ? 1 : batch;
    if ((long long)zgrid * a.splits > 65535) return VFM_ERR_ARGS;
    if (tile < 0 || tile > 7) tile = pick_tile(M, N, zgrid * a.splits);
    const int bm = tile_bm(tile), bn = tile_bn(tile);
    a.tiles_m = (M + bm - 1) / bm;
    a.tiles_n = (N + bn - 1) / bn;
    hipStream_t st = (hipStream_t)stream;
    const int gy = zgrid * a.splits;
    int rc;
    switch (tile) {
    case 0: rc = launch_layout<128, 128, 1>(a, gy, a_kcont, b_kcont, st); break;
    case 1: rc = launch_layout<128, 64, 1>(a, gy, a_kcont, b_kcont, st); break;
    case 2: rc = launch_layout<64, 128, 1>(a, gy, a_kcont, b_kcont, st); break;
    case 3: rc = launch_layout<64, 64, 1>(a, gy, a_kcont, b_kcont, st); break;
    case 4: rc = launch_layout<128, 128, 2>(a, gy, a_kcont, b_kcont, st); break;
    case 5: rc = launch_layout<128, 64, 2>(a, gy, a_kcont, b_kcont, st); break;
    case 6: rc = launch_layout<64, 128, 2>(a, gy, a_kcont, b_kcont, st); break;
    default: rc = launch_layout<64, 64, 2>(a, gy, a_kcont, b_kcont, st); break;
    }
    if (rc != VFM_OK || !use_ws) return rc;
    const long long MN = (long long)M * N;
    const int J = a.splits;
    const int zc = reduce_batch ? 1 : batch;
    VFM_LAUNCH(sgemm_reduce, dim3((unsigned)((MN / 4 + 255) / 256 + 1), zc), dim3(256), 0, st, a, J);
    return launch_status();
}
