// Style affine + demodulation coefficients of a ConvNeXt synthesis layer, forward (two launches)
// and backward (four launches), fp32. Reference: networks/utils/convnext_utils.py ConvNeXtBlock
// (affine_pw1 = StyleSplit(FullyConnectedLayer(w_dim, 3C)), networks/utils/shared.py StyleSplit /
// FullyConnectedLayer, and the demodulation of ModulatedPointwiseConv2DLayer, convnext_utils.py:60-66):
//
//   m[b, j] = wg sum_k w[b, k] A[j, k] + bg ab[j]                     j < 3C   (FullyConnectedLayer)
//   s[b, c] = m[b, c] m[b, C + c] + m[b, 2C + c]                               (StyleSplit)
//   d[b, o] = rsqrt(sum_i W1[o, i]^2 s[b, i]^2 + eps)                 o < O    (demodulation)
//
// torch runs this as ~9 kernels per layer forward (gain scalings, addmm, split products, squares, the
// mm, eps, rsqrt) and ~25 in its backward. Backward, with q = -dd d^3 / 2:
//   ds[b, i]  = ds_in[b, i] + 2 s[b, i] sum_o q[b, o] W1[o, i]^2
//   dW1[o, i] = 2 W1[o, i] sum_b q[b, o] s[b, i]^2
//   dm = (ds m2, ds m1, ds)  (per split part),
//   dA[j, k] = wg sum_b dm[b, j] w[b, k],   dab[j] = bg sum_b dm[b, j],
//   dw[b, k] = wg sum_j dm[b, j] A[j, k]
//
// Every product is skinny: one side is the batch (B <= a few dozen), the other a weight matrix of up to
// 2048 x 512. The kernels read each weight matrix once for the whole batch (32 samples per pass):
//  * forward reductions along the contiguous rows (m over the rows of A, d over the rows of W1): 4-sample
//    x CB-row tiles, one per wave (K < 1024) or per block, lanes striding over k (coalesced), the
//    partial sums reduced across the wave with xor shuffles. (A whole-batch form with the rows staged
//    in LDS, 32 blocks at C = 512, measured 74 us against this form's 24 us: too few waves in flight
//    to cover the load latency.)
//  * column sums over the contiguous axis (backward ds over the rows of W1^2, dw over the rows of A):
//    a block owns 64 columns (lane = column: coalesced rows) and a 64-deep K chunk, each wave 8 samples
//    whose factors it reads from LDS as broadcasts; the K chunks' partial sums [KS][B][N] are added in a
//    fixed order by a small second launch (deterministic; no atomics).
//  * outer products over the batch (dW1, dA, dab): 32-row x 128-column output tiles per block, the
//    batch factors staged in LDS 32 samples at a time, 4 x 4 register tiles, float4 stores.
// All sums are plain fp32 FMAs (the reference runs them in fp32 with TF32 off).
// Backward at C = 512, B = 32 (tools_dev/stylebench.py, profiles/r4_h / r4_i): 58 -> 44 us (ds job 30 -> 21
// us, dw job 20 -> 16 us; they had one 4-sample x 8-column tile per block: the weight matrix re-read
// per sample group and ~200 cross-lane shuffles per tile).
#include "vfm_common.h"

namespace {

using namespace vfm;

constexpr int THREADS = 256, WAVES = THREADS / 64, RB = 4;
constexpr int KCH = 32;                  // K range of one column-sum block (32: four load round trips per column at unroll 8; 64 took eight)
constexpr int SPASS = 32;                // samples per pass of the column sums

struct StyleArgs {
    const float* w;
    long long ldw;                        // row stride of w [B, WD] (a column slice of ws)
    const float* A;                       // [3C, WD]
    const float* ab;                      // [3C]
    const float* W1;                      // [O, C] or null (no demodulation)
    float wg, bg, eps;
    int B, C, WD, O;
    float* m;                             // [B, 3C]
    float* s;                             // [B, C]
    float* d;                             // [B, O]
    const float* dsin;                    // [B, C] or null
    const float* dd;                      // [B, O]
    const float* dsv;                     // ds for the dm factors (the workspace's ds, or dsin)
    float* ds;                            // [B, C] (workspace)
    float* part;                          // [KS][B][N] column-sum partials (workspace)
    float* dW1;                           // [O, C] or null
    float* dA;                            // [3C, WD] or null
    float* dab;                           // [3C] or null
    float* dw;                            // [B, WD] (row stride lddw) or null
    long long lddw;
    int blocks0;                          // blocks of the launch's first job
    int tpb;                              // tiles per block of the forward's tile jobs (1 or WAVES)
    int ks;                               // K chunks of the column-sum job
};

__host__ __device__ inline int cdiv_i(long long a, long long b) { return (int)((a + b - 1) / b); }

// acc[r][c] = sum_k X(r, k) Y(c, k) over k < K: ldx(k, x[RB]) / ldy(k, y[CB]) load the operand values
// of one k (zero outside the operand). tpb = 4 (short K): one tile per wave, its 64 lanes striding
// over k, the partial sums reduced across the wave with xor shuffles (result in every lane).
// tpb = 1 (long K): one tile per block, the 256 threads striding over k, the four waves' sums meeting
// in LDS (result in wave 0). Loads are coalesced along k either way.
template <int CB, class LX, class LY>
__device__ __forceinline__ void tile_mm(int K, int tpb, LX ldx, LY ldy, float (&acc)[RB][CB], float* red) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int c = 0; c < CB; ++c) acc[r][c] = 0.f;
    const int step = tpb == 1 ? THREADS : 64;
#pragma unroll 2
    for (int k = tpb == 1 ? (int)threadIdx.x : lane; k < K; k += step) {
        float x[RB], y[CB];
        ldx(k, x);
        ldy(k, y);
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int c = 0; c < CB; ++c) acc[r][c] = fmaf(x[r], y[c], acc[r][c]);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int c = 0; c < CB; ++c) acc[r][c] += __shfl_xor(acc[r][c], o, 64);
    if (tpb != 1) return;
    if (wave > 0 && lane == 0)
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int c = 0; c < CB; ++c) red[((wave - 1) * RB + r) * CB + c] = acc[r][c];
    __syncthreads();
    if (wave == 0)
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int c = 0; c < CB; ++c)
                acc[r][c] += (red[r * CB + c] + red[(RB + r) * CB + c]) + red[(2 * RB + r) * CB + c];
}

// ---------------------------------------------------------------------------------------------------
// Column sums: part[ks][b][n] = sum_{k in chunk ks} X(b, k) Y(k, n) for the block's 64 columns, all samples
// (passes of 32: wave wv takes samples bp + 8 wv .. + 7). LX(b, k) / LY(k, n) as above.
template <class LX, class LY>
__device__ __forceinline__ void col_sums(int K, int N, int B, int strip, int ks, LX lx, LY ly, float* part,
                                         float* xs) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int n = strip * 64 + lane, k0 = ks * KCH, kn = min(KCH, K - k0);
    for (int bp = 0; bp < B; bp += SPASS) {
        __syncthreads();
        for (int e = t; e < SPASS * KCH; e += THREADS) {        // xs[k][b]: a wave's 8 samples contiguous
            const int b = e / KCH, k = e - b * KCH;
            xs[k * (SPASS + 4) + b] = k < kn ? lx(bp + b, k0 + k) : 0.f;
        }
        __syncthreads();
        float acc[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = 0.f;
        if (n < N) {
#pragma unroll 8
            for (int k = 0; k < kn; ++k) {
                const float y = ly(k0 + k, n);
                const float4 xa = *reinterpret_cast<const float4*>(xs + k * (SPASS + 4) + 8 * wv);
                const float4 xb = *reinterpret_cast<const float4*>(xs + k * (SPASS + 4) + 8 * wv + 4);
                acc[0] = fmaf(xa.x, y, acc[0]); acc[1] = fmaf(xa.y, y, acc[1]);
                acc[2] = fmaf(xa.z, y, acc[2]); acc[3] = fmaf(xa.w, y, acc[3]);
                acc[4] = fmaf(xb.x, y, acc[4]); acc[5] = fmaf(xb.y, y, acc[5]);
                acc[6] = fmaf(xb.z, y, acc[6]); acc[7] = fmaf(xb.w, y, acc[7]);
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int b = bp + 8 * wv + i;
                if (b < B) part[((long long)ks * B + b) * N + n] = acc[i];
            }
        }
    }
}

// sum_{k < ks} p[k stride] added in order k = 0, 1, ... (deterministic), 16 loads in flight per round instead
// of one dependent load-add per partial
__device__ __forceinline__ float sum_parts(const float* p, long long stride, int ks) {
    constexpr int U = 16;
    float acc = 0.f;
    for (int k0 = 0; k0 < ks; k0 += U) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = k0 + u < ks ? p[(k0 + u) * stride] : 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (k0 + u < ks) acc += v[u];
    }
    return acc;
}

__device__ __forceinline__ float dm_at(const StyleArgs& a, int b, int j) {
    const int part = j / a.C, c = j - part * a.C;
    const float g = a.dsv[(long long)b * a.C + c];
    const float* mb = a.m + (long long)b * 3 * a.C;
    return part == 0 ? g * mb[a.C + c] : (part == 1 ? g * mb[c] : g);
}

__device__ __forceinline__ float q_at(const StyleArgs& a, int b, int o) {
    const long long i = (long long)b * a.O + o;
    const float dv = a.d[i];
    return -0.5f * a.dd[i] * dv * dv * dv;
}

// ---------------------------------------------------------------------------------------------------
// out[r][c] = sum_b X(b, r) Y(b, c) over b < B for the block's 32 x 128 tile (r0, c0): X / Y give the
// batch factors (zero outside). Thread t owns rows r0 + 4 (t >> 5) .. + 3, columns c0 + 4 (t & 31) .. + 3;
// rsum (if non-null) gets sum_b X(b, r) of the thread's 4 rows. Staging: xs [32 b][32 r], ys [32 b][128 c].
constexpr int OT_R = 32, OT_C = 128, OT_B = 32;
template <class FX, class FY>
__device__ __forceinline__ void outer_tile(int B, FX X, FY Y, float (&acc)[4][4], float (&rsum)[4], float* xs,
                                           float* ys) {
    const int t = threadIdx.x, ty = t >> 5, tx = t & 31;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        rsum[i] = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
    }
    for (int b0 = 0; b0 < B; b0 += OT_B) {
        __syncthreads();
        {
            const int b = t >> 3, r = 4 * (t & 7);
            float4 v = X(b0 + b, r);
            *reinterpret_cast<float4*>(xs + b * OT_R + r) = v;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = t + 256 * u, b = e >> 5, c = 4 * (e & 31);
            *reinterpret_cast<float4*>(ys + b * OT_C + c) = Y(b0 + b, c);
        }
        __syncthreads();
        const int nb = min(OT_B, B - b0);
        for (int b = 0; b < nb; ++b) {
            const float4 x = *reinterpret_cast<const float4*>(xs + b * OT_R + 4 * ty);
            const float4 y = *reinterpret_cast<const float4*>(ys + b * OT_C + 4 * tx);
            const float xv[4] = {x.x, x.y, x.z, x.w}, yv[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                rsum[i] += xv[i];
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(xv[i], yv[j], acc[i][j]);
            }
        }
    }
}

// four consecutive values of a [rows][cols] fp32 matrix (row stride ld) at (r, c..c+3), zero outside; one
// 16-B load when the row is whole and aligned
__device__ __forceinline__ float4 load4(const float* p, long long ld, int r, int rows, int c, int cols, bool vec) {
    if (r >= rows) return make_float4(0.f, 0.f, 0.f, 0.f);
    const float* q = p + (long long)r * ld + c;
    if (vec && c + 4 <= cols) return *reinterpret_cast<const float4*>(q);
    return make_float4(c < cols ? q[0] : 0.f, c + 1 < cols ? q[1] : 0.f, c + 2 < cols ? q[2] : 0.f,
                       c + 3 < cols ? q[3] : 0.f);
}

__device__ __forceinline__ void store4(float* p, long long ld, int r, int rows, int c, int cols, bool vec, float4 v) {
    if (r >= rows) return;
    float* q = p + (long long)r * ld + c;
    if (vec && c + 4 <= cols) {
        *reinterpret_cast<float4*>(q) = v;
        return;
    }
    const float vv[4] = {v.x, v.y, v.z, v.w};
    for (int j = 0; j < 4 && c + j < cols; ++j) q[j] = vv[j];
}

// LAUNCH 0: m, s   — row dots over A's three split parts of 16 channels (blocks: C / 16)
// LAUNCH 1: d      — row dots over 16 rows of W1 (blocks: O / 16)
// LAUNCH 2: ds partials (column sums over W1^2, blocks0 = strips x K chunks) | dW1 (outer tiles)
// LAUNCH 3: dA + dab (outer tiles, blocks0) | dw partials (column sums over A)
// LAUNCH 4: ds = ds_in + 2 s sum(partials)          LAUNCH 5: dw = wg sum(partials)
template <int LAUNCH>
__device__ __forceinline__ void style_body(const StyleArgs& a, int bid, float* smem) {
    float* red = smem;
    const bool second = bid >= a.blocks0;
    const int blk = second ? bid - a.blocks0 : bid;
    const int C = a.C, C3 = 3 * a.C, WD = a.WD, O = a.O, B = a.B;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    // forward tile jobs: one tile per block (tpb = 1) or per wave (tpb = 4); the result sits in lane
    // `idx` of wave 0 (tpb = 1) or of every wave (tpb = 4)
    const long long wunit = a.tpb == 1 ? (long long)blk : (long long)blk * WAVES + wave;
    const bool owner0 = a.tpb != 1 || wave == 0;
    const int nbg = (B + RB - 1) / RB;                                 // 4-sample groups

    if (LAUNCH == 0) {
        constexpr int CC = 4;
        if (wunit >= (long long)nbg * ((C + CC - 1) / CC)) return;
        const int b0 = (int)(wunit % nbg) * RB, c0 = (int)(wunit / nbg) * CC;
        float acc[RB][3 * CC];
        tile_mm<3 * CC>(WD, a.tpb,
            [&](int k, float (&x)[RB]) {
#pragma unroll
                for (int r = 0; r < RB; ++r) x[r] = b0 + r < B ? a.w[(long long)(b0 + r) * a.ldw + k] : 0.f;
            },
            [&](int k, float (&y)[3 * CC]) {
#pragma unroll
                for (int p = 0; p < 3; ++p)
#pragma unroll
                    for (int c = 0; c < CC; ++c)
                        y[p * CC + c] = c0 + c < C ? a.A[(long long)(p * C + c0 + c) * WD + k] : 0.f;
            }, acc, red);
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int c = 0; c < CC; ++c) {
                const int b = b0 + r, cc = c0 + c;
                if (!owner0 || lane != r * CC + c || b >= B || cc >= C) continue;
                const float m1 = fmaf(a.wg, acc[r][c], a.bg * a.ab[cc]);
                const float m2 = fmaf(a.wg, acc[r][CC + c], a.bg * a.ab[C + cc]);
                const float m3 = fmaf(a.wg, acc[r][2 * CC + c], a.bg * a.ab[2 * C + cc]);
                float* mb = a.m + (long long)b * C3;
                mb[cc] = m1; mb[C + cc] = m2; mb[2 * C + cc] = m3;
                a.s[(long long)b * C + cc] = fmaf(m1, m2, m3);
            }
    } else if (LAUNCH == 1) {
        constexpr int CB = 8;
        if (wunit >= (long long)nbg * ((O + CB - 1) / CB)) return;
        const int b0 = (int)(wunit % nbg) * RB, o0 = (int)(wunit / nbg) * CB;
        float acc[RB][CB];
        tile_mm<CB>(C, a.tpb,
            [&](int k, float (&x)[RB]) {
#pragma unroll
                for (int r = 0; r < RB; ++r) {
                    const float v = b0 + r < B ? a.s[(long long)(b0 + r) * C + k] : 0.f;
                    x[r] = v * v;
                }
            },
            [&](int k, float (&y)[CB]) {
#pragma unroll
                for (int c = 0; c < CB; ++c) {
                    const float v = o0 + c < O ? a.W1[(long long)(o0 + c) * C + k] : 0.f;
                    y[c] = v * v;
                }
            }, acc, red);
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
            for (int c = 0; c < CB; ++c)
                if (owner0 && lane == r * CB + c && b0 + r < B && o0 + c < O)
                    a.d[(long long)(b0 + r) * O + o0 + c] = rsqrtf(acc[r][c] + a.eps);
    } else if (LAUNCH == 2) {
        if (!second) {            // ds partials: sum_o q[b, o] W1[o, i]^2 over the block's 64-deep o chunk
            const int strips = cdiv_i(C, 64);
            col_sums(O, C, B, blk % strips, blk / strips,
                [&](int b, int k) { return b < B ? q_at(a, b, k) : 0.f; },
                [&](int k, int n) {
                    const float v = a.W1[(long long)k * C + n];
                    return v * v;
                }, a.part, smem);
        } else {                  // dW1 [O, C] = 2 W1 (Q^T S^2): outer tiles over the batch
            float* xs = smem;
            float* ys = smem + OT_B * OT_R;
            const int tn = (C + OT_C - 1) / OT_C;
            const int o0 = (blk / tn) * OT_R, i0 = (blk % tn) * OT_C;
            const bool vec = (C % 4) == 0;
            float acc[4][4], rsm[4];
            outer_tile(B,
                [&](int b, int rr) {
                    float v[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) v[j] = (b < B && o0 + rr + j < O) ? q_at(a, b, o0 + rr + j) : 0.f;
                    return make_float4(v[0], v[1], v[2], v[3]);
                },
                [&](int b, int c) {
                    float4 v = b < B ? load4(a.s, C, b, B, i0 + c, C, vec) : make_float4(0.f, 0.f, 0.f, 0.f);
                    return make_float4(v.x * v.x, v.y * v.y, v.z * v.z, v.w * v.w);
                }, acc, rsm, xs, ys);
            const int ty = t >> 5, tx = t & 31;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int o = o0 + 4 * ty + i, c = i0 + 4 * tx;
                const float4 wv = load4(a.W1, C, o, O, c, C, vec);
                store4(a.dW1, C, o, O, c, C, vec,
                       make_float4(2.f * wv.x * acc[i][0], 2.f * wv.y * acc[i][1], 2.f * wv.z * acc[i][2],
                                   2.f * wv.w * acc[i][3]));
            }
        }
    } else if (LAUNCH == 3) {
        if (!second) {            // dA [3C, WD] = wg dm^T w, dab [3C] = bg sum_b dm: outer tiles over the batch
            float* xs = smem;
            float* ys = smem + OT_B * OT_R;
            const int tn = (WD + OT_C - 1) / OT_C;
            const int j0 = (blk / tn) * OT_R, k0 = (blk % tn) * OT_C;
            const bool vec = (WD % 4) == 0 && (a.ldw % 4) == 0 && (reinterpret_cast<uintptr_t>(a.w) % 16) == 0;
            float acc[4][4], rsm[4];
            outer_tile(B,
                [&](int b, int rr) {
                    float v[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) v[j] = (b < B && j0 + rr + j < C3) ? dm_at(a, b, j0 + rr + j) : 0.f;
                    return make_float4(v[0], v[1], v[2], v[3]);
                },
                [&](int b, int c) { return b < B ? load4(a.w, a.ldw, b, B, k0 + c, WD, vec) : make_float4(0.f, 0.f, 0.f, 0.f); },
                acc, rsm, xs, ys);
            const int ty = t >> 5, tx = t & 31;
            const bool dvec = (WD % 4) == 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int j = j0 + 4 * ty + i;
                if (a.dA)
                    store4(a.dA, WD, j, C3, k0 + 4 * tx, WD, dvec,
                           make_float4(a.wg * acc[i][0], a.wg * acc[i][1], a.wg * acc[i][2], a.wg * acc[i][3]));
                if (a.dab && k0 == 0 && tx == 0 && j < C3) a.dab[j] = a.bg * rsm[i];
            }
        } else {                  // dw partials: sum_j dm[b, j] A[j, n] over the block's 64-deep j chunk
            const int strips = cdiv_i(WD, 64);
            col_sums(C3, WD, B, blk % strips, blk / strips,
                [&](int b, int k) { return b < B ? dm_at(a, b, k) : 0.f; },
                [&](int k, int n) { return a.A[(long long)k * WD + n]; }, a.part, smem);
        }
    } else if (LAUNCH == 4) {     // ds = ds_in + 2 s sum_ks part (fixed order)
        const long long i = (long long)bid * THREADS + t;
        if (i >= (long long)B * C) return;
        const float acc = sum_parts(a.part + i, (long long)B * C, a.ks);
        a.ds[i] = (a.dsin ? a.dsin[i] : 0.f) + 2.f * a.s[i] * acc;
    } else {                      // dw = wg sum_ks part (fixed order)
        const long long i = (long long)bid * THREADS + t;
        if (i >= (long long)B * WD) return;
        const float acc = sum_parts(a.part + i, (long long)B * WD, a.ks);
        const long long b = i / WD, n = i - b * WD;
        a.dw[b * a.lddw + n] = a.wg * acc;
    }
}

template <int LAUNCH>
__global__ __launch_bounds__(THREADS) void style_kernel(StyleArgs a) {
    __shared__ __attribute__((aligned(16))) float smem[OT_B * OT_R + OT_B * OT_C];
    style_body<LAUNCH>(a, blockIdx.x, smem);
}

// The same launch over a group of layers (every ConvNeXt layer of the synthesis network in one launch): the
// layer table tab[n] and the block offsets off[n + 1] (layer l owns blocks off[l] .. off[l + 1] - 1).
template <int LAUNCH>
__global__ __launch_bounds__(THREADS) void style_group_kernel(const StyleArgs* __restrict__ tab,
                                                              const int* __restrict__ off, int n) {
    __shared__ __attribute__((aligned(16))) float smem[OT_B * OT_R + OT_B * OT_C];
    int l = 0;
    while (l + 1 < n && (int)blockIdx.x >= off[l + 1]) ++l;
    const StyleArgs a = tab[l];
    style_body<LAUNCH>(a, (int)blockIdx.x - off[l], smem);
}

template <int L>
int launch(StyleArgs& a, long long blocks, hipStream_t st) {
    if (blocks <= 0) return 0;
    if (blocks > 0x7fffffffLL) return VFM_ERR_ARGS;
    VFM_LAUNCH(style_kernel<L>, dim3((unsigned)blocks), dim3(THREADS), 0, st, a);
    return launch_status();
}

bool sizes_ok(int B, int C, int WD, int O) {
    return B > 0 && C > 0 && WD > 0 && O >= 0 && (long long)B * 3 * C < (1LL << 31) &&
           (long long)O * C < (1LL << 31) && (long long)3 * C * WD < (1LL << 31);
}

// tiles per block of a forward tile job with a reduction of length K: the whole block on one tile from
// K >= 1024 on
inline int tiles_per_block(int K) { return K >= 1024 ? 1 : WAVES; }

// K chunks of the backward's column sums and the floats of their partials
inline int ks_ds(int O) { return cdiv_i(O, KCH); }
inline int ks_dw(int C) { return cdiv_i(3LL * C, KCH); }
inline long long part_floats(int B, int C, int WD, int O) {
    const long long pds = O > 0 ? (long long)ks_ds(O) * B * C : 0, pdw = (long long)ks_dw(C) * B * WD;
    return pds > pdw ? pds : pdw;
}

}  // namespace

// m [B, 3C], s [B, C] and (W1 given) d [B, O] of the layer's style path (see the header).
extern "C" int vfm_style_demod_fwd(const float* w, long long ldw, const float* A, const float* ab, const float* W1,
                                   float wg, float bg, float eps, int B, int C, int WD, int O, float* m, float* s,
                                   float* d, void* stream) {
    if (!w || !A || !ab || !m || !s || !sizes_ok(B, C, WD, O) || ldw < WD) return VFM_ERR_ARGS;
    if (W1 && (!d || O <= 0)) return VFM_ERR_ARGS;
    StyleArgs a{};
    a.w = w; a.ldw = ldw; a.A = A; a.ab = ab; a.W1 = W1; a.wg = wg; a.bg = bg; a.eps = eps;
    a.B = B; a.C = C; a.WD = WD; a.O = O; a.m = m; a.s = s; a.d = d;
    hipStream_t st = (hipStream_t)stream;
    const long long nbg = cdiv_i(B, RB);
    a.tpb = tiles_per_block(WD);
    a.blocks0 = cdiv_i(nbg * cdiv_i(C, 4), a.tpb);
    int rc = launch<0>(a, a.blocks0, st);
    if (rc || !W1) return rc;
    a.tpb = tiles_per_block(C);
    a.blocks0 = cdiv_i(nbg * cdiv_i(O, 8), a.tpb);
    return launch<1>(a, a.blocks0, st);
}

// Workspace floats of vfm_style_demod_bwd: ds [B, C] and the column-sum partials.
extern "C" int vfm_style_demod_bwd_workspace_floats(int B, int C, int WD, int O) {
    if (!sizes_ok(B, C, WD, O)) return -1;
    const long long n = (long long)B * C + part_floats(B, C, WD, O);
    return n > 0x7fffffffLL ? -1 : (int)n;
}

// Gradients of the style path from ds_in = dL/ds (or null) and dd = dL/dd (null without demodulation):
// dw [B, WD], dA [3C, WD], dab [3C], dW1 [O, C], each optional (null: not computed). ws: workspace of
// vfm_style_demod_bwd_workspace_floats floats (required).
extern "C" int vfm_style_demod_bwd(const float* w, long long ldw, const float* A, const float* W1, const float* m,
                                   const float* s, const float* d, const float* ds_in, const float* dd, float wg,
                                   float bg, int B, int C, int WD, int O, float* ws, float* dW1, float* dA,
                                   float* dab, float* dw, void* stream) {
    if (!w || !A || !m || !s || !ws || !sizes_ok(B, C, WD, O) || ldw < WD) return VFM_ERR_ARGS;
    const bool demod = dd != nullptr;
    if (demod && (!W1 || !d || O <= 0)) return VFM_ERR_ARGS;
    if (!demod && (dW1 || !ds_in)) return VFM_ERR_ARGS;
    StyleArgs a{};
    a.w = w; a.ldw = ldw; a.A = A; a.W1 = W1; a.wg = wg; a.bg = bg;
    a.B = B; a.C = C; a.WD = WD; a.O = O; a.m = const_cast<float*>(m); a.s = const_cast<float*>(s);
    a.d = const_cast<float*>(d); a.dsin = ds_in; a.dd = dd; a.ds = ws; a.part = ws + (long long)B * C;
    a.dW1 = dW1; a.dA = dA; a.dab = dab; a.dw = dw; a.lddw = WD;
    hipStream_t st = (hipStream_t)stream;
    if (demod) {
        a.ks = ks_ds(O);
        a.blocks0 = cdiv_i(C, 64) * a.ks;
        const long long b1 = dW1 ? (long long)cdiv_i(O, OT_R) * cdiv_i(C, OT_C) : 0;
        int rc = launch<2>(a, a.blocks0 + b1, st);
        if (rc) return rc;
        a.blocks0 = 0;
        rc = launch<4>(a, cdiv_i((long long)B * C, THREADS), st);
        if (rc) return rc;
        a.dsv = a.ds;
    } else {
        a.dsv = ds_in;
    }
    if (!dA && !dab && !dw) return 0;
    a.ks = ks_dw(C);
    a.blocks0 = (dA || dab) ? cdiv_i(3LL * C, OT_R) * cdiv_i(WD, OT_C) : 0;
    const long long b1 = dw ? (long long)cdiv_i(WD, 64) * a.ks : 0;
    int rc = launch<3>(a, a.blocks0 + b1, st);
    if (rc || !dw) return rc;
    a.blocks0 = 0;
    return launch<5>(a, cdiv_i((long long)B * WD, THREADS), st);
}

// ---------------------------------------------------------------------------------------------------------------
// Grouped form: one launch per phase of the style path for all layers of a network (torch_utils/ops/style_group.py).
// The host packs each launch's layer table + block offsets (vfm_style_group_pack, host memory only), uploads the
// packed bytes, and launches vfm_style_group_launch with the device copy.
namespace {
constexpr int GP = 16;           // per-layer pointer slots of the pack call
}

// Bytes of one packed launch section for n layers (table + offsets, 16-B multiple).
extern "C" long long vfm_style_group_bytes(int n) {
    if (n <= 0) return -1;
    const long long b = (long long)n * sizeof(StyleArgs) + (long long)(n + 1) * 4;
    return (b + 15) / 16 * 16;
}

// Pack launch `launch` (0, 1: forward m / s, d; 2, 4, 3, 5: backward, in that order) for n layers into host_out
// (vfm_style_group_bytes(n) bytes). Per layer l: ptrs[GP l ..] = w, A, ab, W1, m, s, d, ds_in, dd, ws (workspace of
// vfm_style_demod_bwd_workspace_floats), dW1, dA, dab, dw, ldw, lddw (null / 0 where absent, as the single-layer
// entry points take them); dims[4 l ..] = B, C, WD, O; gains[3 l ..] = wg, bg, eps. Layers with nothing to do in
// this launch, or whose w slot is null (left out), get no blocks. Returns the launch's total blocks (0: nothing to launch) or an error code < 0.
extern "C" long long vfm_style_group_pack(int launch, int n, const long long* ptrs, const int* dims, const float* gains,
                                          void* host_out) {
    if (n <= 0 || !ptrs || !dims || !gains || !host_out) return VFM_ERR_ARGS;
    StyleArgs* tab = reinterpret_cast<StyleArgs*>(host_out);
    int* off = reinterpret_cast<int*>(reinterpret_cast<char*>(host_out) + (size_t)n * sizeof(StyleArgs));
    long long total = 0;
    for (int l = 0; l < n; ++l) {
        const long long* p = ptrs + (long long)GP * l;
        if (!p[0]) {                 // a layer left out of this call (no gradient reached it): no blocks
            tab[l] = StyleArgs{};
            off[l] = (int)total;
            continue;
        }
        const int B = dims[4 * l], C = dims[4 * l + 1], WD = dims[4 * l + 2], O = dims[4 * l + 3];
        if (!sizes_ok(B, C, WD, O) || !p[0] || !p[1] || !p[4] || !p[5]) return VFM_ERR_ARGS;
        StyleArgs a{};
        a.w = (const float*)p[0]; a.A = (const float*)p[1]; a.ab = (const float*)p[2]; a.W1 = (const float*)p[3];
        a.m = (float*)p[4]; a.s = (float*)p[5]; a.d = (float*)p[6];
        a.dsin = (const float*)p[7]; a.dd = (const float*)p[8];
        float* ws = (float*)p[9];
        a.dW1 = (float*)p[10]; a.dA = (float*)p[11]; a.dab = (float*)p[12]; a.dw = (float*)p[13];
        a.ldw = p[14]; a.lddw = p[15];
        a.wg = gains[3 * l]; a.bg = gains[3 * l + 1]; a.eps = gains[3 * l + 2];
        a.B = B; a.C = C; a.WD = WD; a.O = O;
        if (a.ldw < WD) return VFM_ERR_ARGS;
        const long long nbg = cdiv_i(B, RB);
        const bool demod = a.dd != nullptr;
        long long blocks = 0;
        if (launch == 0) {
            a.tpb = tiles_per_block(WD);
            a.blocks0 = cdiv_i(nbg * cdiv_i(C, 4), a.tpb);
            blocks = a.blocks0;
        } else if (launch == 1) {
            if (a.W1) {
                if (!a.d || O <= 0) return VFM_ERR_ARGS;
                a.tpb = tiles_per_block(C);
                a.blocks0 = cdiv_i(nbg * cdiv_i(O, 8), a.tpb);
                blocks = a.blocks0;
            }
        } else if (launch == 2 || launch == 4 || launch == 3 || launch == 5) {
            if (demod && (!a.W1 || !a.d || O <= 0 || !ws)) return VFM_ERR_ARGS;
            if (!demod && a.dW1) return VFM_ERR_ARGS;
            a.ds = ws;
            a.part = ws ? ws + (long long)B * C : nullptr;
            a.dsv = demod ? a.ds : a.dsin;
            const bool any_out = demod || a.dsin;
            if (launch == 2 && demod) {
                a.ks = ks_ds(O);
                a.blocks0 = cdiv_i(C, 64) * a.ks;
                blocks = a.blocks0 + (a.dW1 ? (long long)cdiv_i(O, OT_R) * cdiv_i(C, OT_C) : 0);
            } else if (launch == 4 && demod) {
                a.ks = ks_ds(O);                 // the partials launch 2 wrote
                a.blocks0 = 0;
                blocks = cdiv_i((long long)B * C, THREADS);
            } else if (launch == 3 && any_out && (a.dA || a.dab || a.dw)) {
                if (!ws) return VFM_ERR_ARGS;
                a.ks = ks_dw(C);
                a.blocks0 = (a.dA || a.dab) ? cdiv_i(3LL * C, OT_R) * cdiv_i(WD, OT_C) : 0;
                blocks = a.blocks0 + (a.dw ? (long long)cdiv_i(WD, 64) * a.ks : 0);
            } else if (launch == 5 && any_out && a.dw) {
                a.ks = ks_dw(C);
                a.blocks0 = 0;
                blocks = cdiv_i((long long)B * WD, THREADS);
            }
        } else {
            return VFM_ERR_ARGS;
        }
        tab[l] = a;
        off[l] = (int)total;
        total += blocks;
        if (total > 0x7fffffffLL) return VFM_ERR_ARGS;
    }
    off[n] = (int)total;
    return total;
}

// Launch a packed section (device copy `dev_packed` of vfm_style_group_pack's output for the same launch / n).
extern "C" int vfm_style_group_launch(int launch, const void* dev_packed, int n, long long total_blocks, void* stream) {
    if (!dev_packed || n <= 0 || total_blocks < 0 || total_blocks > 0x7fffffffLL) return VFM_ERR_ARGS;
    if (total_blocks == 0) return 0;
    const StyleArgs* tab = reinterpret_cast<const StyleArgs*>(dev_packed);
    const int* off = reinterpret_cast<const int*>(reinterpret_cast<const char*>(dev_packed) + (size_t)n * sizeof(StyleArgs));
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)total_blocks), block(THREADS);
    switch (launch) {
    case 0: VFM_LAUNCH(style_group_kernel<0>, grid, block, 0, st, tab, off, n); break;
    case 1: VFM_LAUNCH(style_group_kernel<1>, grid, block, 0, st, tab, off, n); break;
    case 2: VFM_LAUNCH(style_group_kernel<2>, grid, block, 0, st, tab, off, n); break;
    case 3: VFM_LAUNCH(style_group_kernel<3>, grid, block, 0, st, tab, off, n); break;
    case 4: VFM_LAUNCH(style_group_kernel<4>, grid, block, 0, st, tab, off, n); break;
    case 5: VFM_LAUNCH(style_group_kernel<5>, grid, block, 0, st, tab, off, n); break;
    default: return VFM_ERR_ARGS;
    }
    return launch_status();
}
