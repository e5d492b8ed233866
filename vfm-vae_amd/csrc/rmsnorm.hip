// Channel RMS norm of the decoder's attention blocks (reference networks/utils/gigagan_utils.py:31-39,
// ChannelRMSNorm: F.normalize(x, dim=1) * sqrt(C) * gamma) on fp32 NCHW planes, forward and backward,
// one launch each (+ one for the gamma-gradient partial sums). torch's formulation is a norm reduction
// over the strided channel dim, a clamp, a division and two scalings (five kernels; its backward about
// ten), and its global-reduce path zeroes semaphores with a memset per call.
//
//   n[b, p]    = max(sqrt(sum_c x[b, c, p]^2), 1e-12)          (p < P = H W)
//   y[b, c, p] = x[b, c, p] / n[b, p] * k[c],   k = scale * gamma
//   dx         = k dy / n - x (sum_c k dy x) / n^3   where the norm is not clamped,   k dy / n  where it is
//   dgamma[c]  = scale * sum_{b, p} dy x / n
//
// Block = 32 columns (consecutive p) x 32 channel groups; a thread sums every 32nd channel of its
// column (1024 threads), the 32 partial sums meet in LDS, then the same threads write their channels. A
// wave's loads are two 128-B rows (32 consecutive fp32 of two channels): whole cache lines, where the
// 16-column form read 64-B halves whose other halves belonged to the neighbouring block (forward at 32^2 x
// 512: 48 -> 30 us, 64^2 x 256: 82 -> 51 us; backward 64^2: 194 -> 128-154 us, profiles/r6_by_crms_tiling.txt).
// The gamma gradient: each block reduces dy x / n over its columns per channel into one partial
// (channel-major [C][blocks]), and a second kernel sums every channel's partials in a fixed order
// (deterministic).
#include "vfm_common.h"

namespace {

using namespace vfm;

#ifndef CRMS_GROUPS
#define CRMS_GROUPS 32
#endif
#ifndef CRMS_COLS
#define CRMS_COLS 32
#endif
constexpr int COLS = CRMS_COLS, GROUPS = CRMS_GROUPS, THREADS = COLS * GROUPS;
constexpr float NORM_EPS = 1e-12f;

__global__ __launch_bounds__(THREADS) void crms_fwd(const float* __restrict__ x, const float* __restrict__ gamma,
                                                    float* __restrict__ y, float* __restrict__ rinv, int C, int P,
                                                    int tiles, float scale) {
    __shared__ float red[GROUPS][COLS + 1];
    const int b = blockIdx.x / tiles, p0 = (blockIdx.x - b * tiles) * COLS;
    const int col = threadIdx.x % COLS, g = threadIdx.x / COLS;
    const int p = p0 + col;
    const bool ok = p < P;
    const float* xb = x + (long long)b * C * P + p;
    float ss = 0.f;
    if (ok)
        // 8 channels per round, their loads issued before the FMAs (one round trip per 8 channels)
        for (int c0 = g; c0 < C; c0 += 8 * GROUPS) {
            float v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int c = c0 + k * GROUPS;
                v[k] = c < C ? xb[(long long)c * P] : 0.f;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) ss = fmaf(v[k], v[k], ss);
        }
    red[g][col] = ss;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < GROUPS; ++i) tot += red[i][col];
    const float r = 1.f / fmaxf(sqrtf(tot), NORM_EPS);
    if (!ok) return;
    if (g == 0 && rinv) rinv[(long long)b * P + p] = r;
    float* yb = y + (long long)b * C * P + p;
#pragma unroll 8
    for (int c = g; c < C; c += GROUPS) yb[(long long)c * P] = xb[(long long)c * P] * r * (scale * gamma[c]);
}

__global__ __launch_bounds__(THREADS) void crms_bwd(const float* __restrict__ x, const float* __restrict__ gamma,
                                                    const float* __restrict__ rinv, const float* __restrict__ dy,
                                                    float* __restrict__ dx, float* __restrict__ gpart, int C, int P,
                                                    int tiles, float scale) {
    __shared__ float red[GROUPS][COLS + 1];
    const int b = blockIdx.x / tiles, p0 = (blockIdx.x - b * tiles) * COLS;
    const int col = threadIdx.x % COLS, g = threadIdx.x / COLS;
    const int p = p0 + col;
    const bool ok = p < P;
    const long long base = (long long)b * C * P + p;
    float dot = 0.f;
    if (ok)
        for (int c0 = g; c0 < C; c0 += 8 * GROUPS) {
            float dv[8], xv[8], gv[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int c = c0 + k * GROUPS;
                const long long o = base + (long long)c * P;
                dv[k] = c < C ? dy[o] : 0.f;
                xv[k] = c < C ? x[o] : 0.f;
                gv[k] = c < C ? gamma[c] : 0.f;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) dot = fmaf(scale * gv[k] * dv[k], xv[k], dot);
        }
    red[g][col] = dot;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < GROUPS; ++i) tot += red[i][col];
    const float r = ok ? rinv[(long long)b * P + p] : 0.f;
    // r == 1 / 1e-12 exactly when the norm was clamped: no gradient through the norm then
    const float corr = (r < 1.f / NORM_EPS) ? tot * r * r * r : 0.f;
    for (int c = g; c < C; c += GROUPS) {
        float gx = 0.f;
        if (ok) {
            const long long o = base + (long long)c * P;
            const float d = dy[o], xv = x[o];
            dx[o] = scale * gamma[c] * d * r - xv * corr;
            gx = d * xv * r;
        }
        if (gpart) {
            // sum over the block's COLS columns: lanes col = 0..COLS-1 of one channel group are COLS consecutive
            // lanes of one wave (COLS divides 64)
            static_assert(COLS <= 64 && 64 % COLS == 0, "a channel group's columns must lie in one wave");
#pragma unroll
            for (int o = COLS / 2; o >= 1; o >>= 1) gx += __shfl_xor(gx, o, COLS);
            if (col == 0) gpart[(long long)c * gridDim.x + blockIdx.x] = gx;     // channel-major: [C][rows]
        }
    }
}

// dgamma[c] = scale * sum_rows gpart[c, row]: one block per channel over its contiguous row partials (one per
// crms_bwd block), every thread's loads in flight before its strided sum, then a fixed-order tree over the
// block (deterministic). Round 3 summed the rows serially per channel (2048 dependent L2 round trips at
// 32 x 32^2 pixels: ~100 us per launch).
__global__ __launch_bounds__(256) void crms_gamma(const float* __restrict__ gpart, float* __restrict__ dgamma, int C,
                                                  int rows, float scale) {
    __shared__ float red[256];
    const int c = blockIdx.x, t = threadIdx.x;
    const float* row = gpart + (long long)c * rows;
    float s = 0.f;
    for (int r0 = 0; r0 < rows; r0 += 256 * 8) {
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int r = r0 + t + 256 * k;
            v[k] = r < rows ? row[r] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) s += v[k];
    }
    red[t] = s;
    __syncthreads();
#pragma unroll
    for (int w = 128; w >= 1; w >>= 1) {
        if (t < w) red[t] += red[t + w];
        __syncthreads();
    }
    if (t == 0) dgamma[c] = scale * red[0];
}

bool crms_grid(int B, int C, int P, int& tiles, long long& blocks) {
    tiles = (P + COLS - 1) / COLS;
    blocks = (long long)B * tiles;
    return B > 0 && C > 0 && P > 0 && blocks <= 0x7fffffffLL;
}

}  // namespace

// rows of the gamma-gradient partial buffer vfm_channel_rms_norm_bwd needs ([rows, C] fp32)
extern "C" long long vfm_channel_rms_norm_rows(int B, int C, int P) {
    int tiles;
    long long blocks;
    if (!crms_grid(B, C, P, tiles, blocks)) return VFM_ERR_ARGS;
    return blocks;
}

// y = x / max(||x||_channels, 1e-12) * scale * gamma on fp32 [B, C, P]; rinv [B, P] (optional) keeps
// 1 / max(norm, 1e-12) for the backward.
extern "C" int vfm_channel_rms_norm_fwd(const float* x, const float* gamma, float* y, float* rinv, int B, int C, int P,
                                        float scale, void* stream) {
    int tiles;
    long long blocks;
    if (!x || !gamma || !y || !crms_grid(B, C, P, tiles, blocks)) return VFM_ERR_ARGS;
    VFM_LAUNCH(crms_fwd, dim3((unsigned)blocks), dim3(THREADS), 0, (hipStream_t)stream, x, gamma, y, rinv, C,
                       P, tiles, scale);
    return vfm::launch_status();
}

// dx (required) and dgamma (optional: then gpart [vfm_channel_rms_norm_rows, C] is its workspace)
extern "C" int vfm_channel_rms_norm_bwd(const float* x, const float* gamma, const float* rinv, const float* dy,
                                        float* dx, float* gpart, float* dgamma, int B, int C, int P, float scale,
                                        void* stream) {
    int tiles;
    long long blocks;
    if (!x || !gamma || !rinv || !dy || !dx || !crms_grid(B, C, P, tiles, blocks)) return VFM_ERR_ARGS;
    if ((gpart == nullptr) != (dgamma == nullptr)) return VFM_ERR_ARGS;
    hipStream_t st = (hipStream_t)stream;
    VFM_LAUNCH(crms_bwd, dim3((unsigned)blocks), dim3(THREADS), 0, st, x, gamma, rinv, dy, dx, gpart, C, P,
                       tiles, scale);
    if (dgamma)
        VFM_LAUNCH(crms_gamma, dim3(C), dim3(256), 0, st, gpart, dgamma, C, (int)blocks, scale);
    return vfm::launch_status();
}
