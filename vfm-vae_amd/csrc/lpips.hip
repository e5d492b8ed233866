// LPIPS distance head for gfx950 — the per-tap tail of LPIPS.forward:
//     r[b,p] = sum_c w_c * ( f0[b,c,p] / (|f0[b,:,p]| + eps) - f1[b,c,p] / (|f1[b,:,p]| + eps) )^2
// Reference: training/lpips.py (LPIPS.forward: `normalize_tensor(outs0[kk]) -
// normalize_tensor(outs1[kk])`, `** 2`, `lin{kk}` = 1x1 conv C->1 without bias,
// `spatial_average`; normalize_tensor = x / (sqrt(sum_c x^2) + 1e-10)). In torch this is ~8
// full-size fp32 passes per feature map forward and more backward; here forward reads f0 and
// f1 twice (norms, then differences) and writes one float per pixel, backward reads them twice
// and writes the gradient(s).
//
// Layout: fp32 NCHW features (the VGG16 taps), one lane per pixel, lanes along the contiguous
// pixel axis so every channel step is a coalesced 256-byte wave access; channel loops unrolled
// by 8 to keep 16 loads in flight per lane. HBM-bound (algorithmic bytes: forward
// 2 * 2 * B*C*HW*4 re-read + B*HW*12 written; backward 2 * 2 * B*C*HW*4 + grads).
//
// Backward, with G_c = gs_b * 2 w_c (a_c - u_c), a = f0/n0e, u = f1/n1e, n = sqrt(sum x^2),
// ne = n + eps:   dL/df1_k = -G_k / n1e + f1_k * (sum_c G_c f1_c) / (n1e^2 * n1)
//                 dL/df0_k = +G_k / n0e - f0_k * (sum_c G_c f0_c) / (n0e^2 * n0)
// At n == 0 (an all-zero pixel) the second term is taken as 0 (torch's autograd gives NaN there).
#include "vfm_common.h"

namespace {

constexpr int LP_NT = 256;
constexpr float LP_EPS = 1e-10f;

__global__ __launch_bounds__(LP_NT) void lpips_head_fwd(const float* __restrict__ f0, const float* __restrict__ f1,
                                                        const float* __restrict__ w, float* __restrict__ r,
                                                        float* __restrict__ n0s, float* __restrict__ n1s, int C,
                                                        long long HW, long long total) {
    const long long i = (long long)blockIdx.x * LP_NT + threadIdx.x;
    if (i >= total) return;
    const long long b = i / HW, p = i - b * HW;
    const float* a = f0 + b * (long long)C * HW + p;
    const float* u = f1 + b * (long long)C * HW + p;
    float s0 = 0.f, s1 = 0.f;
    int c = 0;
    for (; c + 8 <= C; c += 8) {
        float x[8], y[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { x[j] = a[(c + j) * HW]; y[j] = u[(c + j) * HW]; }
#pragma unroll
        for (int j = 0; j < 8; ++j) { s0 += x[j] * x[j]; s1 += y[j] * y[j]; }
    }
    for (; c < C; ++c) { const float x = a[c * HW], y = u[c * HW]; s0 += x * x; s1 += y * y; }
    const float n0 = sqrtf(s0), n1 = sqrtf(s1);
    const float n0e = n0 + LP_EPS, n1e = n1 + LP_EPS;
    float acc = 0.f;
    c = 0;
    for (; c + 8 <= C; c += 8) {
        float x[8], y[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { x[j] = a[(c + j) * HW]; y[j] = u[(c + j) * HW]; }
#pragma unroll
        for (int j = 0; j < 8; ++j) { const float d = x[j] / n0e - y[j] / n1e; acc += w[c + j] * (d * d); }
    }
    for (; c < C; ++c) { const float d = a[c * HW] / n0e - u[c * HW] / n1e; acc += w[c] * (d * d); }
    r[i] = acc;
    n0s[i] = n0;
    n1s[i] = n1;
}

// gs: per-sample upstream gradient of every r[b, :] (dL/dmean / HW). g0/g1 may be null.
__global__ __launch_bounds__(LP_NT) void lpips_head_bwd(const float* __restrict__ f0, const float* __restrict__ f1,
                                                        const float* __restrict__ w, const float* __restrict__ n0s,
                                                        const float* __restrict__ n1s, const float* __restrict__ gs,
                                                        float* __restrict__ g0, float* __restrict__ g1, int C,
                                                        long long HW, long long total) {
    const long long i = (long long)blockIdx.x * LP_NT + threadIdx.x;
    if (i >= total) return;
    const long long b = i / HW, p = i - b * HW;
    const long long off = b * (long long)C * HW + p;
    const float* a = f0 + off;
    const float* u = f1 + off;
    const float n0 = n0s[i], n1 = n1s[i];
    const float n0e = n0 + LP_EPS, n1e = n1 + LP_EPS;
    const float s2 = 2.f * gs[b];
    float dot0 = 0.f, dot1 = 0.f;
    int c = 0;
    for (; c + 8 <= C; c += 8) {                       // 16 loads in flight per lane
        float x[8], y[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { x[j] = a[(c + j) * HW]; y[j] = u[(c + j) * HW]; }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float G = s2 * w[c + j] * (x[j] / n0e - y[j] / n1e);
            dot0 += G * x[j];
            dot1 += G * y[j];
        }
    }
    for (; c < C; ++c) {
        const float x = a[c * HW], y = u[c * HW];
        const float G = s2 * w[c] * (x / n0e - y / n1e);
        dot0 += G * x;
        dot1 += G * y;
    }
    const float k0 = n0 > 0.f ? dot0 / (n0e * n0e * n0) : 0.f;
    const float k1 = n1 > 0.f ? dot1 / (n1e * n1e * n1) : 0.f;
    c = 0;
    for (; c + 8 <= C; c += 8) {
        float x[8], y[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) { x[j] = a[(c + j) * HW]; y[j] = u[(c + j) * HW]; }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float G = s2 * w[c + j] * (x[j] / n0e - y[j] / n1e);
            if (g0) g0[off + (c + j) * HW] = G / n0e - x[j] * k0;
            if (g1) g1[off + (c + j) * HW] = -G / n1e + y[j] * k1;
        }
    }
    for (; c < C; ++c) {
        const float x = a[c * HW], y = u[c * HW];
        const float G = s2 * w[c] * (x / n0e - y / n1e);
        if (g0) g0[off + c * HW] = G / n0e - x * k0;
        if (g1) g1[off + c * HW] = -G / n1e + y * k1;
    }
}

int grid_of(long long total) { return (int)((total + LP_NT - 1) / LP_NT); }

// ---------------------------------------------------------------------------------------------
// NHWC (channels_last) features, as the HIP VGG16 stack produces them (torch_utils/ops/vgg_hip.py):
// 16 lanes per pixel, lane j holds channels 4j + 64i (i < CH = C/64) as float4 -- each pixel's
// channel vector is read once, coalesced, and kept in registers for the second pass; the
// channel sums are 16-lane xor-shuffle reductions. Same arithmetic as the NCHW kernels above.
template <int CH>
__device__ __forceinline__ void lp_load(const float* p, int j, float4* v) {
#pragma unroll
    for (int i = 0; i < CH; ++i) v[i] = *reinterpret_cast<const float4*>(p + 64 * i + 4 * j);
}
__device__ __forceinline__ float lp_sum16(float s) {
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1) s += __shfl_xor(s, m, 16);
    return s;
}
__device__ __forceinline__ float dot4(float4 a, float4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }

template <int CH>
__global__ __launch_bounds__(LP_NT) void lpips_head_fwd_nhwc(const float* __restrict__ f0, const float* __restrict__ f1,
                                                             const float* __restrict__ w, float* __restrict__ r,
                                                             float* __restrict__ n0s, float* __restrict__ n1s,
                                                             long long total) {
    constexpr int C = 64 * CH;
    const long long pix = (long long)blockIdx.x * (LP_NT / 16) + threadIdx.x / 16;
    const int j = threadIdx.x & 15;
    if (pix >= total) return;                          // uniform over the pixel's 16 lanes
    float4 x[CH], y[CH];
    lp_load<CH>(f0 + pix * C, j, x);
    lp_load<CH>(f1 + pix * C, j, y);
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int i = 0; i < CH; ++i) { s0 += dot4(x[i], x[i]); s1 += dot4(y[i], y[i]); }
    s0 = lp_sum16(s0);
    s1 = lp_sum16(s1);
    const float n0 = sqrtf(s0), n1 = sqrtf(s1);
    const float n0e = n0 + LP_EPS, n1e = n1 + LP_EPS;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
        const float4 wv = *reinterpret_cast<const float4*>(w + 64 * i + 4 * j);
        const float d0 = x[i].x / n0e - y[i].x / n1e, d1 = x[i].y / n0e - y[i].y / n1e;
        const float d2 = x[i].z / n0e - y[i].z / n1e, d3 = x[i].w / n0e - y[i].w / n1e;
        acc += wv.x * (d0 * d0) + wv.y * (d1 * d1) + wv.z * (d2 * d2) + wv.w * (d3 * d3);
    }
    acc = lp_sum16(acc);
    if (j == 0) {
        r[pix] = acc;
        n0s[pix] = n0;
        n1s[pix] = n1;
    }
}

template <int CH>
__global__ __launch_bounds__(LP_NT) void lpips_head_bwd_nhwc(const float* __restrict__ f0, const float* __restrict__ f1,
                                                             const float* __restrict__ w, const float* __restrict__ n0s,
                                                             const float* __restrict__ n1s, const float* __restrict__ gs,
                                                             float* __restrict__ g0, float* __restrict__ g1, long long HW,
                                                             long long total) {
    constexpr int C = 64 * CH;
    const long long pix = (long long)blockIdx.x * (LP_NT / 16) + threadIdx.x / 16;
    const int j = threadIdx.x & 15;
    if (pix >= total) return;
    float4 x[CH], y[CH], G[CH];
    lp_load<CH>(f0 + pix * C, j, x);
    lp_load<CH>(f1 + pix * C, j, y);
    const float n0 = n0s[pix], n1 = n1s[pix];
    const float n0e = n0 + LP_EPS, n1e = n1 + LP_EPS;
    const float s2 = 2.f * gs[pix / HW];
    float dot0 = 0.f, dot1 = 0.f;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
        const float4 wv = *reinterpret_cast<const float4*>(w + 64 * i + 4 * j);
        G[i].x = s2 * wv.x * (x[i].x / n0e - y[i].x / n1e);
        G[i].y = s2 * wv.y * (x[i].y / n0e - y[i].y / n1e);
        G[i].z = s2 * wv.z * (x[i].z / n0e - y[i].z / n1e);
        G[i].w = s2 * wv.w * (x[i].w / n0e - y[i].w / n1e);
        dot0 += dot4(G[i], x[i]);
        dot1 += dot4(G[i], y[i]);
    }
    dot0 = lp_sum16(dot0);
    dot1 = lp_sum16(dot1);
    const float k0 = n0 > 0.f ? dot0 / (n0e * n0e * n0) : 0.f;
    const float k1 = n1 > 0.f ? dot1 / (n1e * n1e * n1) : 0.f;
#pragma unroll
    for (int i = 0; i < CH; ++i) {
        const long long o = pix * C + 64 * i + 4 * j;
        if (g0)
            *reinterpret_cast<float4*>(g0 + o) = make_float4(G[i].x / n0e - x[i].x * k0, G[i].y / n0e - x[i].y * k0,
                                                             G[i].z / n0e - x[i].z * k0, G[i].w / n0e - x[i].w * k0);
        if (g1)
            *reinterpret_cast<float4*>(g1 + o) = make_float4(-G[i].x / n1e + y[i].x * k1, -G[i].y / n1e + y[i].y * k1,
                                                             -G[i].z / n1e + y[i].z * k1, -G[i].w / n1e + y[i].w * k1);
    }
}

int nhwc_grid(long long pixels) { return (int)((pixels + LP_NT / 16 - 1) / (LP_NT / 16)); }

}  // namespace

extern "C" int vfm_lpips_head_fwd(const float* f0, const float* f1, const float* w, float* r, float* n0, float* n1,
                                  int B, int C, long long HW, void* stream) {
    if (B < 0 || C <= 0 || HW < 0) return VFM_ERR_ARGS;
    const long long total = (long long)B * HW;
    if (total == 0) return VFM_OK;
    if (!f0 || !f1 || !w || !r || !n0 || !n1) return VFM_ERR_ARGS;
    if (grid_of(total) <= 0 || (long long)C * HW * B > (1ll << 40)) return VFM_ERR_ARGS;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    VFM_LAUNCH(lpips_head_fwd, dim3(grid_of(total)), dim3(LP_NT), 0, st, f0, f1, w, r, n0, n1, C, HW, total);
    return (int)hipGetLastError();
}

extern "C" int vfm_lpips_head_bwd(const float* f0, const float* f1, const float* w, const float* n0, const float* n1,
                                  const float* gs, float* g0, float* g1, int B, int C, long long HW, void* stream) {
    if (B < 0 || C <= 0 || HW < 0) return VFM_ERR_ARGS;
    const long long total = (long long)B * HW;
    if (total == 0 || (!g0 && !g1)) return VFM_OK;
    if (!f0 || !f1 || !w || !n0 || !n1 || !gs) return VFM_ERR_ARGS;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    VFM_LAUNCH(lpips_head_bwd, dim3(grid_of(total)), dim3(LP_NT), 0, st, f0, f1, w, n0, n1, gs, g0, g1, C, HW,
                       total);
    return (int)hipGetLastError();
}

extern "C" int vfm_lpips_head_fwd_nhwc(const float* f0, const float* f1, const float* w, float* r, float* n0, float* n1,
                                       int B, int C, long long HW, void* stream) {
    if (B < 0 || HW < 0) return VFM_ERR_ARGS;
    if (C != 64 && C != 128 && C != 256 && C != 512) return VFM_NO_KERNEL;
    const long long total = (long long)B * HW;
    if (total == 0) return VFM_OK;
    if (!f0 || !f1 || !w || !r || !n0 || !n1 || total > (1ll << 36)) return VFM_ERR_ARGS;
    if (((uintptr_t)f0 | (uintptr_t)f1 | (uintptr_t)w) % 16) return VFM_ERR_ARGS;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const dim3 g(nhwc_grid(total)), b(LP_NT);
    switch (C) {
        case 64: VFM_LAUNCH(lpips_head_fwd_nhwc<1>, g, b, 0, st, f0, f1, w, r, n0, n1, total); break;
        case 128: VFM_LAUNCH(lpips_head_fwd_nhwc<2>, g, b, 0, st, f0, f1, w, r, n0, n1, total); break;
        case 256: VFM_LAUNCH(lpips_head_fwd_nhwc<4>, g, b, 0, st, f0, f1, w, r, n0, n1, total); break;
        default: VFM_LAUNCH(lpips_head_fwd_nhwc<8>, g, b, 0, st, f0, f1, w, r, n0, n1, total); break;
    }
    return (int)hipGetLastError();
}

extern "C" int vfm_lpips_head_bwd_nhwc(const float* f0, const float* f1, const float* w, const float* n0,
                                       const float* n1, const float* gs, float* g0, float* g1, int B, int C, long long HW,
                                       void* stream) {
    if (B < 0 || HW < 0) return VFM_ERR_ARGS;
    if (C != 64 && C != 128 && C != 256 && C != 512) return VFM_NO_KERNEL;
    const long long total = (long long)B * HW;
    if (total == 0 || (!g0 && !g1)) return VFM_OK;
    if (!f0 || !f1 || !w || !n0 || !n1 || !gs || total > (1ll << 36)) return VFM_ERR_ARGS;
    if (((uintptr_t)f0 | (uintptr_t)f1 | (uintptr_t)w | (uintptr_t)g0 | (uintptr_t)g1) % 16) return VFM_ERR_ARGS;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const dim3 g(nhwc_grid(total)), b(LP_NT);
    switch (C) {
        case 64: VFM_LAUNCH(lpips_head_bwd_nhwc<1>, g, b, 0, st, f0, f1, w, n0, n1, gs, g0, g1, HW, total); break;
        case 128: VFM_LAUNCH(lpips_head_bwd_nhwc<2>, g, b, 0, st, f0, f1, w, n0, n1, gs, g0, g1, HW, total); break;
        case 256: VFM_LAUNCH(lpips_head_bwd_nhwc<4>, g, b, 0, st, f0, f1, w, n0, n1, gs, g0, g1, HW, total); break;
        default: VFM_LAUNCH(lpips_head_bwd_nhwc<8>, g, b, 0, st, f0, f1, w, n0, n1, gs, g0, g1, HW, total); break;
    }
    return (int)hipGetLastError();
}
