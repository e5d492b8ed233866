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

}  // namespace

extern "C" int vfm_lpips_head_fwd(const float* f0, const float* f1, const float* w, float* r, float* n0, float* n1,
                                  int B, int C, long long HW, void* stream) {
    if (B < 0 || C <= 0 || HW < 0) return VFM_ERR_ARGS;
    const long long total = (long long)B * HW;
    if (total == 0) return VFM_OK;
    if (!f0 || !f1 || !w || !r || !n0 || !n1) return VFM_ERR_ARGS;
    if (grid_of(total) <= 0 || (long long)C * HW * B > (1ll << 40)) return VFM_ERR_ARGS;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(lpips_head_fwd, dim3(grid_of(total)), dim3(LP_NT), 0, st, f0, f1, w, r, n0, n1, C, HW, total);
    return (int)hipGetLastError();
}

extern "C" int vfm_lpips_head_bwd(const float* f0, const float* f1, const float* w, const float* n0, const float* n1,
                                  const float* gs, float* g0, float* g1, int B, int C, long long HW, void* stream) {
    if (B < 0 || C <= 0 || HW < 0) return VFM_ERR_ARGS;
    const long long total = (long long)B * HW;
    if (total == 0 || (!g0 && !g1)) return VFM_OK;
    if (!f0 || !f1 || !w || !n0 || !n1 || !gs) return VFM_ERR_ARGS;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(lpips_head_bwd, dim3(grid_of(total)), dim3(LP_NT), 0, st, f0, f1, w, n0, n1, gs, g0, g1, C, HW,
                       total);
    return (int)hipGetLastError();
}
