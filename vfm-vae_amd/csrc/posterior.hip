// Diagonal Gaussian posterior of the continuous latent: reparameterised sample and KL to N(0, I) in
// one pass (reference networks/utils/kl_utils.py:30-56, DiagonalGaussianDistribution: chunk the
// moments into mean / logvar, clamp logvar to [-30, 20], std = exp(logvar / 2), sample = mean +
// std * eps, kl = 0.5 * sum_{c,h,w}(mean^2 + exp(logvar) - 1 - logvar)), and its backward.
//
//   forward   z[b, c, p] = m + exp(lv / 2) e,   kl[b] = 0.5 sum (m^2 + exp(lv) - 1 - lv)
//   backward  dm  = dz + dkl[b] m
//             dlv = [-30 <= lv_raw <= 20] (dz e exp(lv / 2) / 2 + dkl[b] (exp(lv) - 1) / 2)
// params fp32 [B, 2C, P] (mean channels first), eps / z / dz fp32 [B, C, P]. One block per sample for
// the forward (the KL is a per-sample sum: fixed-order block reduction, deterministic); the backward
// is elementwise. The tensors are a few MB: the point is one launch instead of the ~12 elementwise
// and reduction kernels of the torch formulation.
#include "vfm_common.h"

namespace {

using namespace vfm;

// torch.clamp semantics: NaN passes through (fminf / fmaxf alone would turn it into -30 and hide a
// diverging encoder behind a finite z and KL)
__device__ __forceinline__ float clamp_lv(float v) { return v != v ? v : fminf(fmaxf(v, -30.f), 20.f); }

__global__ __launch_bounds__(256) void posterior_fwd(const float* __restrict__ params, const float* __restrict__ eps,
                                                     float* __restrict__ z, float* __restrict__ kl, int C, long long P) {
    __shared__ float red[256];
    const int b = blockIdx.x;
    const long long n = (long long)C * P;
    const float* mb = params + (long long)b * 2 * n;
    const float* lb = mb + n;
    float acc = 0.f;
    for (long long i = threadIdx.x; i < n; i += 256) {
        const float m = mb[i], lv = clamp_lv(lb[i]);
        const float var = expf(lv);
        if (z) z[(long long)b * n + i] = fmaf(expf(0.5f * lv), eps ? eps[(long long)b * n + i] : 0.f, m);
        acc += fmaf(m, m, var - 1.f - lv);
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0 && kl) kl[b] = 0.5f * red[0];
}

__global__ __launch_bounds__(256) void posterior_bwd(const float* __restrict__ params, const float* __restrict__ eps,
                                                     const float* __restrict__ dz, const float* __restrict__ dkl,
                                                     float* __restrict__ dparams, int C, long long P, long long total) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    const long long n = (long long)C * P;
    const long long b = i / n, r = i - b * n;
    const float m = params[b * 2 * n + r], raw = params[b * 2 * n + n + r];
    const float lv = clamp_lv(raw);
    const float g = dz ? dz[i] : 0.f, k = dkl ? dkl[b] : 0.f;
    const float e = eps ? eps[i] : 0.f;
    dparams[b * 2 * n + r] = fmaf(k, m, g);
    const float dlv = 0.5f * (g * e * expf(0.5f * lv) + k * (expf(lv) - 1.f));
    dparams[b * 2 * n + n + r] = (raw >= -30.f && raw <= 20.f) ? dlv : 0.f;
}

}  // namespace

extern "C" int vfm_posterior_fwd(const float* params, const float* eps, float* z, float* kl, int B, int C, long long P,
                                 void* stream) {
    if (!params || B <= 0 || B > 0x7fffffff || C <= 0 || P <= 0 || (!z && !kl)) return VFM_ERR_ARGS;
    VFM_LAUNCH(posterior_fwd, dim3(B), dim3(256), 0, (hipStream_t)stream, params, eps, z, kl, C, P);
    return launch_status();
}

extern "C" int vfm_posterior_bwd(const float* params, const float* eps, const float* dz, const float* dkl,
                                 float* dparams, int B, int C, long long P, void* stream) {
    if (!params || !dparams || B <= 0 || C <= 0 || P <= 0) return VFM_ERR_ARGS;
    const long long total = (long long)B * C * P;
    const long long blocks = (total + 255) / 256;
    if (blocks > 0x7fffffffLL) return VFM_ERR_ARGS;
    VFM_LAUNCH(posterior_bwd, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, params, eps, dz, dkl,
                       dparams, C, P, total);
    return launch_status();
}
