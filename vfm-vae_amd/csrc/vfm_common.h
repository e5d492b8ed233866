// Shared device helpers for the VFM-VAE gfx950 kernels.
//
// Every kernel in this directory computes in fp32 (fp64 for double inputs) and
// stores in the tensor's own dtype, mirroring the `InternalType` promotion of
// the reference plugins (torch_utils/ops/upfirdn2d.cu:16-19, bias_act.cu:16-19).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "../../include/vfmvae.h"

namespace vfm {

template <class T> struct Acc { typedef float type; };
template <> struct Acc<double> { typedef double type; };

__device__ __forceinline__ float ld(const float* p) { return *p; }
__device__ __forceinline__ double ld(const double* p) { return *p; }
__device__ __forceinline__ float ld(const __half* p) { return __half2float(*p); }
__device__ __forceinline__ float ld(const __hip_bfloat16* p) { return __bfloat162float(*p); }

__device__ __forceinline__ void st(float* p, float v) { *p = v; }
__device__ __forceinline__ void st(double* p, double v) { *p = v; }
__device__ __forceinline__ void st(__half* p, float v) { *p = __float2half(v); }
__device__ __forceinline__ void st(__hip_bfloat16* p, float v) { *p = __float2bfloat16(v); }

// floor(a / b) for b > 0 and any sign of a.
__device__ __host__ __forceinline__ int floor_div(int a, int b) {
    int q = a / b;
    return (q * b > a) ? q - 1 : q;
}
// ceil(a / b) for b > 0 and any sign of a.
__device__ __host__ __forceinline__ int ceil_div(int a, int b) { return -floor_div(-a, b); }

// Division by a runtime-invariant divisor via multiply-high (Granlund-Montgomery),
// valid for 0 <= n < 2^31, 1 <= d < 2^31.
struct FastDiv {
    uint32_t d, m, s;
};
static inline FastDiv make_fastdiv(uint32_t d) {
    FastDiv f;
    f.d = d;
    uint32_t s = 0;
    while ((1ull << s) < d) s++;
    f.s = s;
    f.m = (uint32_t)((((1ull << 32) * ((1ull << s) - d)) / d) + 1);
    return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
    uint32_t t = __umulhi(n, f.m);
    return (t + n) >> f.s;
}

struct GeluParts {
    float cdf;    // Phi(z)
    float zpdf;   // z * phi(z)
};
__device__ __forceinline__ GeluParts gelu_parts(float z) {
    const float x = z * 0.70710678118654752f;
    const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, fabsf(x), 1.f));
    float p = fmaf(t, 1.061405429f, -1.453152027f);
    p = fmaf(p, t, 1.421413741f);
    p = fmaf(p, t, -0.284496736f);
    p = fmaf(p, t, 0.254829592f);
    const float e = __builtin_amdgcn_exp2f(-(x * x) * 1.4426950408889634f);   // exp(-z^2/2)
    const float q = 0.5f * (p * t) * e;                                        // 0.5 * erfc(|x|)
    GeluParts r;
    r.cdf = x < 0.f ? q : 1.f - q;
    r.zpdf = z * 0.39894228040143268f * e;
    return r;
}
inline int launch_status() {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? VFM_OK : (int)e;
}

}  // namespace vfm

// Dispatch a templated launcher on the runtime dtype code.
#define VFM_DISPATCH_FLOAT(dtype, T, ...)                                      \
    switch (dtype) {                                                           \
    case VFM_F32: { typedef float T; __VA_ARGS__; break; }                     \
    case VFM_F16: { typedef __half T; __VA_ARGS__; break; }                    \
    case VFM_BF16: { typedef __hip_bfloat16 T; __VA_ARGS__; break; }           \
    case VFM_F64: { typedef double T; __VA_ARGS__; break; }                    \
    default: return VFM_ERR_ARGS;                                              \
    }
