// Shared device helpers for the VFM-VAE gfx950 kernels.
//
// Every kernel in this directory computes in fp32 (fp64 for double inputs) and
// stores in the tensor's own dtype, mirroring the `InternalType` promotion of
// the reference plugins (torch_utils/ops/upfirdn2d.cu:16-19, bias_act.cu:16-19).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
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

// fp32 pair -> packed bf16 hi pair and packed bf16 lo pair (lo = bf16(x - hi)), element 0 in the
// low half: the 3-term split of the f32x3 products. One v_cvt_pk_bf16_f32 per packed pair and a
// packed subtract, instead of a conversion per element plus shifts / ORs to pack; the roundings
// (RNE) and the subtraction are the same IEEE operations, so the result is bit-identical.
typedef float vfm_f2 __attribute__((ext_vector_type(2)));
typedef __bf16 vfm_bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split2_bf16(float x0, float x1, uint32_t& hi, uint32_t& lo) {
    const vfm_f2 x = {x0, x1};
    hi = __builtin_bit_cast(uint32_t, __builtin_convertvector(x, vfm_bf16x2));
    const vfm_f2 h = {__uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
    lo = __builtin_bit_cast(uint32_t, __builtin_convertvector(x - h, vfm_bf16x2));
}

// fp32 pair -> packed bf16 (hi, mid, lo) with x = hi + mid + lo EXACTLY (each remainder is exact in
// fp32 and the last one has at most 8 significant bits): the operand split of the f32x6 products.
// A product a.b then runs as the six bf16 products of order >= 2^-16 (hi.hi, hi.mid, mid.hi,
// hi.lo, mid.mid, lo.hi), each exact in fp32 (|mid| <= 2^-8 |x|, |lo| <= 2^-16 |x|); the three
// dropped ones (mid.lo, lo.mid, lo.lo) total <= ~2^-23 |a b|, the size of one fp32 rounding.
__device__ __forceinline__ void split3_bf16(float x0, float x1, uint32_t& hi, uint32_t& mid, uint32_t& lo) {
    const vfm_f2 x = {x0, x1};
    hi = __builtin_bit_cast(uint32_t, __builtin_convertvector(x, vfm_bf16x2));
    const vfm_f2 h = {__uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
    const vfm_f2 r1 = x - h;
    mid = __builtin_bit_cast(uint32_t, __builtin_convertvector(r1, vfm_bf16x2));
    const vfm_f2 m = {__uint_as_float(mid << 16), __uint_as_float(mid & 0xffff0000u)};
    lo = __builtin_bit_cast(uint32_t, __builtin_convertvector(r1 - m, vfm_bf16x2));
}

// Split an fp32 pair into NP packed bf16 pieces (NP = 2: hi, lo; NP = 3: hi, mid, lo).
template <int NP>
__device__ __forceinline__ void split_pieces(float x0, float x1, uint32_t* p) {
    if (NP == 3) split3_bf16(x0, x1, p[0], p[1], p[2]);
    else split2_bf16(x0, x1, p[0], p[1]);
}

// Product terms of the fp32 emulation over NP pieces per operand, smallest first (fp32
// accumulation): NP = 2 ("f32x3"): lo.hi, hi.lo, hi.hi; NP = 3 ("f32x6"): lo.hi, hi.lo, mid.mid,
// mid.hi, hi.mid, hi.hi. Piece index of operand A / B for term t.
template <int NP> struct Terms;
template <> struct Terms<1> {
    static constexpr int N = 1;
    __device__ __host__ static constexpr int a(int) { return 0; }
    __device__ __host__ static constexpr int b(int) { return 0; }
};
template <> struct Terms<2> {
    static constexpr int N = 3;
    __device__ __host__ static constexpr int a(int t) { return t == 0 ? 1 : 0; }
    __device__ __host__ static constexpr int b(int t) { return t == 1 ? 1 : 0; }
};
template <> struct Terms<3> {
    static constexpr int N = 6;
    __device__ __host__ static constexpr int a(int t) { return t == 0 ? 2 : (t == 2 || t == 3) ? 1 : 0; }
    __device__ __host__ static constexpr int b(int t) { return t == 1 ? 2 : (t == 2 || t == 4) ? 1 : 0; }
};

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
// Kernel timing for bench.py's roofline object (vfm_timer_arm, version.hip): while a pair of events
// is armed, every launch goes through hipExtLaunchKernelGGL, which binds the events to the kernel
// dispatch itself: `start` to the first launch's start, `stop` to the end of each launch (the last
// one wins). The elapsed time is the kernels' own duration, not host launch gaps around them.
struct TimerArm {
    hipEvent_t start = nullptr, stop = nullptr;
    int launches = 0;
    bool first_only = false;   // vfm_timer_arm_first: only the region's first launch is timed (a GEMM's main
                               // kernel without its split-K combine pass, which is a kernel of its own)
};
TimerArm& timer_arm();
// Probe mode (vfm_timer_mode(1), the default): the start event is bound to the END of an empty one-wave probe
// kernel launched right before the timed kernel, not to the timed kernel's own start: a dispatch-bound start
// event reads from the moment the command processor takes the packet, i.e. it includes the tail of the
// previous kernel the timed one waits behind (+10-50 % on the decoder's short kernels against rocprofv3's
// kernel trace, gpurun_out r6p). The probe ends when the previous kernel has drained, so the interval is the
// timed kernel's own execution plus one dispatch gap.
extern int g_timer_mode;
__global__ void timer_probe_kernel(int);

// Per-device launch state (a process may drive several GPUs): the current device's index, its CU count, and
// (at the call sites) one "dynamic LDS attribute set" flag per device for each kernel instantiation.
constexpr int MAXDEV = 64;
inline int cur_dev() {
    int d = 0;
    (void)hipGetDevice(&d);
    return (d < 0 || d >= MAXDEV) ? 0 : d;
}
inline int device_cus(int d) {
    static int cus[MAXDEV] = {};
    if (!cus[d]) {
        int c = 0;
        (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, d);
        cus[d] = c > 0 ? c : 256;
    }
    return cus[d];
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

// Every kernel launch of the library (see TimerArm).
#define VFM_LAUNCH(kern, grid, block, shm, stream, ...)                                                     \
    do {                                                                                                    \
        ::vfm::TimerArm& vfm_ta_ = ::vfm::timer_arm();                                                      \
        if (vfm_ta_.stop) {                                                                                 \
            if (vfm_ta_.start && ::vfm::g_timer_mode == 1) {                                                \
                hipExtLaunchKernelGGL(::vfm::timer_probe_kernel, dim3(1), dim3(64), 0, stream, nullptr,     \
                                      vfm_ta_.start, 0, 0);                                                 \
                vfm_ta_.start = nullptr;                                                                    \
            }                                                                                               \
            hipExtLaunchKernelGGL(kern, grid, block, shm, stream, vfm_ta_.start, vfm_ta_.stop, 0, __VA_ARGS__); \
            vfm_ta_.start = nullptr;                                                                        \
            ++vfm_ta_.launches;                                                                             \
            if (vfm_ta_.first_only) vfm_ta_.stop = nullptr;                                                 \
        } else {                                                                                            \
            hipLaunchKernelGGL(kern, grid, block, shm, stream, __VA_ARGS__);                               \
        }                                                                                                   \
    } while (0)
