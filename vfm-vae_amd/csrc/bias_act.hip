// bias_act for gfx950: y = clamp(act(x + b) * gain) and its 1st/2nd-order gradients.
//
// Semantics (forward, grad=1, grad=2 formulas, expRange guards, clamp behaviour) follow
// the reference kernel `torch_utils/ops/bias_act.cu:23-147`; the activation table
// follows `torch_utils/ops/bias_act.py:21-31`.
//
// HBM-bound elementwise op: each lane handles 4 consecutive elements per grid-stride
// step (16-B loads for fp32, 8-B for 16-bit), the bias index (i / stepB) % sizeB uses
// multiply-high division so the VALU cost stays below the memory time.
#include "vfm_common.h"

namespace {

using namespace vfm;

constexpr int NT = 256;
constexpr int VEC = 4;

struct BiasActArgs {
    const void *x, *b, *xref, *yref, *dy;
    void* y;
    long long numel;
    int grad, act;
    float alpha, gain, clamp;
    FastDiv stepB, sizeB;
};

template <class A, int ACT, int G>
__device__ __forceinline__ A act_eval(A x, A xref, A& yref, A yy, A alpha, A gain) {
    const A one = (A)1, two = (A)2, expRange = (A)80, halfExpRange = (A)40;
    const A seluScale = (A)1.0507009873554804934193349852946;
    const A seluAlpha = (A)1.6732632423543772848170429916717;
    A y = 0;
    if (ACT == 1) { y = x; }
    if (ACT == 2) { if (G == 0) y = (x > 0) ? x : (A)0; if (G == 1) y = (yy > 0) ? x : (A)0; }
    if (ACT == 3) { if (G == 0) y = (x > 0) ? x : x * alpha; if (G == 1) y = (yy > 0) ? x : x * alpha; }
    if (ACT == 4) {
        if (G == 0) { A c = exp(x); A d = one / c; y = (x < -expRange) ? -one : (x > expRange) ? one : (c - d) / (c + d); }
        if (G == 1) y = x * (one - yy * yy);
        if (G == 2) y = x * (one - yy * yy) * (-two * yy);
    }
    if (ACT == 5) {
        if (G == 0) y = (x < -expRange) ? (A)0 : one / (exp(-x) + one);
        if (G == 1) y = x * yy * (one - yy);
        if (G == 2) y = x * yy * (one - yy) * (one - two * yy);
    }
    if (ACT == 6) {
        if (G == 0) y = (x >= 0) ? x : exp(x) - one;
        if (G == 1) y = (yy >= 0) ? x : x * (yy + one);
        if (G == 2) y = (yy >= 0) ? (A)0 : x * (yy + one);
    }
    if (ACT == 7) {
        if (G == 0) y = (x >= 0) ? seluScale * x : (seluScale * seluAlpha) * (exp(x) - one);
        if (G == 1) y = (yy >= 0) ? x * seluScale : x * (yy + seluScale * seluAlpha);
        if (G == 2) y = (yy >= 0) ? (A)0 : x * (yy + seluScale * seluAlpha);
    }
    if (ACT == 8) {
        if (G == 0) y = (x > expRange) ? x : log(exp(x) + one);
        if (G == 1) y = x * (one - exp(-yy));
        if (G == 2) { A c = exp(-yy); y = x * c * (one - c); }
    }
    if (ACT == 9) {
        if (G == 0) {
            y = (x < -expRange) ? (A)0 : x / (exp(-x) + one);
        } else {
            A c = exp(xref);
            A d = c + one;
            if (G == 1) y = (xref > halfExpRange) ? x : x * c * (xref + d) / (d * d);
            else        y = (xref > halfExpRange) ? (A)0 : x * c * (xref * (two - d) + two * d) / (d * d * d);
            yref = (xref < -expRange) ? (A)0 : xref / (exp(-xref) + one) * gain;
        }
    }
    return y;
}

template <class T, int ACT, int G>
__global__ __launch_bounds__(NT) void bias_act_kernel(BiasActArgs p) {
    typedef typename Acc<T>::type A;
    const T* X = reinterpret_cast<const T*>(p.x);
    const T* B = reinterpret_cast<const T*>(p.b);
    const T* XR = reinterpret_cast<const T*>(p.xref);
    const T* YR = reinterpret_cast<const T*>(p.yref);
    const T* DY = reinterpret_cast<const T*>(p.dy);
    T* Y = reinterpret_cast<T*>(p.y);
    const A alpha = (A)p.alpha, gain = (A)p.gain, clampv = (A)p.clamp;
    const long long stride = (long long)gridDim.x * NT * VEC;
    for (long long base = ((long long)blockIdx.x * NT + threadIdx.x) * VEC; base < p.numel; base += stride) {
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
            const long long i = base + k;
            if (i >= p.numel) break;
            A x = (A)ld(X + i);
            A b = 0;
            if (B) {
                uint32_t q = fdiv((uint32_t)i, p.stepB);
                uint32_t r = q - fdiv(q, p.sizeB) * p.sizeB.d;
                b = (A)ld(B + r);
            }
            A xref = XR ? (A)ld(XR + i) : (A)0;
            A yref = YR ? (A)ld(YR + i) : (A)0;
            A dy = DY ? (A)ld(DY + i) : (A)1;
            A yy = (gain != 0) ? yref / gain : (A)0;
            if (G == 0) x += b; else xref += b;
            A y = act_eval<A, ACT, G>(x, xref, yref, yy, alpha, gain);
            y *= gain * dy;
            if (clampv >= 0) {
                if (G == 0) y = (y > -clampv && y < clampv) ? y : (y >= 0) ? clampv : -clampv;
                else        y = (yref > -clampv && yref < clampv) ? y : (A)0;
            }
            st(Y + i, y);
        }
    }
}

template <class T, int ACT>
int launch_act(BiasActArgs& p, hipStream_t st) {
    long long blocks = (p.numel + (long long)NT * VEC - 1) / ((long long)NT * VEC);
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    dim3 g((unsigned)blocks), b(NT);
    if (p.grad == 0) VFM_LAUNCH((bias_act_kernel<T, ACT, 0>), g, b, 0, st, p);
    else if (p.grad == 1) VFM_LAUNCH((bias_act_kernel<T, ACT, 1>), g, b, 0, st, p);
    else VFM_LAUNCH((bias_act_kernel<T, ACT, 2>), g, b, 0, st, p);
    return launch_status();
}

template <class T>
int run(BiasActArgs& p, hipStream_t st) {
    switch (p.act) {
    case 1: return launch_act<T, 1>(p, st);
    case 2: return launch_act<T, 2>(p, st);
    case 3: return launch_act<T, 3>(p, st);
    case 4: return launch_act<T, 4>(p, st);
    case 5: return launch_act<T, 5>(p, st);
    case 6: return launch_act<T, 6>(p, st);
    case 7: return launch_act<T, 7>(p, st);
    case 8: return launch_act<T, 8>(p, st);
    case 9: return launch_act<T, 9>(p, st);
    default: return VFM_ERR_ARGS;
    }
}

}  // namespace

extern "C" int vfm_bias_act(const void* x, const void* b, const void* xref, const void* yref,
                            const void* dy, void* y, int dtype, long long numel,
                            int grad, int act, float alpha, float gain, float clamp,
                            long long stepB, int sizeB, void* stream) {
    if (!x || !y || numel < 0 || grad < 0 || grad > 2) return VFM_ERR_ARGS;
    if (numel == 0) return VFM_OK;
    if (numel >= (1ll << 31)) return VFM_ERR_ARGS;  // reference: x.numel() <= INT_MAX
    if (b && (stepB <= 0 || sizeB <= 0 || stepB >= (1ll << 31))) return VFM_ERR_ARGS;
    BiasActArgs p;
    p.x = x; p.b = b; p.xref = xref; p.yref = yref; p.dy = dy; p.y = y;
    p.numel = numel; p.grad = grad; p.act = act;
    p.alpha = alpha; p.gain = gain; p.clamp = clamp;
    p.stepB = make_fastdiv(b ? (uint32_t)stepB : 1u);
    p.sizeB = make_fastdiv(b ? (uint32_t)sizeB : 1u);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    VFM_DISPATCH_FLOAT(dtype, T, return run<T>(p, st));
    return VFM_ERR_ARGS;
}
