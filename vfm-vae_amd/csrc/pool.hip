// 2x2 / stride-2 max pooling of the LPIPS VGG16 stack on NHWC fp32 activations, forward and a fused
// backward. Reference: training/lpips.py:126-163 (torchvision vgg16().features: nn.MaxPool2d(2, 2)
// after relu1_2 / relu2_2 / relu3_3 / relu4_3) and the autograd chain through it, which in torch is
// max_pool2d_with_indices (int64 indices written), its scatter backward, the tap gradient's add and
// the ReLU derivative of the conv below (`g * (y > 0)`): five passes over full-resolution tensors.
//
//   forward:  out[b, i, j, c] = max over the 2x2 window of x (torch's rule: a value replaces the
//             running max when it is strictly greater or NaN, scanning rows then columns from -inf)
//   backward: dx[b, h, w, c] = ((h, w) is the window's argmax ? g[b, h/2, w/2, c] : 0
//                               + gt[b, h, w, c]) * (x[b, h, w, c] > 0 ? 1 : 0)
//             with the argmax recomputed from x (the pool input = the ReLU output of the conv below,
//             saved for the backward anyway) under the same rule, so no indices are stored. Same
//             operations and roundings as the torch chain (the scatter and the mask are exact, the
//             add is one fp32 rounding): bit-identical.
//
// One thread per window and 4 channels (16-B loads / stores along C). HBM-bound: forward reads x once
// and writes a quarter of it; backward reads x, gt and g once and writes dx once.
#include "vfm_common.h"

namespace {

using namespace vfm;

constexpr int PL_NT = 256;

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float comp(const float4& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }

// window element index (0..3, row-major) of the max of v[0..3] under torch's rule
__device__ __forceinline__ int argmax4(float v0, float v1, float v2, float v3, float& m) {
    m = -__builtin_inff();
    int a = 0;
    const float v[4] = {v0, v1, v2, v3};
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (v[k] > m || __builtin_isnan(v[k])) { m = v[k]; a = k; }
    return a;
}

__global__ __launch_bounds__(PL_NT) void maxpool_fwd(const float* __restrict__ x, float* __restrict__ y, int H, int W,
                                                     int C, long long total) {
    const long long t = (long long)blockIdx.x * PL_NT + threadIdx.x;
    if (t >= total) return;
    const int C4 = C >> 2, Wo = W >> 1, Ho = H >> 1;
    const int c = (int)(t % C4) * 4;
    long long r = t / C4;
    const int j = (int)(r % Wo);
    r /= Wo;
    const int i = (int)(r % Ho);
    const long long b = r / Ho;
    const float* p = x + ((b * H + 2 * i) * W + 2 * j) * C + c;
    const float4 a0 = ld4(p), a1 = ld4(p + C), a2 = ld4(p + (long long)W * C), a3 = ld4(p + (long long)W * C + C);
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) argmax4(comp(a0, k), comp(a1, k), comp(a2, k), comp(a3, k), o[k]);
    st4(y + t * 4, make_float4(o[0], o[1], o[2], o[3]));
}

__global__ __launch_bounds__(PL_NT) void maxpool_bwd(const float* __restrict__ g, const float* __restrict__ x,
                                                     const float* __restrict__ gt, float* __restrict__ dx, int H, int W,
                                                     int C, long long total) {
    const long long t = (long long)blockIdx.x * PL_NT + threadIdx.x;
    if (t >= total) return;
    const int C4 = C >> 2, Wo = W >> 1, Ho = H >> 1;
    const int c = (int)(t % C4) * 4;
    long long r = t / C4;
    const int j = (int)(r % Wo);
    r /= Wo;
    const int i = (int)(r % Ho);
    const long long b = r / Ho;
    const long long o0 = ((b * H + 2 * i) * W + 2 * j) * C + c;
    const long long off[4] = {o0, o0 + C, o0 + (long long)W * C, o0 + (long long)W * C + C};
    float4 xv[4], tv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) xv[q] = ld4(x + off[q]);
    if (gt) {
#pragma unroll
        for (int q = 0; q < 4; ++q) tv[q] = ld4(gt + off[q]);
    }
    const float4 gv = ld4(g + t * 4);
    float out[4][4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float m;
        const int a = argmax4(comp(xv[0], k), comp(xv[1], k), comp(xv[2], k), comp(xv[3], k), m);
        const float gk = comp(gv, k);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float v = q == a ? 0.f + gk : 0.f;       // torch scatters into zeros: 0 + g
            if (gt) v = v + comp(tv[q], k);
            out[q][k] = v * (comp(xv[q], k) > 0.f ? 1.f : 0.f);
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) st4(dx + off[q], make_float4(out[q][0], out[q][1], out[q][2], out[q][3]));
}

bool pool_ok(const void* a, const void* b, int B, int H, int W, int C) {
    return a && b && B > 0 && H > 1 && W > 1 && C > 0 && (C & 3) == 0 && !(H & 1) && !(W & 1) &&
           ((uintptr_t)a % 16) == 0 && ((uintptr_t)b % 16) == 0;
}

}  // namespace

using vfm::launch_status;

extern "C" int vfm_maxpool2x2_nhwc_f32(const float* x, float* y, int B, int H, int W, int C, void* stream) {
    if (!x || !y || B <= 0 || H <= 0 || W <= 0 || C <= 0) return VFM_ERR_ARGS;
    if (!pool_ok(x, y, B, H, W, C)) return VFM_NO_KERNEL;
    const long long total = (long long)B * (H / 2) * (W / 2) * (C / 4);
    VFM_LAUNCH(maxpool_fwd, dim3((unsigned)((total + PL_NT - 1) / PL_NT)), dim3(PL_NT), 0, (hipStream_t)stream, x, y,
               H, W, C, total);
    return launch_status();
}

extern "C" int vfm_maxpool2x2_bwd_nhwc_f32(const float* g, const float* x, const float* gt, float* dx, int B, int H,
                                           int W, int C, void* stream) {
    if (!g || !x || !dx || B <= 0 || H <= 0 || W <= 0 || C <= 0) return VFM_ERR_ARGS;
    if (!pool_ok(x, dx, B, H, W, C) || ((uintptr_t)g % 16) || ((uintptr_t)gt % 16)) return VFM_NO_KERNEL;
    const long long total = (long long)B * (H / 2) * (W / 2) * (C / 4);
    VFM_LAUNCH(maxpool_bwd, dim3((unsigned)((total + PL_NT - 1) / PL_NT)), dim3(PL_NT), 0, (hipStream_t)stream, g, x,
               gt, dx, H, W, C, total);
    return launch_status();
}
