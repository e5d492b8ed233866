// Modulated 1x1 ToRGB (no demodulation) as one HBM pass per direction
// (reference networks/utils/convnext_utils.py:145-187, ConvNeXtToRGBLayer.forward):
//
//   forward   y[b, o, p]  = r( sum_c wm[b, o, c] x[b, c, p] ) + bias[o],  wm[b, o, c] = w[o, c] s[b, c]
//             (r = rounding to bf16 when x is bf16: the reference's bf16 GEMM output, then the fp32 bias)
//   backward  dx[b, c, p] = sum_o wm[b, o, c] dy[b, o, p]
//             T[b, o, c]  = sum_p x[b, c, p] dy[b, o, p]        (-> dstyle, dw on the host: [B, O, C])
//
// O (image channels) <= 4, so both directions are HBM-bound streams over x: the forward reads x once
// (8 pixels per lane, 16-B loads, a loop over channels split across the block's lanes on small planes), the backward reads
// x and writes dx once (one wave per 4 channels, 8 pixels per lane, 512 contiguous pixels per wave
// step; dy's O rows are re-read per channel group from L2 / MALL) and reduces T per wave in registers,
// one fp32 partial per pixel split (no atomics: fixed order, deterministic).
#include "vfm_common.h"

namespace {

using namespace vfm;

template <class T> struct Vec8;
template <> struct Vec8<float> {
    static __device__ __forceinline__ void load(const float* p, float v[8]) {
        const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    }
    static __device__ __forceinline__ void store(float* p, const float v[8]) {
        *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
    static __device__ __forceinline__ float round(float v) { return v; }
};
template <> struct Vec8<__hip_bfloat16> {
    static __device__ __forceinline__ void load(const __hip_bfloat16* p, float v[8]) {
        const uint4 r = *reinterpret_cast<const uint4*>(p);
        const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            v[2 * i] = __uint_as_float(w[i] << 16);
            v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
        }
    }
    static __device__ __forceinline__ uint32_t bits(float v) {
        return (uint32_t)__builtin_bit_cast(uint16_t, __float2bfloat16(v));
    }
    static __device__ __forceinline__ void store(__hip_bfloat16* p, const float v[8]) {
        *reinterpret_cast<uint4*>(p) = make_uint4(bits(v[0]) | (bits(v[1]) << 16), bits(v[2]) | (bits(v[3]) << 16),
                                                  bits(v[4]) | (bits(v[5]) << 16), bits(v[6]) | (bits(v[7]) << 16));
    }
    static __device__ __forceinline__ float round(float v) { return __bfloat162float(__float2bfloat16(v)); }
};

// block = PL pixel lanes (8 pixels each) x NCS = 256 / PL channel splits; the splits' partial sums
// meet in LDS (small planes: the low-resolution blocks have P / 8 < 256 pixel lanes per sample)
template <class T, int O>
__global__ __launch_bounds__(256) void torgb_fwd(const T* __restrict__ x, const float* __restrict__ wm,
                                                const float* __restrict__ bias, float* __restrict__ y, int C, int P,
                                                int PL) {
    __shared__ float red[256 * O * 8];
    const int b = blockIdx.y, NCS = 256 / PL;
    const int pl = threadIdx.x % PL, cs = threadIdx.x / PL;
    const long long p0 = 8ll * ((long long)blockIdx.x * PL + pl);
    const bool live = p0 < P;
    const T* xb = x + (long long)b * C * P + (live ? p0 : 0);
    const float* w = wm + (long long)b * O * C;
    float acc[O][8];
#pragma unroll
    for (int o = 0; o < O; ++o)
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[o][k] = 0.f;
    if (live) {
#pragma unroll 4
        for (int c = cs; c < C; c += NCS) {
            float v[8];
            Vec8<T>::load(xb + (long long)c * P, v);
#pragma unroll
            for (int o = 0; o < O; ++o) {
                const float wo = w[o * C + c];
#pragma unroll
                for (int k = 0; k < 8; ++k) acc[o][k] = fmaf(wo, v[k], acc[o][k]);
            }
        }
    }
    if (NCS > 1) {
#pragma unroll
        for (int o = 0; o < O; ++o)
#pragma unroll
            for (int k = 0; k < 8; ++k) red[(o * 8 + k) * 256 + threadIdx.x] = acc[o][k];
        __syncthreads();
        if (cs != 0) return;
#pragma unroll
        for (int o = 0; o < O; ++o)
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                float s = 0.f;
                for (int j = 0; j < NCS; ++j) s += red[(o * 8 + k) * 256 + j * PL + pl];   // fixed order
                acc[o][k] = s;
            }
    }
    if (!live) return;
#pragma unroll
    for (int o = 0; o < O; ++o) {
        float r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = Vec8<T>::round(acc[o][k]) + bias[o];
        Vec8<float>::store(y + ((long long)b * O + o) * P + p0, r);
    }
}

// grid (S pixel splits, C / 16 channel groups, B); block 256 = 4 waves x 4 channels
template <class T, int O>
__global__ __launch_bounds__(256) void torgb_bwd(const T* __restrict__ x, const float* __restrict__ dy,
                                                const float* __restrict__ wm, T* __restrict__ dx,
                                                float* __restrict__ tpart, int C, int P, int span) {
    const int s = blockIdx.x, b = blockIdx.z, S = gridDim.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int c0 = blockIdx.y * 16 + wave * 4;
    const float* w = wm + (long long)b * O * C;
    float wv[4][O];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int o = 0; o < O; ++o) wv[j][o] = w[o * C + c0 + j];
    float t[4][O];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int o = 0; o < O; ++o) t[j][o] = 0.f;
    const int pb = s * span, pe = min(P, pb + span);
    const T* xb = x + ((long long)b * C + c0) * P;
    T* dxb = dx + ((long long)b * C + c0) * P;
    const float* dyb = dy + (long long)b * O * P;
    for (int p = pb + 8 * lane; p < pe; p += 512) {
        float g[O][8];
#pragma unroll
        for (int o = 0; o < O; ++o) Vec8<float>::load(dyb + (long long)o * P + p, g[o]);
        float v[4][8];
#pragma unroll
        for (int j = 0; j < 4; ++j) Vec8<T>::load(xb + (long long)j * P + p, v[j]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float d[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                float a = 0.f;
#pragma unroll
                for (int o = 0; o < O; ++o) {
                    a = fmaf(wv[j][o], g[o][k], a);
                    t[j][o] = fmaf(v[j][k], g[o][k], t[j][o]);
                }
                d[k] = a;
            }
            Vec8<T>::store(dxb + (long long)j * P + p, d);
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int o = 0; o < O; ++o) {
            float r = t[j][o];
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) r += __shfl_xor(r, m, 64);
            t[j][o] = r;
        }
    if (lane == 0) {
        float* tp = tpart + ((long long)b * S + s) * O * C;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int o = 0; o < O; ++o) tp[o * C + c0 + j] = t[j][o];
    }
}

template <class T>
int fwd_launch(const void* x, const float* wm, const float* bias, float* y, int B, int O, int C, int P, hipStream_t st) {
    int PL = 8;
    while (PL < 256 && PL < P / 8) PL *= 2;
    dim3 grid((unsigned)((P / 8 + PL - 1) / PL), B);
#define VFM_TF(OO) VFM_LAUNCH((torgb_fwd<T, OO>), grid, dim3(256), 0, st, (const T*)x, wm, bias, y, C, P, PL)
    switch (O) {
    case 1: VFM_TF(1); break;
    case 2: VFM_TF(2); break;
    case 3: VFM_TF(3); break;
    default: VFM_TF(4); break;
    }
#undef VFM_TF
    return launch_status();
}

template <class T>
int bwd_launch(const void* x, const float* dy, const float* wm, void* dx, float* tpart, int B, int O, int C, int P,
               int S, hipStream_t st) {
    const int span = ((P + S - 1) / S + 511) / 512 * 512;
    dim3 grid(S, C / 16, B);
#define VFM_TB(OO) \
    VFM_LAUNCH((torgb_bwd<T, OO>), grid, dim3(256), 0, st, (const T*)x, dy, wm, (T*)dx, tpart, C, P, span)
    switch (O) {
    case 1: VFM_TB(1); break;
    case 2: VFM_TB(2); break;
    case 3: VFM_TB(3); break;
    default: VFM_TB(4); break;
    }
#undef VFM_TB
    return launch_status();
}

}  // namespace

extern "C" int vfm_torgb_fwd(const void* x, const float* wm, const float* bias, float* y, int dtype, int B, int O,
                             int C, int P, void* stream) {
    if (!x || !wm || !bias || !y || B <= 0 || B > 65535 || O < 1 || O > 4 || C <= 0 || P <= 0) return VFM_ERR_ARGS;
    if (P % 8 || ((uintptr_t)x | (uintptr_t)y) % 16) return VFM_NO_KERNEL;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == VFM_F32) return fwd_launch<float>(x, wm, bias, y, B, O, C, P, st);
    if (dtype == VFM_BF16) return fwd_launch<__hip_bfloat16>(x, wm, bias, y, B, O, C, P, st);
    return VFM_NO_KERNEL;
}

// pixel splits S of the backward (tpart holds B * S * O * C floats)
extern "C" int vfm_torgb_bwd_splits(int B, int C, int P) {
    if (B <= 0 || C <= 0 || P <= 0) return -1;
    const long long waves = (long long)B * (C / 4);
    int S = (int)((16384 + waves - 1) / waves);
    const int smax = (P + 511) / 512;
    if (S > smax) S = smax;
    if (S > 65535) S = 65535;
    return S < 1 ? 1 : S;
}

extern "C" int vfm_torgb_bwd(const void* x, const float* dy, const float* wm, void* dx, float* tpart, int dtype, int B,
                             int O, int C, int P, int S, void* stream) {
    if (!x || !dy || !wm || !dx || !tpart || B <= 0 || B > 65535 || O < 1 || O > 4 || C <= 0 || P <= 0 || S < 1)
        return VFM_ERR_ARGS;
    if (P % 8 || C % 16 || C / 16 > 65535 || S > 65535) return VFM_NO_KERNEL;
    if (((uintptr_t)x | (uintptr_t)dy | (uintptr_t)dx) % 16) return VFM_NO_KERNEL;
    hipStream_t st = (hipStream_t)stream;
    if (dtype == VFM_F32) return bwd_launch<float>(x, dy, wm, dx, tpart, B, O, C, P, S, st);
    if (dtype == VFM_BF16) return bwd_launch<__hip_bfloat16>(x, dy, wm, dx, tpart, B, O, C, P, S, st);
    return VFM_NO_KERNEL;
}
