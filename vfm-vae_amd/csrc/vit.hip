// Row kernels of the frozen ViT towers (SigLIP2 encoder) for gfx950.
//
// Reference: HF SiglipEncoderLayer under bf16 autocast, as called by
// networks/utils/vfms/siglip2_utils.py:114-137: the fp32 residual stream h is normalised by
// LayerNorm (fp32 statistics) and handed to the bf16 GEMMs, and every sub-block output is
// added back to h in fp32. Unfused, torch runs LayerNorm (fp32 out) + a cast kernel, and a
// cast + add for every residual; here one pass per row does
//     h' = h + delta            (optional; delta in the GEMM dtype, h' written in fp32)
//     y  = LN(h') * w + b       (written directly in the GEMM dtype)
// so each residual/LN pair moves 4+2 bytes in and 4+2 bytes out per element.
//
// One wave per row, D = 256 * NCH (NCH float4 chunks per lane kept in registers: exact
// two-pass mean / variance, no re-read).
#include "vfm_common.h"

namespace {

using namespace vfm;

struct LnArgs {
    const float* h;       // [rows, D] fp32
    const void* delta;    // [rows, D] (dtype_delta) or null
    float* h_out;         // [rows, D] fp32 or null (h + delta)
    const float* w;       // [D] or null
    const float* b;       // [D] or null
    void* y;              // [rows, D] dtype_out
    int rows, D;
    float eps;
};

template <class T>
__device__ __forceinline__ void ld4v(const T* p, float* v) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = ld(p + i);
}
template <>
__device__ __forceinline__ void ld4v<__hip_bfloat16>(const __hip_bfloat16* p, float* v) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(u.x << 16);
    v[1] = __uint_as_float(u.x & 0xffff0000u);
    v[2] = __uint_as_float(u.y << 16);
    v[3] = __uint_as_float(u.y & 0xffff0000u);
}
template <>
__device__ __forceinline__ void ld4v<float>(const float* p, float* v) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}
template <class T>
__device__ __forceinline__ void st4v(T* p, const float* v) {
    T t[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) st(&t[i], v[i]);
    *reinterpret_cast<uint2*>(p) = *reinterpret_cast<const uint2*>(t);
}
template <>
__device__ __forceinline__ void st4v<float>(float* p, const float* v) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

template <class TD, class TO, int NCH>
__global__ __launch_bounds__(256) void ln_rows(LnArgs a) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= a.rows) return;
    const int lane = threadIdx.x & 63;
    const long long off = (long long)row * a.D;
    float v[NCH][4];
#pragma unroll
    for (int j = 0; j < NCH; ++j) ld4v(a.h + off + (j * 64 + lane) * 4, v[j]);
    if (a.delta) {
        const TD* dp = reinterpret_cast<const TD*>(a.delta) + off;
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
            float d[4];
            ld4v(dp + (j * 64 + lane) * 4, d);
#pragma unroll
            for (int i = 0; i < 4; ++i) v[j][i] += d[i];
        }
        if (a.h_out) {
#pragma unroll
            for (int j = 0; j < NCH; ++j) st4v(a.h_out + off + (j * 64 + lane) * 4, v[j]);
        }
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NCH; ++j) s += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
    const float mean = wsum(s) / (float)a.D;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < NCH; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float d = v[j][i] - mean;
            q = fmaf(d, d, q);
        }
    const float rstd = rsqrtf(wsum(q) / (float)a.D + a.eps);
    TO* yp = reinterpret_cast<TO*>(a.y) + off;
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
        const int c0 = (j * 64 + lane) * 4;
        // affine parameters as 16-B loads (c0 is a multiple of 4; host: D % 256 == 0)
        const float4 wv = a.w ? *reinterpret_cast<const float4*>(a.w + c0) : make_float4(1.f, 1.f, 1.f, 1.f);
        const float4 bv = a.b ? *reinterpret_cast<const float4*>(a.b + c0) : make_float4(0.f, 0.f, 0.f, 0.f);
        float o[4];
        o[0] = fmaf((v[j][0] - mean) * rstd, wv.x, bv.x);
        o[1] = fmaf((v[j][1] - mean) * rstd, wv.y, bv.y);
        o[2] = fmaf((v[j][2] - mean) * rstd, wv.z, bv.z);
        o[3] = fmaf((v[j][3] - mean) * rstd, wv.w, bv.w);
        st4v(yp + c0, o);
    }
}

template <class TD, class TO>
int ln_dispatch(LnArgs& a, hipStream_t st) {
    const dim3 grid((unsigned)((a.rows + 3) / 4)), blk(256);
    switch (a.D / 256) {
    case 1: VFM_LAUNCH((ln_rows<TD, TO, 1>), grid, blk, 0, st, a); break;
    case 2: VFM_LAUNCH((ln_rows<TD, TO, 2>), grid, blk, 0, st, a); break;
    case 3: VFM_LAUNCH((ln_rows<TD, TO, 3>), grid, blk, 0, st, a); break;
    case 4: VFM_LAUNCH((ln_rows<TD, TO, 4>), grid, blk, 0, st, a); break;
    case 5: VFM_LAUNCH((ln_rows<TD, TO, 5>), grid, blk, 0, st, a); break;
    case 6: VFM_LAUNCH((ln_rows<TD, TO, 6>), grid, blk, 0, st, a); break;
    case 8: VFM_LAUNCH((ln_rows<TD, TO, 8>), grid, blk, 0, st, a); break;
    default: return VFM_NO_KERNEL;
    }
    return launch_status();
}

// ---- LayerNorm with autograd (the DINOv2 discriminator backbone: frozen parameters, gradient to the input;
// reference HF Dinov2Layer norm1 / norm2 through networks/discriminator.py's DINO feature network) --------
// One wave per row, D = 128 NV (NV float2 per lane: D = 384 for ViT-S, which the float4 form above does not
// take). Forward: exact two-pass mean / variance from registers, y in the compute dtype, mean / rstd saved.
// Backward (dx only): g = dy w, dx = rstd (g - mean(g) - xhat mean(g xhat)).
template <class TO, int NV>
__global__ __launch_bounds__(256) void ln2_fwd(const float* __restrict__ x, const float* __restrict__ w,
                                               const float* __restrict__ b, TO* __restrict__ y, float* mean_out,
                                               float* rstd_out, int rows, int D, float eps) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int lane = threadIdx.x & 63;
    const long long off = (long long)row * D;
    float v[NV][2];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const float2 t = *reinterpret_cast<const float2*>(x + off + (j * 64 + lane) * 2);
        v[j][0] = t.x; v[j][1] = t.y;
    }
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) s += v[j][0] + v[j][1];
    const float mean = wsum(s) / (float)D;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const float d0 = v[j][0] - mean, d1 = v[j][1] - mean;
        q = fmaf(d0, d0, fmaf(d1, d1, q));
    }
    const float rstd = rsqrtf(wsum(q) / (float)D + eps);
    if (lane == 0) {
        mean_out[row] = mean;
        rstd_out[row] = rstd;
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int c0 = (j * 64 + lane) * 2;
        const float2 wv = w ? *reinterpret_cast<const float2*>(w + c0) : make_float2(1.f, 1.f);
        const float2 bv = b ? *reinterpret_cast<const float2*>(b + c0) : make_float2(0.f, 0.f);
        const float o0 = fmaf((v[j][0] - mean) * rstd, wv.x, bv.x);
        const float o1 = fmaf((v[j][1] - mean) * rstd, wv.y, bv.y);
        if constexpr (sizeof(TO) == 4) {
            *reinterpret_cast<float2*>(y + off + c0) = make_float2(o0, o1);
        } else {
            TO t[2];
            st(&t[0], o0);
            st(&t[1], o1);
            *reinterpret_cast<uint32_t*>(y + off + c0) = *reinterpret_cast<const uint32_t*>(t);
        }
    }
}

template <class TG, int NV>
__global__ __launch_bounds__(256) void ln2_bwd(const float* __restrict__ x, const TG* __restrict__ dy,
                                               const float* __restrict__ w, const float* __restrict__ mean_in,
                                               const float* __restrict__ rstd_in, float* __restrict__ dx, int rows,
                                               int D) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const int lane = threadIdx.x & 63;
    const long long off = (long long)row * D;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[NV][2], g[NV][2];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int c0 = (j * 64 + lane) * 2;
        const float2 t = *reinterpret_cast<const float2*>(x + off + c0);
        const float2 wv = w ? *reinterpret_cast<const float2*>(w + c0) : make_float2(1.f, 1.f);
        float d0, d1;
        if constexpr (sizeof(TG) == 4) {
            const float2 u = *reinterpret_cast<const float2*>(dy + off + c0);
            d0 = u.x; d1 = u.y;
        } else {
            d0 = ld(dy + off + c0);
            d1 = ld(dy + off + c0 + 1);
        }
        xh[j][0] = (t.x - mean) * rstd;
        xh[j][1] = (t.y - mean) * rstd;
        g[j][0] = d0 * wv.x;
        g[j][1] = d1 * wv.y;
        sg += g[j][0] + g[j][1];
        sgx = fmaf(g[j][0], xh[j][0], fmaf(g[j][1], xh[j][1], sgx));
    }
    const float mg = wsum(sg) / (float)D, mgx = wsum(sgx) / (float)D;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int c0 = (j * 64 + lane) * 2;
        *reinterpret_cast<float2*>(dx + off + c0) =
            make_float2(rstd * (g[j][0] - mg - xh[j][0] * mgx), rstd * (g[j][1] - mg - xh[j][1] * mgx));
    }
}

#define LN2_NV(M)                                                   \
    switch (D / 128) {                                              \
    case 1: M(1) break;                                             \
    case 2: M(2) break;                                             \
    case 3: M(3) break;                                             \
    case 4: M(4) break;                                             \
    case 5: M(5) break;                                             \
    case 6: M(6) break;                                             \
    case 7: M(7) break;                                             \
    case 8: M(8) break;                                             \
    default: return VFM_NO_KERNEL;                                  \
    }

template <class TO>
int ln2_fwd_launch(const float* x, const float* w, const float* b, void* y, float* mean, float* rstd, int rows,
                   int D, float eps, hipStream_t st) {
    const dim3 grid((unsigned)((rows + 3) / 4)), blk(256);
#define LN2F(NV) VFM_LAUNCH((ln2_fwd<TO, NV>), grid, blk, 0, st, x, w, b, (TO*)y, mean, rstd, rows, D, eps);
    LN2_NV(LN2F)
#undef LN2F
    return launch_status();
}

template <class TG>
int ln2_bwd_launch(const float* x, const void* dy, const float* w, const float* mean, const float* rstd, float* dx,
                   int rows, int D, hipStream_t st) {
    const dim3 grid((unsigned)((rows + 3) / 4)), blk(256);
#define LN2B(NV) VFM_LAUNCH((ln2_bwd<TG, NV>), grid, blk, 0, st, x, (const TG*)dy, w, mean, rstd, dx, rows, D);
    LN2_NV(LN2B)
#undef LN2B
    return launch_status();
}

}  // namespace

extern "C" int vfm_layer_norm_fwd(const float* x, const float* w, const float* b, void* y, float* mean, float* rstd,
                                  int dtype_out, int rows, int D, float eps, void* stream) {
    if (!x || !y || !mean || !rstd || rows < 0 || D <= 0) return VFM_ERR_ARGS;
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(w) |
         reinterpret_cast<uintptr_t>(b)) % 8)
        return VFM_ERR_ARGS;
    if (D % 128 || D > 1024) return VFM_NO_KERNEL;
    if (rows == 0) return VFM_OK;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (dtype_out == VFM_F32) return ln2_fwd_launch<float>(x, w, b, y, mean, rstd, rows, D, eps, st);
    if (dtype_out == VFM_BF16) return ln2_fwd_launch<__hip_bfloat16>(x, w, b, y, mean, rstd, rows, D, eps, st);
    if (dtype_out == VFM_F16) return ln2_fwd_launch<__half>(x, w, b, y, mean, rstd, rows, D, eps, st);
    return VFM_ERR_ARGS;
}

extern "C" int vfm_layer_norm_bwd(const float* x, const void* dy, const float* w, const float* mean,
                                  const float* rstd, float* dx, int dtype_dy, int rows, int D, void* stream) {
    if (!x || !dy || !mean || !rstd || !dx || rows < 0 || D <= 0) return VFM_ERR_ARGS;
    if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dx) | reinterpret_cast<uintptr_t>(w)) % 8)
        return VFM_ERR_ARGS;
    if (D % 128 || D > 1024) return VFM_NO_KERNEL;
    if (rows == 0) return VFM_OK;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (dtype_dy == VFM_F32) return ln2_bwd_launch<float>(x, dy, w, mean, rstd, dx, rows, D, st);
    if (dtype_dy == VFM_BF16) return ln2_bwd_launch<__hip_bfloat16>(x, dy, w, mean, rstd, dx, rows, D, st);
    if (dtype_dy == VFM_F16) return ln2_bwd_launch<__half>(x, dy, w, mean, rstd, dx, rows, D, st);
    return VFM_ERR_ARGS;
}

extern "C" int vfm_residual_layer_norm(const float* h, const void* delta, float* h_out, const float* w,
                                       const float* b, void* y, int dtype_delta, int dtype_out, int rows, int D,
                                       float eps, void* stream) {
    if (!h || !y || rows < 0 || D <= 0) return VFM_ERR_ARGS;
    if ((reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(b)) % 16) return VFM_ERR_ARGS;   // 16-B vector loads
    if (D % 256 || D > 2048) return VFM_NO_KERNEL;
    if (rows == 0) return VFM_OK;
    LnArgs a{h, delta, h_out, w, b, y, rows, D, eps};
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define LN_OUT(TD)                                                            \
    if (dtype_out == VFM_F32) return ln_dispatch<TD, float>(a, st);           \
    if (dtype_out == VFM_BF16) return ln_dispatch<TD, __hip_bfloat16>(a, st); \
    if (dtype_out == VFM_F16) return ln_dispatch<TD, __half>(a, st);
    if (!delta || dtype_delta == VFM_F32) { LN_OUT(float) }
    else if (dtype_delta == VFM_BF16) { LN_OUT(__hip_bfloat16) }
    else if (dtype_delta == VFM_F16) { LN_OUT(__half) }
#undef LN_OUT
    return VFM_ERR_ARGS;
}
