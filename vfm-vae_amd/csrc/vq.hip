// Codebook lookup of the discrete latent for gfx950:
//     idx[n] = argmax_v < f_n / max(|f_n|, eps), w_v / max(|w_v|, eps) >
// Reference: networks/utils/quant_utils.py:84-86 (VectorQuantizer.forward: F.normalize both
// sides, fp32 `features @ codebook.T`, torch.argmax) and :126-131 (f_to_idx).
//
// The indices are integers, so the target is bit-exactness. Every floating-point step has a
// fixed order, the one torch's fp32 CPU path uses (measured: F.normalize sums the rounded
// squares left to right; the [N,4]x[4,V] GEMM is a left-to-right FMA chain): squares summed
// left to right without contraction, correctly rounded sqrt and division, the dot product as
// d = f0*w0, d = fma(f_i, w_i, d). oracle/ops_oracle.c restates it operation for operation.
// Ties resolve to the first (lowest) index and NaN counts as the maximum, as torch.argmax.
//
// Work shape (config 4: 8 codebooks of 4096 x 4, B*256 tokens each): one lane per token, the
// normalised codebook staged through LDS in chunks (every lane reads the same code ->
// LDS broadcast), 64-lane workgroups so a 8192-token codebook fills 128 workgroups.
#include "vfm_common.h"

namespace {

constexpr int VQ_NT = 64;
constexpr int VQ_LDS_FLOATS = 8192;   // 32 KiB of normalised codes per chunk

#pragma clang fp contract(off)

template <int C>
__device__ __forceinline__ void vq_normalize(const float* x, float* o) {
    float s = x[0] * x[0];
#pragma unroll
    for (int i = 1; i < C; ++i) s = s + x[i] * x[i];
    float n = sqrtf(s);
    n = n < 1e-12f ? 1e-12f : n;          // clamp_min (NaN propagates)
#pragma unroll
    for (int i = 0; i < C; ++i) o[i] = x[i] / n;
}

template <int C>
__global__ __launch_bounds__(VQ_NT) void codebook_argmax_kernel(const float* __restrict__ f, long long ldf,
                                                                const float* __restrict__ w, int N, int V,
                                                                long long* __restrict__ idx) {
    __shared__ __attribute__((aligned(16))) float sw[VQ_LDS_FLOATS];
    constexpr int CH = VQ_LDS_FLOATS / C;
    const int t = blockIdx.x * VQ_NT + threadIdx.x;
    const bool live = t < N;
    float fn[C];
    {
        float fx[C];
#pragma unroll
        for (int i = 0; i < C; ++i) fx[i] = live ? f[(long long)t * ldf + i] : 0.f;
        vq_normalize<C>(fx, fn);
    }
    float best = -INFINITY;
    bool best_nan = false;
    int bi = 0;
    for (int v0 = 0; v0 < V; v0 += CH) {
        const int n = min(CH, V - v0);
        __syncthreads();
        for (int j = threadIdx.x; j < n; j += VQ_NT) {
            float wx[C];
#pragma unroll
            for (int i = 0; i < C; ++i) wx[i] = w[(long long)(v0 + j) * C + i];
            vq_normalize<C>(wx, sw + j * C);
        }
        __syncthreads();
        if (live && !best_nan) {
            for (int j = 0; j < n; ++j) {
                const float* cw = sw + j * C;
                float d = fn[0] * cw[0];
#pragma unroll
                for (int i = 1; i < C; ++i) d = __builtin_fmaf(fn[i], cw[i], d);
                if (d > best) {
                    best = d;
                    bi = v0 + j;
                } else if (d != d) {             // first NaN wins and stays
                    bi = v0 + j;
                    best_nan = true;
                    break;
                }
            }
        }
    }
    if (live) idx[t] = bi;
}

template <int C>
int vq_launch(const float* f, long long ldf, const float* w, int N, int V, long long* idx, hipStream_t st) {
    const dim3 grid((unsigned)((N + VQ_NT - 1) / VQ_NT));
    VFM_LAUNCH((codebook_argmax_kernel<C>), grid, dim3(VQ_NT), 0, st, f, ldf, w, N, V, idx);
    return vfm::launch_status();
}

}  // namespace

extern "C" int vfm_codebook_argmax(const float* features, long long ld, const float* codebook, int N, int C, int V,
                                   long long* indices, void* stream) {
    if (N < 0 || V <= 0 || C <= 0 || ld < C) return VFM_ERR_ARGS;
    if (N == 0) return VFM_OK;
    if (!features || !codebook || !indices) return VFM_ERR_ARGS;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    switch (C) {
    case 1: return vq_launch<1>(features, ld, codebook, N, V, indices, st);
    case 2: return vq_launch<2>(features, ld, codebook, N, V, indices, st);
    case 3: return vq_launch<3>(features, ld, codebook, N, V, indices, st);
    case 4: return vq_launch<4>(features, ld, codebook, N, V, indices, st);
    case 8: return vq_launch<8>(features, ld, codebook, N, V, indices, st);
    case 16: return vq_launch<16>(features, ld, codebook, N, V, indices, st);
    case 32: return vq_launch<32>(features, ld, codebook, N, V, indices, st);
    case 64: return vq_launch<64>(features, ld, codebook, N, V, indices, st);
    }
    return VFM_NO_KERNEL;
}
