// Spectral normalisation of a weight in training mode (torch.nn.utils.spectral_norm with one power
// iteration, dim 0, as the projected discriminator's heads use it: reference networks/discriminator.py
// SpectralConv1d, `SpectralNorm.apply(self, name='weight', n_power_iterations=1, dim=0, eps=1e-12)`),
// forward in three launches and backward in two (torch: ~13 and ~6 small kernels per call).
//
// W [O, I] (the weight reshaped to a matrix), u [O] and v [I] the persistent power-iteration vectors:
//   v <- normalize(W^T u),  u <- normalize(W v)          (normalize(x) = x / max(||x||, eps)), in place
//   sigma = u . (W v) = ||W v||^2 / max(||W v||, eps),  W_sn = W / sigma
// backward (u, v constants, as torch detaches them):
//   dW = g / sigma - (sum_ij g_ij W_ij) / sigma^2 * u v^T
// Launches (fwd): K1 t = W^T u (16 columns x 16 row groups per block) + per-block ||t||^2 partials;
// K2 r = W v (one row per block, v = t / max(||t||, eps) formed from the K1 partials on the fly; block 0
// stores v) + per-row ||r||^2 partials; K3 W_sn = W / sigma (grid-stride; block 0 stores u and sigma).
// (bwd): K4 per-block partials of sum g W; K5 dW. Partial sums are added in a fixed order.
#include "vfm_common.h"

namespace {

using namespace vfm;

constexpr int THREADS = 256;

__device__ __forceinline__ float block_reduce(float v, float* sh) {
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) sh[wave] = v;
    __syncthreads();
    return (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

// sum of n partials in a fixed order (every thread gets the same value)
__device__ __forceinline__ float sum_parts(const float* p, int n, float* sh) {
    float s = 0.f;
    for (int i = threadIdx.x; i < n; i += THREADS) s += p[i];
    return block_reduce(s, sh);
}

// 16 columns x 16 row groups per block (4x the blocks of a 64-column tile, a quarter of the serial row loop
// per thread: the heads' W is only 384 x 3456, so the 64-column form ran 54 blocks of 96-row loops)
constexpr int TU_COLS = 16, TU_RG = THREADS / TU_COLS;

__device__ __forceinline__ void sn_wtu_body(const float* __restrict__ W, const float* __restrict__ u,
                                            float* __restrict__ t, float* __restrict__ part, int O, int I, int bid) {
    __shared__ float red[TU_RG][TU_COLS + 1];
    __shared__ float sh[4];
    const int col = threadIdx.x % TU_COLS, rg = threadIdx.x / TU_COLS;
    const int i = bid * TU_COLS + col;
    float s = 0.f;
    if (i < I)
        // 8 rows per round, their loads issued before the FMAs (one round trip per 8 rows)
        for (int o0 = rg; o0 < O; o0 += 8 * TU_RG) {
            float w[8], uv[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int o = o0 + k * TU_RG;
                w[k] = o < O ? W[(long long)o * I + i] : 0.f;
                uv[k] = o < O ? u[o] : 0.f;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) s = fmaf(w[k], uv[k], s);
        }
    red[rg][col] = s;
    __syncthreads();
    float tv = 0.f;
    if (rg == 0) {
#pragma unroll
        for (int g = 0; g < TU_RG; ++g) tv += red[g][col];
        if (i < I) t[i] = tv;
    }
    const float ss = block_reduce(rg == 0 && i < I ? tv * tv : 0.f, sh);
    if (threadIdx.x == 0) part[bid] = ss;
}

__global__ __launch_bounds__(THREADS) void sn_wtu(const float* __restrict__ W, const float* __restrict__ u,
                                                  float* __restrict__ t, float* __restrict__ part, int O, int I) {
    sn_wtu_body(W, u, t, part, O, I, blockIdx.x);
}

// one row of W per block (the 256 threads striding over the row, their loads issued in rounds of 8 before
// the FMAs: a 3456-wide row is two round trips; one row per wave took fourteen)
__device__ __forceinline__ void sn_wv_body(const float* __restrict__ W, const float* __restrict__ t,
                                           const float* __restrict__ tpart, int ntp, float* __restrict__ v,
                                           float* __restrict__ v_copy, float* __restrict__ r,
                                           float* __restrict__ rpart, int O, int I, float eps, int bid) {
    __shared__ float sh[4];
    const float inv = 1.f / fmaxf(sqrtf(sum_parts(tpart, ntp, sh)), eps);
    if (bid == 0)
        for (int i = threadIdx.x; i < I; i += THREADS) {
            const float x = t[i] * inv;
            v[i] = x;
            if (v_copy) v_copy[i] = x;
        }
    const int o = bid;
    const float* wr = W + (long long)o * I;
    float s = 0.f;
    for (int i0 = threadIdx.x; i0 < I; i0 += 8 * THREADS) {
        float w[8], tv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int i = i0 + k * THREADS;
            w[k] = i < I ? wr[i] : 0.f;
            tv[k] = i < I ? t[i] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) s = fmaf(w[k], tv[k] * inv, s);
    }
    s = block_reduce(s, sh);
    if (threadIdx.x == 0) {
        r[o] = s;
        rpart[o] = s * s;
    }
}

__global__ __launch_bounds__(THREADS) void sn_wv(const float* __restrict__ W, const float* __restrict__ t,
                                                 const float* __restrict__ tpart, int ntp, float* __restrict__ v,
                                                 float* __restrict__ v_copy, float* __restrict__ r,
                                                 float* __restrict__ rpart, int O, int I, float eps) {
    sn_wv_body(W, t, tpart, ntp, v, v_copy, r, rpart, O, I, eps, blockIdx.x);
}

__device__ __forceinline__ void sn_scale_body(const float* __restrict__ W, const float* __restrict__ r,
                                              const float* __restrict__ rpart, int nrp, float* __restrict__ u,
                                              float* __restrict__ u_copy, float* __restrict__ sigma,
                                              float* __restrict__ Wsn, int O, long long n, float eps, int vec, int bid,
                                              int nblk) {
    __shared__ float sh[4];
    const float rr = sum_parts(rpart, nrp, sh);
    const float inv = 1.f / fmaxf(sqrtf(rr), eps);
    const float sg = rr * inv;                       // u . r with u = r * inv
    if (bid == 0) {
        for (int o = threadIdx.x; o < O; o += THREADS) {
            const float x = r[o] * inv;
            u[o] = x;
            if (u_copy) u_copy[o] = x;
        }
        if (threadIdx.x == 0) sigma[0] = sg;
    }
    const float is = 1.f / sg;
    if (vec) {                                       // float4 per thread (n % 4 == 0, 16-B aligned W / Wsn)
        const long long n4 = n >> 2;
        for (long long e = (long long)bid * THREADS + threadIdx.x; e < n4; e += (long long)nblk * THREADS) {
            float4 w = reinterpret_cast<const float4*>(W)[e];
            w.x *= is; w.y *= is; w.z *= is; w.w *= is;
            reinterpret_cast<float4*>(Wsn)[e] = w;
        }
        return;
    }
    for (long long e = (long long)bid * THREADS + threadIdx.x; e < n; e += (long long)nblk * THREADS)
        Wsn[e] = W[e] * is;
}

__global__ __launch_bounds__(THREADS) void sn_scale(const float* __restrict__ W, const float* __restrict__ r,
                                                    const float* __restrict__ rpart, int nrp, float* __restrict__ u,
                                                    float* __restrict__ u_copy, float* __restrict__ sigma,
                                                    float* __restrict__ Wsn, int O, long long n, float eps, int vec) {
    sn_scale_body(W, r, rpart, nrp, u, u_copy, sigma, Wsn, O, n, eps, vec, blockIdx.x, gridDim.x);
}

__device__ __forceinline__ void sn_gw_body(const float* __restrict__ g, const float* __restrict__ W,
                                           float* __restrict__ part, long long n, int vec, int bid, int nblk) {
    __shared__ float sh[4];
    float s = 0.f;
    if (vec) {                                       // n % 4 == 0, 16-B aligned g / W
        const long long n4 = n >> 2;
        for (long long e = (long long)bid * THREADS + threadIdx.x; e < n4; e += (long long)nblk * THREADS) {
            const float4 a = reinterpret_cast<const float4*>(g)[e], b = reinterpret_cast<const float4*>(W)[e];
            s = fmaf(a.x, b.x, s); s = fmaf(a.y, b.y, s); s = fmaf(a.z, b.z, s); s = fmaf(a.w, b.w, s);
        }
    } else {
        for (long long e = (long long)bid * THREADS + threadIdx.x; e < n; e += (long long)nblk * THREADS)
            s = fmaf(g[e], W[e], s);
    }
    s = block_reduce(s, sh);
    if (threadIdx.x == 0) part[bid] = s;
}

__global__ __launch_bounds__(THREADS) void sn_gw(const float* __restrict__ g, const float* __restrict__ W,
                                                 float* __restrict__ part, long long n, int vec) {
    sn_gw_body(g, W, part, n, vec, blockIdx.x, gridDim.x);
}

__device__ __forceinline__ void sn_dw_body(const float* __restrict__ g, const float* __restrict__ u,
                                           const float* __restrict__ v, const float* __restrict__ sigma,
                                           const float* __restrict__ part, int np, float* __restrict__ dW,
                                           int I, long long n, int vec, int bid, int nblk) {
    __shared__ float sh[4];
    const float S = sum_parts(part, np, sh);
    const float sg = sigma[0];
    const float is = 1.f / sg, c = S / (sg * sg);
    if (vec) {                                       // float4 per thread (I % 4 == 0, 16-B aligned g / v / dW)
        const long long n4 = n >> 2;
        const int I4 = I >> 2;
        for (long long e = (long long)bid * THREADS + threadIdx.x; e < n4; e += (long long)nblk * THREADS) {
            const long long o = e / I4;
            const float4 gv = reinterpret_cast<const float4*>(g)[e];
            const float4 vv = reinterpret_cast<const float4*>(v)[e - o * I4];
            const float cu = c * u[o];
            reinterpret_cast<float4*>(dW)[e] =
                make_float4(gv.x * is - cu * vv.x, gv.y * is - cu * vv.y, gv.z * is - cu * vv.z, gv.w * is - cu * vv.w);
        }
        return;
    }
    for (long long e = (long long)bid * THREADS + threadIdx.x; e < n; e += (long long)nblk * THREADS) {
        const long long o = e / I;
        dW[e] = g[e] * is - c * u[o] * v[e - o * I];
    }
}

__global__ __launch_bounds__(THREADS) void sn_dw(const float* __restrict__ g, const float* __restrict__ u,
                                                 const float* __restrict__ v, const float* __restrict__ sigma,
                                                 const float* __restrict__ part, int np, float* __restrict__ dW,
                                                 int I, long long n, int vec) {
    sn_dw_body(g, u, v, sigma, part, np, dW, I, n, vec, blockIdx.x, gridDim.x);
}

constexpr int SCALE_BLOCKS = 512;

}  // namespace

// floats of workspace vfm_specnorm_fwd / _bwd need for an [O, I] weight
extern "C" long long vfm_specnorm_workspace_floats(int O, int I) {
    if (O <= 0 || I <= 0) return VFM_ERR_ARGS;
    const long long tb = (I + TU_COLS - 1) / TU_COLS, rb = O;
    return (long long)I + O + tb + rb + SCALE_BLOCKS;
}

// One power iteration on (u [O], v [I]) in place, sigma [1] and Wsn = W / sigma for fp32 W [O, I];
// u_copy / v_copy (optional) receive the new u / v too (the backward's constants: torch clones them,
// since a later forward updates the buffers before this call's backward runs).
extern "C" int vfm_specnorm_fwd(const float* W, float* u, float* v, float* u_copy, float* v_copy, float* sigma,
                                float* Wsn, float* ws, int O, int I, float eps, void* stream) {
    if (!W || !u || !v || !sigma || !Wsn || !ws || O <= 0 || I <= 0) return VFM_ERR_ARGS;
    const int tb = (I + TU_COLS - 1) / TU_COLS, rb = O;
    float* t = ws;
    float* r = t + I;
    float* tpart = r + O;
    float* rpart = tpart + tb;
    hipStream_t st = (hipStream_t)stream;
    VFM_LAUNCH(sn_wtu, dim3(tb), dim3(THREADS), 0, st, W, u, t, tpart, O, I);
    VFM_LAUNCH(sn_wv, dim3(rb), dim3(THREADS), 0, st, W, t, tpart, tb, v, v_copy, r, rpart, O, I, eps);
    const long long n = (long long)O * I;
    // float4 only on 16-B aligned views (a weight view with a storage offset takes the scalar loop)
    const int vec = (n & 3) == 0 && (((uintptr_t)W | (uintptr_t)Wsn) & 15) == 0;
    const long long work = vec ? n / 4 : n;           // threads' items
    const int sb = (int)std::min<long long>(4096, (work + THREADS - 1) / THREADS);
    VFM_LAUNCH(sn_scale, dim3(sb), dim3(THREADS), 0, st, W, r, rpart, rb, u, u_copy, sigma, Wsn, O, n, eps, vec);
    return launch_status();
}

// dW = g / sigma - (sum g W) / sigma^2 u v^T (u, v, sigma as left by the forward).
extern "C" int vfm_specnorm_bwd(const float* g, const float* W, const float* u, const float* v, const float* sigma,
                                float* dW, float* ws, int O, int I, void* stream) {
    if (!g || !W || !u || !v || !sigma || !dW || !ws || O <= 0 || I <= 0) return VFM_ERR_ARGS;
    const long long n = (long long)O * I;
    const int nb = (int)std::min<long long>(SCALE_BLOCKS, (n + THREADS - 1) / THREADS);
    hipStream_t st = (hipStream_t)stream;
    const int vg = (n & 3) == 0 && (((uintptr_t)g | (uintptr_t)W) & 15) == 0;
    const int vd = (I & 3) == 0 && (((uintptr_t)g | (uintptr_t)v | (uintptr_t)dW) & 15) == 0;
    VFM_LAUNCH(sn_gw, dim3(nb), dim3(THREADS), 0, st, g, W, ws, n, vg);
    VFM_LAUNCH(sn_dw, dim3(nb), dim3(THREADS), 0, st, g, u, v, sigma, ws, nb, dW, I, n, vd);
    return launch_status();
}

// ---------------------------------------------------------------------------------------------------------------
// Grouped form: every spectral-normalised weight of the discriminator heads in one launch per phase (forward
// phases 0, 1, 2 = the K1, K2, K3 launches above; backward 3, 4 = K4, K5), torch_utils/ops/specnorm_group.py. The
// host packs each phase's table (vfm_specnorm_group_pack, host memory) and uploads it; vfm_specnorm_group_launch
// runs it. Per weight the same blocks and arithmetic as vfm_specnorm_fwd / _bwd.
namespace {

struct SnArgs {
    const float* W;
    float* u;
    float* v;
    float* uc;
    float* vc;
    float* sigma;
    float* Wsn;
    float* ws;
    const float* g;
    float* dW;
    int O, I, tb, sb, vec, nb, vg, vd;
    float eps;
    int pad;
};

constexpr int SNP = 10;          // pointer slots per weight in the pack call

template <int PH>
__global__ __launch_bounds__(THREADS) void sn_group_kernel(const SnArgs* __restrict__ tab, const int* __restrict__ off,
                                                           int n) {
    int l = 0;
    while (l + 1 < n && (int)blockIdx.x >= off[l + 1]) ++l;
    const SnArgs a = tab[l];
    const int bid = (int)blockIdx.x - off[l], nblk = off[l + 1] - off[l];
    float* t = a.ws;
    float* r = t + a.I;
    float* tpart = r + a.O;
    float* rpart = tpart + a.tb;
    const long long nn = (long long)a.O * a.I;
    if (PH == 0) sn_wtu_body(a.W, a.u, t, tpart, a.O, a.I, bid);
    else if (PH == 1) sn_wv_body(a.W, t, tpart, a.tb, a.v, a.vc, r, rpart, a.O, a.I, a.eps, bid);
    else if (PH == 2) sn_scale_body(a.W, r, rpart, a.O, a.u, a.uc, a.sigma, a.Wsn, a.O, nn, a.eps, a.vec, bid, nblk);
    else if (PH == 3) sn_gw_body(a.g, a.W, a.ws, nn, a.vg, bid, nblk);
    else sn_dw_body(a.g, a.uc, a.vc, a.sigma, a.ws, a.nb, a.dW, a.I, nn, a.vd, bid, nblk);
}

}  // namespace

// Bytes of one packed phase section for n weights (table + offsets, 16-B multiple).
extern "C" long long vfm_specnorm_group_bytes(int n) {
    if (n <= 0) return VFM_ERR_ARGS;
    const long long b = (long long)n * sizeof(SnArgs) + (long long)(n + 1) * 4;
    return (b + 15) / 16 * 16;
}

// Pack phase `phase` for n weights into host_out (vfm_specnorm_group_bytes(n) bytes). Per weight l:
// ptrs[10 l ..] = W, u, v, u_copy, v_copy, sigma, Wsn, ws (forward: vfm_specnorm_workspace_floats(O, I) floats;
// backward: the same), g, dW (forward phases ignore g / dW; backward phases read W, u_copy, v_copy, sigma, g and
// write dW); dims[2 l ..] = O, I; eps[l]. Returns the phase's total blocks or an error code < 0.
extern "C" long long vfm_specnorm_group_pack(int phase, int n, const long long* ptrs, const int* dims, const float* eps,
                                             void* host_out) {
    if (n <= 0 || !ptrs || !dims || !eps || !host_out || phase < 0 || phase > 4) return VFM_ERR_ARGS;
    SnArgs* tab = reinterpret_cast<SnArgs*>(host_out);
    int* off = reinterpret_cast<int*>(reinterpret_cast<char*>(host_out) + (size_t)n * sizeof(SnArgs));
    long long total = 0;
    for (int l = 0; l < n; ++l) {
        const long long* p = ptrs + (long long)SNP * l;
        SnArgs a{};
        a.W = (const float*)p[0]; a.u = (float*)p[1]; a.v = (float*)p[2]; a.uc = (float*)p[3]; a.vc = (float*)p[4];
        a.sigma = (float*)p[5]; a.Wsn = (float*)p[6]; a.ws = (float*)p[7]; a.g = (const float*)p[8];
        a.dW = (float*)p[9];
        a.O = dims[2 * l]; a.I = dims[2 * l + 1]; a.eps = eps[l];
        if (a.O <= 0 || a.I <= 0 || !a.W || !a.ws || !a.sigma) return VFM_ERR_ARGS;
        const long long nn = (long long)a.O * a.I;
        a.tb = (a.I + TU_COLS - 1) / TU_COLS;
        a.vec = (nn & 3) == 0 && (((uintptr_t)a.W | (uintptr_t)a.Wsn) & 15) == 0;
        a.sb = (int)std::min<long long>(4096, ((a.vec ? nn / 4 : nn) + THREADS - 1) / THREADS);
        a.nb = (int)std::min<long long>(SCALE_BLOCKS, (nn + THREADS - 1) / THREADS);
        a.vg = (nn & 3) == 0 && (((uintptr_t)a.g | (uintptr_t)a.W) & 15) == 0;
        a.vd = (a.I & 3) == 0 && (((uintptr_t)a.g | (uintptr_t)a.vc | (uintptr_t)a.dW) & 15) == 0;
        long long blocks = 0;
        if (phase <= 2) {
            if (!a.u || !a.v || !a.Wsn) return VFM_ERR_ARGS;
            blocks = phase == 0 ? a.tb : phase == 1 ? a.O : a.sb;
        } else {
            if (!a.g || !a.dW || !a.uc || !a.vc) return VFM_ERR_ARGS;
            blocks = a.nb;
        }
        tab[l] = a;
        off[l] = (int)total;
        total += blocks;
        if (total > 0x7fffffffLL) return VFM_ERR_ARGS;
    }
    off[n] = (int)total;
    return total;
}

extern "C" int vfm_specnorm_group_launch(int phase, const void* dev_packed, int n, long long total_blocks,
                                         void* stream) {
    if (!dev_packed || n <= 0 || total_blocks < 0 || total_blocks > 0x7fffffffLL) return VFM_ERR_ARGS;
    if (total_blocks == 0) return 0;
    const SnArgs* tab = reinterpret_cast<const SnArgs*>(dev_packed);
    const int* off = reinterpret_cast<const int*>(reinterpret_cast<const char*>(dev_packed) + (size_t)n * sizeof(SnArgs));
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)total_blocks), block(THREADS);
    switch (phase) {
    case 0: VFM_LAUNCH(sn_group_kernel<0>, grid, block, 0, st, tab, off, n); break;
    case 1: VFM_LAUNCH(sn_group_kernel<1>, grid, block, 0, st, tab, off, n); break;
    case 2: VFM_LAUNCH(sn_group_kernel<2>, grid, block, 0, st, tab, off, n); break;
    case 3: VFM_LAUNCH(sn_group_kernel<3>, grid, block, 0, st, tab, off, n); break;
    case 4: VFM_LAUNCH(sn_group_kernel<4>, grid, block, 0, st, tab, off, n); break;
    default: return VFM_ERR_ARGS;
    }
    return launch_status();
}
