// Multi-scale PatchGAN discriminator kernels (stage 3; reference networks/discriminator.py:75-99
// BatchNormLocal2d, :180-228 NLayerDiscriminator: k4 convs at stride 2 / 1, pad 2, BatchNormLocal2d,
// LeakyReLU(0.2)), fp32 as the reference runs them, activations NHWC ([B, H, W, C], channels_last).
//
// A k x k conv is an implicit GEMM over the im2col matrix A[m, (ky k + kx) C + c] (m = (b, oy, ox)):
//   forward      Y[M, Cout]  = A W^T (+ bias)               -- our MFMA GEMM (f32x3), Y is NHWC
//   weight grad  dW[Cout, K] = dY^T A                        -- same GEMM, split-K
//   data grad    dX = col2im(dY W)                           -- GEMM, then the gather below
// so these kernels are the layout passes around the GEMMs (HBM-bound streams: im2col writes A once
// reading x from L2; col2im reads each dA element once and writes dX once, no atomics) plus, for the
// 1-channel logit layer, a row dot / column dot in place of a 1-wide GEMM, and the virtual-batch
// BatchNorm + LeakyReLU forward / backward (per-(group, channel) statistics over NHWC rows: lanes along
// channels, 16-B loads, fixed-order partial sums -> deterministic).
#include "vfm_common.h"

namespace {

using namespace vfm;

struct ConvGeo {
    int B, H, W, C, Ho, Wo, k, stride, pad;
    long long ldA;
};

// A[m, tap C + c] for one (m, tap, 4-channel chunk) per thread (C % 4 == 0), or one channel (else)
template <bool V4>
__global__ __launch_bounds__(256) void im2col_nhwc(const float* __restrict__ x, float* __restrict__ A, ConvGeo g,
                                                   long long total) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    const int CV = V4 ? g.C / 4 : g.C;
    const int cv = (int)(i % CV);
    const long long r = i / CV;
    const int kk = g.k * g.k;
    const int tap = (int)(r % kk);
    const long long m = r / kk;
    const int ox = (int)(m % g.Wo);
    const long long t = m / g.Wo;
    const int oy = (int)(t % g.Ho), b = (int)(t / g.Ho);
    const int iy = oy * g.stride - g.pad + tap / g.k, ix = ox * g.stride - g.pad + tap % g.k;
    const bool ok = iy >= 0 && iy < g.H && ix >= 0 && ix < g.W;
    float* dst = A + m * g.ldA + (long long)tap * g.C;
    if (V4) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ok) v = *reinterpret_cast<const float4*>(x + (((long long)b * g.H + iy) * g.W + ix) * g.C + 4 * cv);
        *reinterpret_cast<float4*>(dst + 4 * cv) = v;
    } else {
        dst[cv] = ok ? x[(((long long)b * g.H + iy) * g.W + ix) * g.C + cv] : 0.f;
    }
}

// dX[b, iy, ix, c] = sum over the taps that read (iy, ix) of dA[m, tap C + c]; with dy1 / w1 (the
// 1-channel layer) dA[m, kk] = dy1[m] w1[kk] is formed on the fly
template <bool V4>
__global__ __launch_bounds__(256) void col2im_nhwc(const float* __restrict__ dA, const float* __restrict__ dy1,
                                                   const float* __restrict__ w1, float* __restrict__ dX, ConvGeo g,
                                                   long long total) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    const int CV = V4 ? g.C / 4 : g.C;
    const int cv = (int)(i % CV);
    const long long p = i / CV;
    const int ix = (int)(p % g.W);
    const long long t = p / g.W;
    const int iy = (int)(t % g.H), b = (int)(t / g.H);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int ky = 0; ky < g.k; ++ky) {
        const int ny = iy + g.pad - ky;
        if (ny < 0 || ny % g.stride) continue;
        const int oy = ny / g.stride;
        if (oy >= g.Ho) continue;
        for (int kx = 0; kx < g.k; ++kx) {
            const int nx = ix + g.pad - kx;
            if (nx < 0 || nx % g.stride) continue;
            const int ox = nx / g.stride;
            if (ox >= g.Wo) continue;
            const long long m = ((long long)b * g.Ho + oy) * g.Wo + ox;
            const int col = (ky * g.k + kx) * g.C + (V4 ? 4 * cv : cv);
            if (dy1) {
                const float d = dy1[m];
                if (V4) {
                    const float4 w = *reinterpret_cast<const float4*>(w1 + col);
                    acc.x = fmaf(d, w.x, acc.x); acc.y = fmaf(d, w.y, acc.y);
                    acc.z = fmaf(d, w.z, acc.z); acc.w = fmaf(d, w.w, acc.w);
                } else {
                    acc.x = fmaf(d, w1[col], acc.x);
                }
            } else if (V4) {
                const float4 v = *reinterpret_cast<const float4*>(dA + m * g.ldA + col);
                acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
            } else {
                acc.x += dA[m * g.ldA + col];
            }
        }
    }
    float* dst = dX + (((long long)b * g.H + iy) * g.W + ix) * g.C;
    if (V4) *reinterpret_cast<float4*>(dst + 4 * cv) = acc;
    else dst[cv] = acc.x;
}

// y[m] = sum_k A[m, k] w[k] + bias: one wave per row (K % 4 == 0)
__global__ __launch_bounds__(256) void rowdot(const float* __restrict__ A, long long ldA, const float* __restrict__ w,
                                              const float* __restrict__ bias, float* __restrict__ y, int M, int K) {
    const int lane = threadIdx.x & 63;
    const long long m = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (m >= M) return;
    const float* a = A + m * ldA;
    float s = 0.f;
    for (int k = 4 * lane; k < K; k += 256) {
        const float4 u = *reinterpret_cast<const float4*>(a + k), v = *reinterpret_cast<const float4*>(w + k);
        s = fmaf(u.x, v.x, s); s = fmaf(u.y, v.y, s); s = fmaf(u.z, v.z, s); s = fmaf(u.w, v.w, s);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) y[m] = s + (bias ? bias[0] : 0.f);
}

// part[s, k] = sum_{m in split s} A[m, k] v[m]; grid (ceil(K / 1024), S), 4 columns per thread
__global__ __launch_bounds__(256) void coldot(const float* __restrict__ A, long long ldA, const float* __restrict__ v,
                                              float* __restrict__ part, int M, int K, int span) {
    const int k = 4 * (blockIdx.x * 256 + threadIdx.x);
    if (k >= K) return;
    const int m0 = blockIdx.y * span, m1 = min(M, m0 + span);
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int m = m0; m < m1; ++m) {
        const float d = v[m];
        const float4 u = *reinterpret_cast<const float4*>(A + (long long)m * ldA + k);
        s.x = fmaf(u.x, d, s.x); s.y = fmaf(u.y, d, s.y); s.z = fmaf(u.z, d, s.z); s.w = fmaf(u.w, d, s.w);
    }
    *reinterpret_cast<float4*>(part + (long long)blockIdx.y * K + k) = s;
}

// ---- BatchNormLocal2d + LeakyReLU over NHWC rows ---------------------------------------------
// x [B, P, C]; group g = samples [g n, (g+1) n), n = B / G; statistics per (g, c) over n * P rows.
// Block 256 threads = R row lanes x C/4 channel lanes (C / 4 divides 256); grid (chunks, G).

struct BnArgs {
    const float* x;
    const float* dy;
    const float* w;
    const float* b;
    const float* mean;
    const float* rstd;
    float* out;          // y (fwd) / dx (bwd)
    float* part;         // [G, chunks, 2, C]
    int B, P, C, G, n, chunks;
    long long rows_g;    // n * P
    long long span;      // rows per chunk
    float slope;
};

// MODE 0: sum x; 1: sum (x - mean)^2; 2: sum dz, sum dz * xhat (dz = dy * lrelu'(xhat w + b))
template <int MODE>
__global__ __launch_bounds__(256) void bn_reduce(BnArgs a) {
    __shared__ float4 red[2][256];
    const int C4 = a.C / 4, R = 256 / C4;
    const int c4 = threadIdx.x % C4, r = threadIdx.x / C4;
    const int g = blockIdx.y, ch = blockIdx.x;
    const long long q0 = (long long)ch * a.span, q1 = min(a.rows_g, q0 + a.span);
    const float* xg = a.x + (long long)g * a.rows_g * a.C + 4 * c4;
    float4 m4 = make_float4(0.f, 0.f, 0.f, 0.f), s4 = m4, w4 = m4, b4 = m4;
    if (MODE >= 1) m4 = *reinterpret_cast<const float4*>(a.mean + (long long)g * a.C + 4 * c4);
    if (MODE == 2) {
        s4 = *reinterpret_cast<const float4*>(a.rstd + (long long)g * a.C + 4 * c4);
        w4 = a.w ? *reinterpret_cast<const float4*>(a.w + 4 * c4) : make_float4(1.f, 1.f, 1.f, 1.f);
        b4 = a.b ? *reinterpret_cast<const float4*>(a.b + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float4 acc0 = make_float4(0.f, 0.f, 0.f, 0.f), acc1 = acc0;
    for (long long q = q0 + r; q < q1; q += R) {
        const float4 v = *reinterpret_cast<const float4*>(xg + q * a.C);
        if (MODE == 0) {
            acc0.x += v.x; acc0.y += v.y; acc0.z += v.z; acc0.w += v.w;
        } else if (MODE == 1) {
            const float dx_ = v.x - m4.x, dy_ = v.y - m4.y, dz_ = v.z - m4.z, dw_ = v.w - m4.w;
            acc0.x = fmaf(dx_, dx_, acc0.x); acc0.y = fmaf(dy_, dy_, acc0.y);
            acc0.z = fmaf(dz_, dz_, acc0.z); acc0.w = fmaf(dw_, dw_, acc0.w);
        } else {
            const float4 d = *reinterpret_cast<const float4*>(a.dy + (long long)g * a.rows_g * a.C + q * a.C + 4 * c4);
            const float h[4] = {(v.x - m4.x) * s4.x, (v.y - m4.y) * s4.y, (v.z - m4.z) * s4.z, (v.w - m4.w) * s4.w};
            const float ww[4] = {w4.x, w4.y, w4.z, w4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
            const float dd[4] = {d.x, d.y, d.z, d.w};
            float z[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float zz = fmaf(h[e], ww[e], bb[e]);
                z[e] = zz > 0.f ? dd[e] : dd[e] * a.slope;
            }
            acc0.x += z[0]; acc0.y += z[1]; acc0.z += z[2]; acc0.w += z[3];
            acc1.x = fmaf(z[0], h[0], acc1.x); acc1.y = fmaf(z[1], h[1], acc1.y);
            acc1.z = fmaf(z[2], h[2], acc1.z); acc1.w = fmaf(z[3], h[3], acc1.w);
        }
    }
    red[0][threadIdx.x] = acc0;
    red[1][threadIdx.x] = acc1;
    __syncthreads();
    if (r == 0) {
        for (int j = 1; j < R; ++j) {
            const float4 u = red[0][j * C4 + c4], v = red[1][j * C4 + c4];
            acc0.x += u.x; acc0.y += u.y; acc0.z += u.z; acc0.w += u.w;
            acc1.x += v.x; acc1.y += v.y; acc1.z += v.z; acc1.w += v.w;
        }
        float* p = a.part + (((long long)g * a.chunks + ch) * 2) * a.C + 4 * c4;
        *reinterpret_cast<float4*>(p) = acc0;
        *reinterpret_cast<float4*>(p + a.C) = acc1;
    }
}

// MODE 0: mean = S0 / cnt; 1: rstd = rsqrt(S0 / cnt + eps); 2: dw / db (summed over groups) and the
// per-(g, c) backward coefficients kept in part's first chunk: [mean(dz), mean(dz xhat)]
template <int MODE>
__global__ __launch_bounds__(256) void bn_finalize(BnArgs a, float* __restrict__ o0, float* __restrict__ o1,
                                                   float* __restrict__ dw, float* __restrict__ db, float eps) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= a.C) return;
    const float cnt = (float)a.rows_g;
    float tw = 0.f, tb = 0.f;
    for (int g = 0; g < a.G; ++g) {
        float s0 = 0.f, s1 = 0.f;
        for (int ch = 0; ch < a.chunks; ++ch) {
            const float* p = a.part + (((long long)g * a.chunks + ch) * 2) * a.C + c;
            s0 += p[0];
            s1 += p[a.C];
        }
        if (MODE == 0) o0[(long long)g * a.C + c] = s0 / cnt;
        else if (MODE == 1) o0[(long long)g * a.C + c] = 1.f / sqrtf(s0 / cnt + eps);
        else {
            tb += s0;
            tw += s1;
            o0[(long long)g * a.C + c] = s0 / cnt;
            o1[(long long)g * a.C + c] = s1 / cnt;
        }
    }
    if (MODE == 2) {
        if (dw) dw[c] = tw;
        if (db) db[c] = tb;
    }
}

// forward apply: y = lrelu((x - mean) rstd w + b); backward apply (BWD):
// dx = rstd w (dz - mean(dz) - xhat mean(dz xhat)), coefficients from bn_finalize<2> in c0 / c1
template <bool BWD>
__global__ __launch_bounds__(256) void bn_apply(BnArgs a, const float* __restrict__ c0, const float* __restrict__ c1,
                                                long long total4) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= total4) return;
    const int C4 = a.C / 4;
    const int c = 4 * (int)(i % C4);
    const long long row = i / C4;                    // b * P + p
    const int g = (int)(row / a.rows_g);
    const long long gc = (long long)g * a.C + c;
    const float4 v = *reinterpret_cast<const float4*>(a.x + 4 * i);
    const float4 m4 = *reinterpret_cast<const float4*>(a.mean + gc);
    const float4 s4 = *reinterpret_cast<const float4*>(a.rstd + gc);
    const float4 w4 = a.w ? *reinterpret_cast<const float4*>(a.w + c) : make_float4(1.f, 1.f, 1.f, 1.f);
    const float4 b4 = a.b ? *reinterpret_cast<const float4*>(a.b + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float xv[4] = {v.x, v.y, v.z, v.w}, mm[4] = {m4.x, m4.y, m4.z, m4.w}, ss[4] = {s4.x, s4.y, s4.z, s4.w};
    const float ww[4] = {w4.x, w4.y, w4.z, w4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
    float o[4];
    if (!BWD) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float z = fmaf((xv[e] - mm[e]) * ss[e], ww[e], bb[e]);
            o[e] = z > 0.f ? z : z * a.slope;
        }
    } else {
        const float4 d = *reinterpret_cast<const float4*>(a.dy + 4 * i);
        const float4 k0 = *reinterpret_cast<const float4*>(c0 + gc), k1 = *reinterpret_cast<const float4*>(c1 + gc);
        const float dd[4] = {d.x, d.y, d.z, d.w}, q0[4] = {k0.x, k0.y, k0.z, k0.w}, q1[4] = {k1.x, k1.y, k1.z, k1.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float h = (xv[e] - mm[e]) * ss[e];
            const float z = fmaf(h, ww[e], bb[e]);
            const float dz = z > 0.f ? dd[e] : dd[e] * a.slope;
            o[e] = ss[e] * ww[e] * (dz - q0[e] - h * q1[e]);
        }
    }
    *reinterpret_cast<float4*>(a.out + 4 * i) = make_float4(o[0], o[1], o[2], o[3]);
}


// ---- BatchNormLocal (1-d, the projected discriminator's heads) + LeakyReLU over [B, C, L] -----------
// reference networks/discriminator.py:45-71 (BatchNormLocal over virtual batches of 8: statistics per
// (group, channel) over the group's samples and L) and the head blocks' LeakyReLU(0.2) (:102-109).
// One block per (group, channel): the n * L values (<= 8 x 200 here) are reduced in two passes
// (mean, then centred variance), fixed-order block reductions; backward: sum dz, sum dz xhat, dx.

__device__ __forceinline__ float block_sum256(float v, float* red) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void bn1d_fwd(const float* __restrict__ x, const float* __restrict__ w,
                                                const float* __restrict__ b, float* __restrict__ y,
                                                float* __restrict__ mean, float* __restrict__ rstd, int C, int L,
                                                int n, float eps, float slope) {
    __shared__ float red[4];
    const int g = blockIdx.y, c = blockIdx.x;
    const int cnt = n * L;
    auto at = [&](int i) -> long long { const int s = i / L; return ((long long)(g * n + s) * C + c) * L + (i - s * L); };
    float s1 = 0.f;
    for (int i = threadIdx.x; i < cnt; i += 256) s1 += x[at(i)];
    const float mu = block_sum256(s1, red) / (float)cnt;
    float s2 = 0.f;
    for (int i = threadIdx.x; i < cnt; i += 256) {
        const float d = x[at(i)] - mu;
        s2 = fmaf(d, d, s2);
    }
    const float rs = 1.f / sqrtf(block_sum256(s2, red) / (float)cnt + eps);
    const float wc = w ? w[c] : 1.f, bc = b ? b[c] : 0.f;
    for (int i = threadIdx.x; i < cnt; i += 256) {
        const long long o = at(i);
        const float z = fmaf((x[o] - mu) * rs, wc, bc);
        y[o] = z > 0.f ? z : z * slope;
    }
    if (threadIdx.x == 0) {
        mean[g * C + c] = mu;
        rstd[g * C + c] = rs;
    }
}

__global__ __launch_bounds__(256) void bn1d_bwd(const float* __restrict__ x, const float* __restrict__ dy,
                                                const float* __restrict__ w, const float* __restrict__ b,
                                                const float* __restrict__ mean, const float* __restrict__ rstd,
                                                float* __restrict__ dx, float* __restrict__ part, int C, int L, int n,
                                                float slope) {
    __shared__ float red[4];
    const int g = blockIdx.y, c = blockIdx.x, G = gridDim.y;
    const int cnt = n * L;
    auto at = [&](int i) -> long long { const int s = i / L; return ((long long)(g * n + s) * C + c) * L + (i - s * L); };
    const float mu = mean[g * C + c], rs = rstd[g * C + c];
    const float wc = w ? w[c] : 1.f, bc = b ? b[c] : 0.f;
    float a0 = 0.f, a1 = 0.f;
    for (int i = threadIdx.x; i < cnt; i += 256) {
        const long long o = at(i);
        const float h = (x[o] - mu) * rs;
        const float z = fmaf(h, wc, bc);
        const float dz = z > 0.f ? dy[o] : dy[o] * slope;
        a0 += dz;
        a1 = fmaf(dz, h, a1);
    }
    const float S1 = block_sum256(a0, red);
    const float S2 = block_sum256(a1, red);
    const float m1 = S1 / (float)cnt, m2 = S2 / (float)cnt;
    for (int i = threadIdx.x; i < cnt; i += 256) {
        const long long o = at(i);
        const float h = (x[o] - mu) * rs;
        const float z = fmaf(h, wc, bc);
        const float dz = z > 0.f ? dy[o] : dy[o] * slope;
        dx[o] = rs * wc * (dz - m1 - h * m2);
    }
    if (threadIdx.x == 0) {                 // per-group partials of dw (sum dz xhat) and db (sum dz)
        part[(long long)g * C + c] = S2;
        part[((long long)G + g) * C + c] = S1;
    }
}

int bn_setup(BnArgs& a, int B, int P, int C, int G) {
    if (B <= 0 || P <= 0 || C < 4 || C % 4 || C > 1024 || 256 % (C / 4) || G <= 0 || B % G) return VFM_ERR_ARGS;
    a.B = B; a.P = P; a.C = C; a.G = G; a.n = B / G;
    a.rows_g = (long long)a.n * P;
    const int R = 256 / (C / 4);
    long long want = (1024 + G - 1) / G;
    const long long maxc = (a.rows_g + R - 1) / R;
    if (want > maxc) want = maxc;
    if (want > 65535) want = 65535;
    a.chunks = (int)(want < 1 ? 1 : want);
    a.span = (a.rows_g + a.chunks - 1) / a.chunks;
    return VFM_OK;
}

}  // namespace

extern "C" int vfm_im2col_nhwc_f32(const float* x, float* A, long long ldA, int B, int H, int W, int C, int Ho, int Wo,
                                   int k, int stride, int pad, void* stream) {
    if (!x || !A || B <= 0 || H <= 0 || W <= 0 || C <= 0 || Ho <= 0 || Wo <= 0 || k <= 0 || stride <= 0 || pad < 0)
        return VFM_ERR_ARGS;
    if (ldA < (long long)k * k * C) return VFM_ERR_ARGS;
    const bool v4 = C % 4 == 0 && ldA % 4 == 0 && ((uintptr_t)x | (uintptr_t)A) % 16 == 0;
    ConvGeo g{B, H, W, C, Ho, Wo, k, stride, pad, ldA};
    const long long total = (long long)B * Ho * Wo * k * k * (v4 ? C / 4 : C);
    const long long blocks = (total + 255) / 256;
    if (blocks > 0x7fffffffLL) return VFM_ERR_ARGS;
    hipStream_t st = (hipStream_t)stream;
    if (v4) VFM_LAUNCH(im2col_nhwc<true>, dim3((unsigned)blocks), dim3(256), 0, st, x, A, g, total);
    else VFM_LAUNCH(im2col_nhwc<false>, dim3((unsigned)blocks), dim3(256), 0, st, x, A, g, total);
    return launch_status();
}

extern "C" int vfm_col2im_nhwc_f32(const float* dA, long long ldA, const float* dy1, const float* w1, float* dX, int B,
                                   int H, int W, int C, int Ho, int Wo, int k, int stride, int pad, void* stream) {
    if (!dX || (!dA && !(dy1 && w1)) || B <= 0 || H <= 0 || W <= 0 || C <= 0 || Ho <= 0 || Wo <= 0 || k <= 0 ||
        stride <= 0 || pad < 0)
        return VFM_ERR_ARGS;
    if (dA && ldA < (long long)k * k * C) return VFM_ERR_ARGS;
    const bool v4 = C % 4 == 0 && (!dA || ldA % 4 == 0) &&
                    ((uintptr_t)dA | (uintptr_t)dX | (uintptr_t)w1) % 16 == 0;
    ConvGeo g{B, H, W, C, Ho, Wo, k, stride, pad, ldA};
    const long long total = (long long)B * H * W * (v4 ? C / 4 : C);
    const long long blocks = (total + 255) / 256;
    if (blocks > 0x7fffffffLL) return VFM_ERR_ARGS;
    hipStream_t st = (hipStream_t)stream;
    const float* a = (dy1 && w1) ? nullptr : dA;
    if (v4) VFM_LAUNCH(col2im_nhwc<true>, dim3((unsigned)blocks), dim3(256), 0, st, a, dy1, w1, dX, g, total);
    else VFM_LAUNCH(col2im_nhwc<false>, dim3((unsigned)blocks), dim3(256), 0, st, a, dy1, w1, dX, g, total);
    return launch_status();
}

extern "C" int vfm_rowdot_f32(const float* A, long long ldA, const float* w, const float* bias, float* y, int M, int K,
                              void* stream) {
    if (!A || !w || !y || M <= 0 || K <= 0 || ldA < K) return VFM_ERR_ARGS;
    if (K % 4 || ldA % 4 || ((uintptr_t)A | (uintptr_t)w) % 16) return VFM_NO_KERNEL;
    VFM_LAUNCH(rowdot, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, (hipStream_t)stream, A, ldA, w, bias, y, M,
                       K);
    return launch_status();
}

// splits S of vfm_coldot_f32 (part holds S * K floats)
extern "C" int vfm_coldot_splits(int M, int K) {
    if (M <= 0 || K <= 0) return -1;
    const int cols = (K + 1023) / 1024;
    int S = (1024 + cols - 1) / cols;
    const int smax = (M + 63) / 64;
    if (S > smax) S = smax;
    if (S > 65535) S = 65535;
    return S < 1 ? 1 : S;
}

extern "C" int vfm_coldot_f32(const float* A, long long ldA, const float* v, float* part, int M, int K, int S,
                              void* stream) {
    if (!A || !v || !part || M <= 0 || K <= 0 || S <= 0 || S > 65535 || ldA < K) return VFM_ERR_ARGS;
    if (K % 4 || ldA % 4 || ((uintptr_t)A | (uintptr_t)part) % 16) return VFM_NO_KERNEL;
    const int span = (M + S - 1) / S;
    VFM_LAUNCH(coldot, dim3((unsigned)((K + 1023) / 1024), S), dim3(256), 0, (hipStream_t)stream, A, ldA, v,
                       part, M, K, span);
    return launch_status();
}

// workspace floats of the BatchNormLocal2d kernels
extern "C" long long vfm_bnl_workspace_floats(int B, int P, int C, int G) {
    BnArgs a;
    if (bn_setup(a, B, P, C, G) != VFM_OK) return -1;
    return (long long)G * a.chunks * 2 * C + 2ll * G * C;
}

extern "C" int vfm_bnl_lrelu_fwd(const float* x, const float* w, const float* b, float* y, float* mean, float* rstd,
                                 float* ws, int B, int P, int C, int G, float eps, float slope, void* stream) {
    BnArgs a = {};
    int rc = bn_setup(a, B, P, C, G);
    if (rc != VFM_OK) return rc;
    if (!x || !y || !mean || !rstd || !ws) return VFM_ERR_ARGS;
    if (((uintptr_t)x | (uintptr_t)y | (uintptr_t)mean | (uintptr_t)rstd | (uintptr_t)ws | (uintptr_t)w |
         (uintptr_t)b) % 16)
        return VFM_NO_KERNEL;
    a.x = x; a.w = w; a.b = b; a.mean = mean; a.rstd = rstd; a.out = y; a.part = ws; a.slope = slope;
    hipStream_t st = (hipStream_t)stream;
    const dim3 rg(a.chunks, G), fg((C + 255) / 256);
    VFM_LAUNCH(bn_reduce<0>, rg, dim3(256), 0, st, a);
    VFM_LAUNCH(bn_finalize<0>, fg, dim3(256), 0, st, a, mean, (float*)nullptr, (float*)nullptr,
                       (float*)nullptr, eps);
    VFM_LAUNCH(bn_reduce<1>, rg, dim3(256), 0, st, a);
    VFM_LAUNCH(bn_finalize<1>, fg, dim3(256), 0, st, a, rstd, (float*)nullptr, (float*)nullptr,
                       (float*)nullptr, eps);
    const long long total4 = (long long)B * P * C / 4;
    const long long blocks = (total4 + 255) / 256;
    if (blocks > 0x7fffffffLL) return VFM_ERR_ARGS;
    VFM_LAUNCH(bn_apply<false>, dim3((unsigned)blocks), dim3(256), 0, st, a, (const float*)nullptr,
                       (const float*)nullptr, total4);
    return launch_status();
}

extern "C" int vfm_bnl_lrelu_bwd(const float* x, const float* dy, const float* w, const float* b, const float* mean,
                                 const float* rstd, float* dx, float* dw, float* db, float* ws, int B, int P, int C,
                                 int G, float slope, void* stream) {
    BnArgs a = {};
    int rc = bn_setup(a, B, P, C, G);
    if (rc != VFM_OK) return rc;
    if (!x || !dy || !dx || !mean || !rstd || !ws) return VFM_ERR_ARGS;
    if (((uintptr_t)x | (uintptr_t)dy | (uintptr_t)dx | (uintptr_t)mean | (uintptr_t)rstd | (uintptr_t)ws |
         (uintptr_t)w | (uintptr_t)b) % 16)
        return VFM_NO_KERNEL;
    a.x = x; a.dy = dy; a.w = w; a.b = b; a.mean = mean; a.rstd = rstd; a.out = dx; a.part = ws; a.slope = slope;
    float* c0 = ws + (long long)G * a.chunks * 2 * C;
    float* c1 = c0 + (long long)G * C;
    hipStream_t st = (hipStream_t)stream;
    VFM_LAUNCH(bn_reduce<2>, dim3(a.chunks, G), dim3(256), 0, st, a);
    VFM_LAUNCH(bn_finalize<2>, dim3((C + 255) / 256), dim3(256), 0, st, a, c0, c1, dw, db, 0.f);
    const long long total4 = (long long)B * P * C / 4;
    const long long blocks = (total4 + 255) / 256;
    if (blocks > 0x7fffffffLL) return VFM_ERR_ARGS;
    VFM_LAUNCH(bn_apply<true>, dim3((unsigned)blocks), dim3(256), 0, st, a, (const float*)c0,
                       (const float*)c1, total4);
    return launch_status();
}

// BatchNormLocal (1-d) + LeakyReLU over x [B, C, L] fp32 in G virtual batches (B % G == 0); mean / rstd
// [G, C] saved for the backward. bwd: dx, and part [2, G, C] = per-group (sum dz xhat, sum dz).
extern "C" int vfm_bnl1d_lrelu_fwd(const float* x, const float* w, const float* b, float* y, float* mean, float* rstd,
                                   int B, int C, int L, int G, float eps, float slope, void* stream) {
    if (!x || !y || !mean || !rstd || B <= 0 || C <= 0 || L <= 0 || G <= 0 || B % G || C > 65535 || G > 65535)
        return VFM_ERR_ARGS;
    if ((long long)(B / G) * L > 0x7fffffffLL) return VFM_ERR_ARGS;
    VFM_LAUNCH(bn1d_fwd, dim3(C, G), dim3(256), 0, (hipStream_t)stream, x, w, b, y, mean, rstd, C, L, B / G,
                       eps, slope);
    return launch_status();
}

extern "C" int vfm_bnl1d_lrelu_bwd(const float* x, const float* dy, const float* w, const float* b, const float* mean,
                                   const float* rstd, float* dx, float* part, int B, int C, int L, int G, float slope,
                                   void* stream) {
    if (!x || !dy || !dx || !part || !mean || !rstd || B <= 0 || C <= 0 || L <= 0 || G <= 0 || B % G ||
        C > 65535 || G > 65535)
        return VFM_ERR_ARGS;
    VFM_LAUNCH(bn1d_bwd, dim3(C, G), dim3(256), 0, (hipStream_t)stream, x, dy, w, b, mean, rstd, dx, part, C,
                       L, B / G, slope);
    return launch_status();
}
