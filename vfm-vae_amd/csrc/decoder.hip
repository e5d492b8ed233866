// Decoder kernels for gfx950: the ops the shipped ConvNeXt decoder actually runs
// (reference networks/utils/convnext_utils.py:36-257, networks/utils/shared.py:165-167).
//
//  * dwconv2d fwd / bwd-weight: depthwise KxK conv (K = 3, 5, 7), stride 1, zero padding,
//    fused bias and legacy additive noise plane. LDS-staged input tile with halo; every lane
//    owns one column and an 8-row strip (sliding K-row register window), so an output costs
//    K*K FMAs but only ~(K+8)/8 LDS row reads. Narrow planes (W < 64) pack several planes
//    side by side in one wave. bwd-data is the forward with the flipped kernel.
//  * group_norm fwd / bwd: one workgroup per (sample, group); the group is one contiguous
//    [C/G x HW] chunk in NCHW, read with 16-B vector loads; fp32 statistics (shifted sums);
//    optional per-(sample, channel) scale folded in (modulated-conv input modulation).
//  * scale_bias_gelu fwd / bwd: gelu(h * s[b,o] + b[o]) (exact erf GELU) on [B, O, P], one
//    wave per (b, o) row so the backward's d_scale / d_bias row sums need no atomics.
//  * layer_scale_residual fwd / bwd: x_in + gamma[c] * (y + b[c]), same row structure.
//  * shuffle_blur fwd / bwd: PixelShuffle(r) + replicate padding + fixed normalised separable
//    blur, fused (the shuffled tensor is never materialised); the backward is the exact
//    gather-form adjoint including the replicate-padding edge folding.
#include "vfm_common.h"

#include <type_traits>

namespace {

using namespace vfm;

constexpr int NT = 256;
constexpr int RPT = 8;   // output rows per lane in the depthwise conv

// -------------------------------------------------------------------------------------------
// Depthwise conv.

struct DwArgs {
    const void* x;
    const float* w;       // [C, K, K] fp32
    const float* bias;    // [C] or null
    const float* noise;   // [Ho, Wo] or null
    const void* res;      // [B, C, Ho, Wo] in y's dtype, added to y, or null
    void* y;
    int B, C, H, W, Ho, Wo, pad;
    int flip;             // taps read rotated by 180 degrees (the data gradient)
    int TW, TH;           // tile width (pow2, <= 64), tile height (multiple of RPT)
    int ppw;              // planes side by side in one wave row (64 / TW)
    int spp;              // row strips per plane tile (TH / RPT)
    int ppb;              // planes per block = ppw * (4 / spp)
    int tilesX, tilesY, planeGroups;
};

// Stage ppb halo tiles [LH x LW] (zero padded) into LDS without per-element divisions:
// a wave covers `rpw` rows per instruction with `lpr` (pow2 >= LW, <= 64) lanes per row.
template <class T>
__device__ __forceinline__ void dw_stage(const DwArgs& a, float* lds, int pg, int ox0, int oy0, int LW, int LH) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int lpr = 1;
    while (lpr < LW && lpr < 64) lpr <<= 1;
    const int rpw = 64 / lpr;
    const int sub = lane / lpr, cx = lane - sub * lpr;
    const int nplanes = a.B * a.C;
    const int rows = a.ppb * LH;
    const T* xbase = reinterpret_cast<const T*>(a.x);
    for (int q0 = wave * rpw; q0 < rows; q0 += 4 * rpw) {
        const int q = q0 + sub;
        if (q >= rows) continue;
        const int p = q / LH, ry = q - p * LH;
        const int plane = pg * a.ppb + p;
        const int iy = oy0 + ry - a.pad;
        const bool rok = plane < nplanes && iy >= 0 && iy < a.H;
        const T* src = xbase + ((long long)plane * a.H + iy) * a.W;
        float* dst = lds + (p * LH + ry) * LW;
        for (int rx = cx; rx < LW; rx += lpr) {
            const int ix = ox0 + rx - a.pad;
            dst[rx] = (rok && ix >= 0 && ix < a.W) ? ld(src + ix) : 0.f;
        }
    }
}

template <class T, int K>
__global__ __launch_bounds__(NT) void dw_fwd(DwArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int LW = a.TW + K - 1, LH = a.TH + K - 1;
    int bid = blockIdx.x;
    const int tx = bid % a.tilesX; bid /= a.tilesX;
    const int ty = bid % a.tilesY; bid /= a.tilesY;
    const int pg = bid;                                  // plane group
    const int ox0 = tx * a.TW, oy0 = ty * a.TH;
    const int nplanes = a.B * a.C;

    const int per = LW * LH;
    dw_stage<T>(a, lds, pg, ox0, oy0, LW, LH);
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int col = lane % a.TW, psub = lane / a.TW;
    const int strip = wave % a.spp, pgrp = wave / a.spp;
    const int pl = pgrp * a.ppw + psub;
    const int plane = pg * a.ppb + pl;
    if (pl >= a.ppb || plane >= nplanes) return;
    const int c = plane % a.C;
    const int ox = ox0 + col;
    const int r0 = strip * RPT;
    if (ox >= a.Wo) return;

    float wk[K * K];
#pragma unroll
    for (int i = 0; i < K * K; ++i) wk[i] = a.w[c * K * K + (a.flip ? K * K - 1 - i : i)];
    float acc[RPT];
    const float b = a.bias ? a.bias[c] : 0.f;
#pragma unroll
    for (int i = 0; i < RPT; ++i) acc[i] = b;

    const float* tile = lds + pl * per + col;
    // Input row (r0 + j) contributes to output rows r0 + j - ky for ky in [0, K).
#pragma unroll
    for (int j = 0; j < RPT + K - 1; ++j) {
        float row[K];
#pragma unroll
        for (int kx = 0; kx < K; ++kx) row[kx] = tile[(r0 + j) * LW + kx];
#pragma unroll
        for (int ky = 0; ky < K; ++ky) {
            const int o = j - ky;
            if (o >= 0 && o < RPT) {
#pragma unroll
                for (int kx = 0; kx < K; ++kx) acc[o] = fmaf(row[kx], wk[ky * K + kx], acc[o]);
            }
        }
    }
    T* yp = reinterpret_cast<T*>(a.y) + (long long)plane * a.Ho * a.Wo + ox;
    const T* rp = a.res ? reinterpret_cast<const T*>(a.res) + (long long)plane * a.Ho * a.Wo + ox : nullptr;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
        const int oy = oy0 + r0 + i;
        if (oy < a.Ho) {
            float v = acc[i];
            if (a.noise) v += a.noise[oy * a.Wo + ox];
            if (rp) v += ld(rp + (long long)oy * a.Wo);
            st(yp + (long long)oy * a.Wo, v);
        }
    }
}

// dW[plane][ky][kx] = sum_{y,x} dy[y][x] * x[y+ky-pad][x+kx-pad]; db[plane] = sum dy.
// One workgroup per (plane group, column tile) walks all row tiles of its planes, so the
// K*K+1 per-lane sums are reduced once per column band. Inner loop = the forward's sliding
// window: each staged input row is read once (K LDS reads) and meets the RPT dy values held
// in registers. Per-(column tile, plane) partials are summed by the host in a fixed order.
template <class T, int K>
__global__ __launch_bounds__(NT) void dw_bwd_w(DwArgs a, const void* dy, float* partial) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int LW = a.TW + K - 1, LH = a.TH + K - 1;
    const int tx = blockIdx.x % a.tilesX;
    const int pg = blockIdx.x / a.tilesX;
    const int ox0 = tx * a.TW;
    const int nplanes = a.B * a.C;
    const int per = LW * LH;

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int col = lane % a.TW, psub = lane / a.TW;
    const int strip = wave % a.spp, pgrp = wave / a.spp;
    const int pl = pgrp * a.ppw + psub;
    const int plane = pg * a.ppb + pl;
    const int ox = ox0 + col;
    const int r0 = strip * RPT;
    const bool live = pl < a.ppb && plane < nplanes && ox < a.Wo;
    const T* dyp = reinterpret_cast<const T*>(dy) + (long long)plane * a.Ho * a.Wo + ox;
    const float* tile = lds + pl * per + col;

    float acc[K * K + 1];
#pragma unroll
    for (int i = 0; i < K * K + 1; ++i) acc[i] = 0.f;

    for (int ty = 0; ty < a.tilesY; ++ty) {
        const int oy0 = ty * a.TH;
        __syncthreads();                       // previous tile fully consumed
        dw_stage<T>(a, lds, pg, ox0, oy0, LW, LH);
        __syncthreads();
        if (live) {
            float g[RPT];
#pragma unroll
            for (int i = 0; i < RPT; ++i) {
                const int oy = oy0 + r0 + i;
                g[i] = oy < a.Ho ? ld(dyp + (long long)oy * a.Wo) : 0.f;
                acc[K * K] += g[i];
            }
#pragma unroll
            for (int j = 0; j < RPT + K - 1; ++j) {
                float row[K];
#pragma unroll
                for (int kx = 0; kx < K; ++kx) row[kx] = tile[(r0 + j) * LW + kx];
#pragma unroll
                for (int ky = 0; ky < K; ++ky) {
                    const int o = j - ky;
                    if (o >= 0 && o < RPT) {
#pragma unroll
                        for (int kx = 0; kx < K; ++kx) acc[ky * K + kx] = fmaf(g[o], row[kx], acc[ky * K + kx]);
                    }
                }
            }
        }
    }
    // Reduce over the lanes that belong to the same plane: first within the wave (lanes
    // with equal psub are TW apart), then across waves through LDS.
    __syncthreads();
    float* red = lds;   // reuse: [4 waves][ppw][K*K+1]
#pragma unroll
    for (int i = 0; i < K * K + 1; ++i) {
        float v = acc[i];
        for (int off = a.TW / 2; off >= 1; off >>= 1) v += __shfl_xor(v, off);
        if (col == 0) red[(wave * a.ppw + psub) * (K * K + 1) + i] = v;
    }
    __syncthreads();
    // Plane p of this block lives in waves {grp*spp .. grp*spp+spp-1}, slot sub.
    for (int i = threadIdx.x; i < a.ppb * (K * K + 1); i += NT) {
        const int p = i / (K * K + 1), k = i - p * (K * K + 1);
        const int plane_g = pg * a.ppb + p;
        if (plane_g >= nplanes) continue;
        const int grp = p / a.ppw, sub = p - grp * a.ppw;
        float s = 0.f;
        for (int st_ = 0; st_ < a.spp; ++st_) s += red[((grp * a.spp + st_) * a.ppw + sub) * (K * K + 1) + k];
        partial[((long long)tx * nplanes + plane_g) * (K * K + 1) + k] = s;
    }
}

template <class T, int K>
int dw_launch(DwArgs& a, int mode, const void* dy, float* partial, hipStream_t st) {
    const size_t lds = sizeof(float) * (size_t)a.ppb * (a.TW + K - 1) * (a.TH + K - 1);
    const size_t red = sizeof(float) * 4 * a.ppw * (K * K + 1);
    if (mode == 0) {
        const long long blocks = (long long)a.tilesX * a.tilesY * a.planeGroups;
        VFM_LAUNCH((dw_fwd<T, K>), dim3((unsigned)blocks), dim3(NT), lds, st, a);
    } else {
        const long long blocks = (long long)a.tilesX * a.planeGroups;
        VFM_LAUNCH((dw_bwd_w<T, K>), dim3((unsigned)blocks), dim3(NT), lds > red ? lds : red, st, a, dy,
                           partial);
    }
    return launch_status();
}

int next_pow2(int v) {
    int p = 1;
    while (p < v) p <<= 1;
    return p;
}

void dw_plan(DwArgs& a) {
    a.TW = next_pow2(a.Wo) < 64 ? next_pow2(a.Wo) : 64;
    if (a.TW < 1) a.TW = 1;
    a.ppw = 64 / a.TW;
    const int rows_needed = (a.Ho + RPT - 1) / RPT;           // strips to cover the plane height
    a.spp = rows_needed >= 4 ? 4 : (rows_needed >= 2 ? 2 : 1);
    a.TH = a.spp * RPT;
    a.ppb = a.ppw * (4 / a.spp);
    a.tilesX = (a.Wo + a.TW - 1) / a.TW;
    a.tilesY = (a.Ho + a.TH - 1) / a.TH;
    a.planeGroups = (a.B * a.C + a.ppb - 1) / a.ppb;
}

template <class T>
int dw_dispatch(DwArgs& a, int K, int mode, const void* dy, float* partial, hipStream_t st) {
    switch (K) {
    case 1: return dw_launch<T, 1>(a, mode, dy, partial, st);
    case 3: return dw_launch<T, 3>(a, mode, dy, partial, st);
    case 5: return dw_launch<T, 5>(a, mode, dy, partial, st);
    case 7: return dw_launch<T, 7>(a, mode, dy, partial, st);
    }
    return VFM_NO_KERNEL;
}

// -------------------------------------------------------------------------------------------
// Row-streaming depthwise conv for "same" convolutions (odd K, pad = (K-1)/2) on planes
// 16..256 wide. L = W/4 lanes span one image row (4 adjacent columns per lane), so a wave
// holds R = 64 / L independent row groups. Work unit = (sample b, row band) of ONE channel c:
// a wave always works on a single channel (the K*K weights are wave-uniform scalars) and
// its R groups take R consecutive units of that channel -- different bands of one plane for
// wide planes, different samples for narrow ones -- so every lane is busy even when a plane
// is only 16 rows tall. Each lane streams its band top to bottom: one 4-element vector load
// per input row (issued one row ahead in the forward), the K-1 halo columns from the
// neighbouring lanes by cross-lane shuffles (a group spans a full image row, so the group
// edge is the zero-padded image border), and K rotating output-row accumulators. No LDS;
// every input byte is loaded ~once (band halo only).

struct DwRowArgs {
    const void* x;
    const float* w;       // [C, K, K]
    const float* bias;    // [C] or null
    const float* noise;   // [H, W] or null
    const void* res;      // [B, C, H, W] in y's dtype, added to y, or null
    void* y;
    const void* dy;       // weight-gradient mode
    float* partial;       // [wpc, C, K*K+1]
    int B, C, H, W;
    int flip;             // taps read rotated by 180 degrees (the data gradient)
    int L, R;             // lanes per row, row groups per wave
    int BH;               // band height
    int nb;               // bands per plane
    int wpc;              // waves per channel = ceil(B * nb / R)
};

template <class T>
__device__ __forceinline__ void ld4(const T* p, float* v) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = ld(p + i);
}
template <>
__device__ __forceinline__ void ld4<__hip_bfloat16>(const __hip_bfloat16* p, float* v) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(u.x << 16);
    v[1] = __uint_as_float(u.x & 0xffff0000u);
    v[2] = __uint_as_float(u.y << 16);
    v[3] = __uint_as_float(u.y & 0xffff0000u);
}
template <>
__device__ __forceinline__ void ld4<__half>(const __half* p, float* v) {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    const __half2* h = reinterpret_cast<const __half2*>(&u);
    const float2 a = __half22float2(h[0]), b = __half22float2(h[1]);
    v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
}
template <>
__device__ __forceinline__ void ld4<float>(const float* p, float* v) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
}
template <class T>
__device__ __forceinline__ void st4(T* p, const float* v) {
    T t[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) st(&t[i], v[i]);
    *reinterpret_cast<uint2*>(p) = *reinterpret_cast<const uint2*>(t);
}
template <>
__device__ __forceinline__ void st4<float>(float* p, const float* v) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}

typedef float f2 __attribute__((ext_vector_type(2)));

// v[0 .. K+2]: the lane's 4 columns with PAD columns of left and K-1-PAD of right halo.
template <int K>
__device__ __forceinline__ void dwr_halo(const float* own, float* v, int q, int L) {
    constexpr int PAD = (K - 1) / 2;
#pragma unroll
    for (int t = 0; t < PAD; ++t) {
        const float s = __shfl_up(own[4 - PAD + t], 1, L);
        v[t] = q == 0 ? 0.f : s;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) v[PAD + c] = own[c];
#pragma unroll
    for (int t = 0; t < K - 1 - PAD; ++t) {
        const float s = __shfl_down(own[t], 1, L);
        v[PAD + 4 + t] = q == L - 1 ? 0.f : s;
    }
}

// Lane -> (channel, plane offset, band start, live) for the unit decomposition above.
struct DwrLane {
    int c, q, y0, wv;
    long long poff;
    bool live;
};
__device__ __forceinline__ DwrLane dwr_lane(const DwRowArgs& a) {
    DwrLane r;
    const int wave_g = blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
    r.c = __builtin_amdgcn_readfirstlane(wave_g / a.wpc);
    r.wv = wave_g - r.c * a.wpc;
    const int lane = threadIdx.x & 63;
    const int grp = lane / a.L;
    r.q = lane - grp * a.L;
    const int u = r.wv * a.R + grp;                    // unit within the channel
    r.live = r.c < a.C && u < a.B * a.nb;
    const int b = r.live ? u / a.nb : 0;
    const int band = r.live ? u - b * a.nb : 0;
    r.y0 = band * a.BH;
    r.poff = ((long long)b * a.C + (r.live ? r.c : 0)) * a.H * a.W + 4 * r.q;
    return r;
}

template <class T, int K>
__global__ __launch_bounds__(NT) void dwr_fwd(DwRowArgs a) {
    constexpr int PAD = (K - 1) / 2;
    const DwrLane ln = dwr_lane(a);
    if (ln.c >= a.C) return;                            // wave-uniform
    const int c = ln.c, q = ln.q, y0 = ln.y0;
    const bool live = ln.live;
    float wk[K * K];
#pragma unroll
    for (int i = 0; i < K * K; ++i) wk[i] = a.w[c * K * K + (a.flip ? K * K - 1 - i : i)];
    const float bias = a.bias ? a.bias[c] : 0.f;
    const T* xp = reinterpret_cast<const T*>(a.x) + ln.poff;
    T* yp = reinterpret_cast<T*>(a.y) + ln.poff;
    const T* rp = a.res ? reinterpret_cast<const T*>(a.res) + ln.poff : nullptr;
    const float* np = a.noise ? a.noise + 4 * q : nullptr;

    f2 acc2[K][2];
#pragma unroll
    for (int s = 0; s < K; ++s) acc2[s][0] = acc2[s][1] = f2{0.f, 0.f};
    const int nrows = a.BH + K - 1;
    float nxt[4] = {0.f, 0.f, 0.f, 0.f};
    if (live && y0 - PAD >= 0 && y0 - PAD < a.H) ld4(xp + (long long)(y0 - PAD) * a.W, nxt);
    for (int jj0 = 0; jj0 < nrows; jj0 += K) {
#pragma unroll
        for (int u = 0; u < K; ++u) {
            const int jj = jj0 + u;
            if (jj < nrows) {
                acc2[u][0] = acc2[u][1] = f2{bias, bias};              // output row jj starts here
                float own[4] = {nxt[0], nxt[1], nxt[2], nxt[3]};
                const int iyn = y0 - PAD + jj + 1;                     // prefetch the next input row
#pragma unroll
                for (int c4 = 0; c4 < 4; ++c4) nxt[c4] = 0.f;
                if (live && jj + 1 < nrows && iyn >= 0 && iyn < a.H) ld4(xp + (long long)iyn * a.W, nxt);
                float v[K + 3];
                dwr_halo<K>(own, v, q, a.L);
                // column pairs (2p, 2p+1) as packed fp32 (v_pk_fma_f32): the operand pair for tap kx
                // is (v[2p+kx], v[2p+kx+1]) = ve[p + kx/2] (kx even) or vo[p + kx/2] (kx odd)
                f2 ve[(K + 3) / 2], vo[(K + 2) / 2];
#pragma unroll
                for (int i = 0; i < (K + 3) / 2; ++i) ve[i] = f2{v[2 * i], v[2 * i + 1]};
#pragma unroll
                for (int i = 0; i < (K + 2) / 2; ++i) vo[i] = f2{v[2 * i + 1], v[2 * i + 2]};
#pragma unroll
                for (int ky = 0; ky < K; ++ky) {
                    const int sl = (u - ky + K) % K;                    // output row jj - ky
#pragma unroll
                    for (int p2 = 0; p2 < 2; ++p2)
#pragma unroll
                        for (int kx = 0; kx < K; ++kx) {
                            const f2 xv = (kx & 1) ? vo[p2 + kx / 2] : ve[p2 + kx / 2];
                            const float wv = wk[ky * K + kx];
                            acc2[sl][p2] = __builtin_elementwise_fma(xv, f2{wv, wv}, acc2[sl][p2]);
                        }
                }
                const int ob = jj - (K - 1);                           // completed output row
                const int oy = y0 + ob;
                if (live && ob >= 0 && ob < a.BH && oy < a.H) {
                    const f2 o0 = acc2[(u + 1) % K][0], o1 = acc2[(u + 1) % K][1];
                    float o[4] = {o0.x, o0.y, o1.x, o1.y};
                    if (np) {
#pragma unroll
                        for (int c4 = 0; c4 < 4; ++c4) o[c4] += np[oy * a.W + c4];
                    }
                    if (rp) {
                        float rv[4];
                        ld4(rp + (long long)oy * a.W, rv);
#pragma unroll
                        for (int c4 = 0; c4 < 4; ++c4) o[c4] += rv[c4];
                    }
                    st4(yp + (long long)oy * a.W, o);
                }
            }
        }
    }
}

// dW[ky][kx] = sum dy[oy][ox] x[oy + ky - PAD][ox + kx - PAD], db = sum dy, per channel;
// the wave's total (all its lanes share the channel) goes to partial[wv][c][:], summed by
// the host in a fixed order (deterministic).
template <class T, int K>
__global__ __launch_bounds__(NT) void dwr_bwd_w(DwRowArgs a) {
    constexpr int PAD = (K - 1) / 2;
    const DwrLane ln = dwr_lane(a);
    if (ln.c >= a.C) return;                            // wave-uniform
    const int lane = threadIdx.x & 63;
    const int q = ln.q, y0 = ln.y0;
    const bool live = ln.live;
    const T* xp = reinterpret_cast<const T*>(a.x) + ln.poff;
    const T* gp = reinterpret_cast<const T*>(a.dy) + ln.poff;

    float acc[K * K + 1];
#pragma unroll
    for (int i = 0; i < K * K + 1; ++i) acc[i] = 0.f;
    float gw[K][4];                                   // dy rows jj-K+1 .. jj (rotating)
#pragma unroll
    for (int s = 0; s < K; ++s)
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) gw[s][c4] = 0.f;
    const int nrows = a.BH + K - 1;
    for (int jj0 = 0; jj0 < nrows; jj0 += K) {
#pragma unroll
        for (int u = 0; u < K; ++u) {
            const int jj = jj0 + u;
            if (jj < nrows) {
                const int oy = y0 + jj;
#pragma unroll
                for (int c4 = 0; c4 < 4; ++c4) gw[u][c4] = 0.f;
                if (live && jj < a.BH && oy < a.H) ld4(gp + (long long)oy * a.W, gw[u]);
                acc[K * K] += (gw[u][0] + gw[u][1]) + (gw[u][2] + gw[u][3]);
                const int iy = y0 - PAD + jj;
                float own[4] = {0.f, 0.f, 0.f, 0.f};
                if (live && iy >= 0 && iy < a.H) ld4(xp + (long long)iy * a.W, own);
                float v[K + 3];
                dwr_halo<K>(own, v, q, a.L);
                // scalar FMAs here: the packed form (v_pk_fma_f32 over column pairs) measured 13-18 %
                // slower at 158 VGPRs (occupancy 3)
#pragma unroll
                for (int ky = 0; ky < K; ++ky) {
                    const int sl = (u - ky + K) % K;                    // dy row jj - ky
#pragma unroll
                    for (int kx = 0; kx < K; ++kx) {
                        float t = acc[ky * K + kx];
#pragma unroll
                        for (int c4 = 0; c4 < 4; ++c4) t = fmaf(gw[sl][c4], v[c4 + kx], t);
                        acc[ky * K + kx] = t;
                    }
                }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < K * K + 1; ++i) {
        float t = acc[i];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) t += __shfl_xor(t, off);
        if (lane == 0) a.partial[((long long)ln.wv * a.C + ln.c) * (K * K + 1) + i] = t;
    }
}

// Row-streaming plan; returns false when the shape is not covered (caller uses dw_fwd / dw_bwd_w).
// Band height: as tall as possible (halo re-reads (K-1)/BH), never much taller than the plane,
// halved while the grid has fewer than 16384 waves (64 per CU).
bool dwr_plan(DwRowArgs& a, int K, int pad) {
    if (K % 2 == 0 || pad != (K - 1) / 2 || K > 7) return false;
    if (a.W < 16 || a.W > 256 || a.W % 4) return false;
    const int L = a.W / 4;
    if (L & (L - 1)) return false;
    a.L = L;
    a.R = 64 / L;
    int BH = 64;
    while (BH > 8 && BH / 2 >= a.H) BH /= 2;
    for (;;) {
        a.nb = (a.H + BH - 1) / BH;
        a.wpc = (a.B * a.nb + a.R - 1) / a.R;
        if (BH <= 8 || (long long)a.C * a.wpc >= 16384) break;
        BH /= 2;
    }
    a.BH = BH;
    return true;
}

template <class T>
int dwr_launch(DwRowArgs& a, int K, int mode, hipStream_t st) {
    const long long waves = (long long)a.C * a.wpc;
    const dim3 grid((unsigned)((waves + 3) / 4));
#define DWR_CASE(KK)                                                                   \
    case KK:                                                                           \
        if (mode == 0) VFM_LAUNCH((dwr_fwd<T, KK>), grid, dim3(NT), 0, st, a); \
        else VFM_LAUNCH((dwr_bwd_w<T, KK>), grid, dim3(NT), 0, st, a);         \
        break;
    switch (K) {
        DWR_CASE(3)
        DWR_CASE(5)
        DWR_CASE(7)
    default: return VFM_NO_KERNEL;
    }
#undef DWR_CASE
    return launch_status();
}

// -------------------------------------------------------------------------------------------
// Block reductions.

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// Sum over the 256 threads; result broadcast to all. `scratch` needs 4 floats + a barrier-safe slot.
__device__ __forceinline__ float block_sum(float v, float* scratch) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) scratch[w] = v;
    __syncthreads();
    return scratch[0] + scratch[1] + scratch[2] + scratch[3];
}

// Vector loads of 8 elements (16 B for 16-bit types, 2 x 16 B for fp32).
template <class T>
__device__ __forceinline__ void load8(const T* p, float* v) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = ld(p + i);
}
template <>
__device__ __forceinline__ void load8<__hip_bfloat16>(const __hip_bfloat16* p, float* v) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const unsigned w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(w[i] << 16);
        v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
}
template <>
__device__ __forceinline__ void load8<__half>(const __half* p, float* v) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const __half2* h = reinterpret_cast<const __half2*>(&u);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        float2 f = __half22float2(h[i]);
        v[2 * i] = f.x;
        v[2 * i + 1] = f.y;
    }
}
template <>
__device__ __forceinline__ void load8<float>(const float* p, float* v) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

template <class T>
__device__ __forceinline__ void store8(T* p, const float* v) {
#pragma unroll
    for (int i = 0; i < 8; ++i) st(p + i, v[i]);
}
template <>
__device__ __forceinline__ void store8<__hip_bfloat16>(__hip_bfloat16* p, const float* v) {
    typedef float f8 __attribute__((ext_vector_type(8)));
    typedef __bf16 b8 __attribute__((ext_vector_type(8)));
    const f8 x = {v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]};
    *reinterpret_cast<uint4*>(p) = __builtin_bit_cast(uint4, __builtin_convertvector(x, b8));   // 4 v_cvt_pk_bf16_f32
}
template <>
__device__ __forceinline__ void store8<__half>(__half* p, const float* v) {
    __half t[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) t[i] = __float2half(v[i]);
    *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(t);
}
template <>
__device__ __forceinline__ void store8<float>(float* p, const float* v) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

// -------------------------------------------------------------------------------------------
// GroupNorm.

struct GnArgs {
    const void* x;
    const float* w;      // [C] or null
    const float* b;      // [C] or null
    const float* s;      // [B, C] or null (style)
    void* y;
    float* mean;         // [B*G]
    float* rstd;         // [B*G]
    int B, C, G, HW;
    float eps;
    // precomputed statistics (vfm_dwconv2d_fwd_mfma_gs): [B C upc][4] {count, shift, sum (x - shift),
    // sum (x - shift)^2} per producer wave, upc per (sample, channel) plane; null: computed here
    const float* stats;
    int upc;
    __hip_bfloat16* pc;  // fp32 y only: its exact bf16 pieces [3][B C HW] (store_pieces8), or null
};

// (count, sum, sum of squares) of a (sample, group) about the shift of its first partial, merged from the
// producer's per-wave partials in double precision, in a fixed order (thread-strided then a fixed tree)
__device__ __forceinline__ void gn_merge_stats(const GnArgs& a, int bg, float& mean_out, float& rstd_out) {
    __shared__ double red[3][NT];
    const int cpg = a.C / a.G;
    const long long n_units = (long long)cpg * a.upc;
    const float* st = a.stats + (long long)bg * n_units * 4;    // (b, g) units are consecutive: (b C + g cpg) upc
    const double S = st[1];
    double n = 0.0, s1 = 0.0, s2 = 0.0;
    for (long long u = threadIdx.x; u < n_units; u += NT) {
        const float4 v = *reinterpret_cast<const float4*>(st + 4 * u);
        const double c = v.x, d = (double)v.y - S;
        n += c;
        s1 += (double)v.z + c * d;
        s2 += (double)v.w + 2.0 * d * (double)v.z + c * d * d;
    }
    red[0][threadIdx.x] = n;
    red[1][threadIdx.x] = s1;
    red[2][threadIdx.x] = s2;
    __syncthreads();
    for (int w = NT / 2; w >= 1; w >>= 1) {
        if ((int)threadIdx.x < w) {
#pragma unroll
            for (int k = 0; k < 3; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + w];
        }
        __syncthreads();
    }
    const double m1 = red[1][0] / red[0][0];
    const double var = fmax(red[2][0] / red[0][0] - m1 * m1, 0.0);
    mean_out = (float)(S + m1);
    rstd_out = rsqrtf((float)var + a.eps);
}

// Flat forms (8 | HW, HW / 8 a power of two, at most GN_FLAT_MAX channels per group): the
// group is walked as one run of 8-element chunks by all threads instead of channel by channel
// (which left most threads idle on planes under 2048 elements and cost two barriers per channel).
// the three bf16 pieces (hi, mid, lo) of 8 consecutive fp32 outputs at element offset off of a planar
// [3][n] piece array: bit-identical to csrc/gemm8.hip split_planar_kernel<3> over the same values
__device__ __forceinline__ void store_pieces8(__hip_bfloat16* pc, long long n, long long off, const float (&v)[8]) {
    uint32_t q[4][3];
#pragma unroll
    for (int j = 0; j < 4; ++j) split_pieces<3>(v[2 * j], v[2 * j + 1], q[j]);
#pragma unroll
    for (int p = 0; p < 3; ++p)
        *reinterpret_cast<uint4*>(pc + (long long)p * n + off) = make_uint4(q[0][p], q[1][p], q[2][p], q[3][p]);
}

constexpr int GN_FLAT_MAX = 128;

template <class TI, class TO>
__global__ __launch_bounds__(NT) void gn_fwd(GnArgs a) {
    __shared__ float scratch[8];
    const int bg = blockIdx.x;
    const int bidx = bg / a.G, g = bg - bidx * a.G;
    const int cpg = a.C / a.G;
    const long long n = (long long)cpg * a.HW;
    const bool vec = (a.HW % 8) == 0;
    const TI* xp = reinterpret_cast<const TI*>(a.x) + (long long)bg * n;
    const long long nv = vec ? n / 8 : 0;
    float mean, rstd;
    if (a.stats) {
        gn_merge_stats(a, bg, mean, rstd);
    } else {
    // Shifted sums (shift = first element of the group) keep the one-pass variance accurate.
    const float shift = ld(xp);
    float s1 = 0.f, s2 = 0.f;
    // unrolled so that several 16-B loads per thread are in flight (the loop is latency-bound otherwise)
#pragma unroll 4
    for (long long i = threadIdx.x; i < nv; i += NT) {
        float v[8];
        load8(xp + i * 8, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float d = v[k] - shift;
            s1 += d;
            s2 = fmaf(d, d, s2);
        }
    }
    for (long long i = nv * 8 + threadIdx.x; i < n; i += NT) {
        const float d = ld(xp + i) - shift;
        s1 += d;
        s2 = fmaf(d, d, s2);
    }
    s1 = block_sum(s1, scratch);
    s2 = block_sum(s2, scratch + 4);
    const float m1 = s1 / (float)n;
    const float var = fmaxf(s2 / (float)n - m1 * m1, 0.f);
    mean = shift + m1;
    rstd = rsqrtf(var + a.eps);
    }
    if (threadIdx.x == 0) {
        a.mean[bg] = mean;
        a.rstd[bg] = rstd;
    }
    TO* yp = reinterpret_cast<TO*>(a.y) + (long long)bg * n;
    const int cpc = a.HW >> 3;                     // 8-element chunks per channel
    if (vec && cpg <= GN_FLAT_MAX && (cpc & (cpc - 1)) == 0) {
        // flat form: every thread walks the whole group in chunks, so small planes (8x8 ..
        // 32x32 in the fp32 blocks) keep all 256 threads busy; per-channel affine from LDS
        __shared__ float s_sc[GN_FLAT_MAX], s_sh[GN_FLAT_MAX];
        for (int cl = threadIdx.x; cl < cpg; cl += NT) {
            const int c = g * cpg + cl;
            float sc = rstd * (a.w ? a.w[c] : 1.f);
            float sh = (a.b ? a.b[c] : 0.f) - mean * sc;
            if (a.s) {
                const float m = a.s[bidx * a.C + c];
                sc *= m;
                sh *= m;
            }
            s_sc[cl] = sc;
            s_sh[cl] = sh;
        }
        __syncthreads();
        const int lg = __builtin_ctz(cpc);
#pragma unroll 4
        for (long long i = threadIdx.x; i < nv; i += NT) {
            const int cl = (int)(i >> lg);
            const float sc = s_sc[cl], sh = s_sh[cl];
            float v[8];
            load8(xp + i * 8, v);
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = fmaf(v[k], sc, sh);
            store8(yp + i * 8, v);
            if (std::is_same<TO, float>::value && a.pc)
                store_pieces8(a.pc, (long long)a.B * a.C * a.HW, (long long)bg * n + i * 8, v);
        }
        return;
    }
    for (int cl = 0; cl < cpg; ++cl) {
        const int c = g * cpg + cl;
        float sc = rstd * (a.w ? a.w[c] : 1.f);
        float sh = (a.b ? a.b[c] : 0.f) - mean * sc;
        if (a.s) {
            const float m = a.s[bidx * a.C + c];
            sc *= m;
            sh *= m;
        }
        const TI* xc = xp + (long long)cl * a.HW;
        TO* yc = yp + (long long)cl * a.HW;
        if (vec) {
            for (int i = threadIdx.x; i < a.HW / 8; i += NT) {
                float v[8];
                load8(xc + i * 8, v);
#pragma unroll
                for (int k = 0; k < 8; ++k) v[k] = fmaf(v[k], sc, sh);
                store8(yc + i * 8, v);
                if (std::is_same<TO, float>::value && a.pc)
                    store_pieces8(a.pc, (long long)a.B * a.C * a.HW, (long long)bg * n + (long long)cl * a.HW + i * 8, v);
            }
        } else {
            for (int i = threadIdx.x; i < a.HW; i += NT) st(yc + i, fmaf(ld(xc + i), sc, sh));
        }
    }
}

// Statistics-mode apply (vfm_group_norm_fwd_stats): with the statistics already merged from the producer's
// partials the pass is one read + one write of the group, so the group is split over gridDim.y blocks of
// GN_APPLY_VEC 8-element chunks each (the one-block-per-group form leaves ~4 waves per SIMD in flight at
// 1024 groups). Every block merges the (few) partials itself; block y == 0 writes mean/rstd.
constexpr int GN_APPLY_VEC = 2048;

template <class TI, class TO>
__global__ __launch_bounds__(NT) void gn_apply(GnArgs a) {
    __shared__ float s_sc[GN_FLAT_MAX], s_sh[GN_FLAT_MAX];
    const int bg = blockIdx.x;
    const int bidx = bg / a.G, g = bg - bidx * a.G;
    const int cpg = a.C / a.G;
    const long long n = (long long)cpg * a.HW;
    float mean, rstd;
    gn_merge_stats(a, bg, mean, rstd);
    if (threadIdx.x == 0 && blockIdx.y == 0) {
        a.mean[bg] = mean;
        a.rstd[bg] = rstd;
    }
    for (int cl = threadIdx.x; cl < cpg; cl += NT) {
        const int c = g * cpg + cl;
        float sc = rstd * (a.w ? a.w[c] : 1.f);
        float sh = (a.b ? a.b[c] : 0.f) - mean * sc;
        if (a.s) {
            const float m = a.s[bidx * a.C + c];
            sc *= m;
            sh *= m;
        }
        s_sc[cl] = sc;
        s_sh[cl] = sh;
    }
    __syncthreads();
    const TI* xp = reinterpret_cast<const TI*>(a.x) + (long long)bg * n;
    TO* yp = reinterpret_cast<TO*>(a.y) + (long long)bg * n;
    const int cpc = a.HW >> 3;
    const long long v0 = (long long)blockIdx.y * GN_APPLY_VEC;
    const long long v1 = min((long long)(n >> 3), v0 + GN_APPLY_VEC);
#pragma unroll 8
    for (long long i = v0 + threadIdx.x; i < v1; i += NT) {
        const int cl = (int)(i / cpc);
        const float sc = s_sc[cl], sh = s_sh[cl];
        float v[8];
        load8(xp + i * 8, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = fmaf(v[k], sc, sh);
        store8(yp + i * 8, v);
    }
}

struct GnBwdArgs {
    const void* x;
    const void* dy;
    const float* mean;
    const float* rstd;
    const float* w;
    const float* b;
    const float* s;
    void* dx;
    float* dw_part;   // [B, C]  sum_p dy*s*xhat
    float* db_part;   // [B, C]  sum_p dy*s
    float* ds;        // [B, C]  (if s)
    int B, C, G, HW;
};

// Flat backward. Pass 1: per-channel sums A_c = sum dy*xhat, B_c = sum dy with the group
// walked in chunks by all threads; a thread's partial sums are reduced over the lanes that share
// its channel (an aligned segment of min(HW/8, 64) lanes) whenever the wave moves to the next
// channel, and each wave stores its channel partial in its own LDS slot: every (wave, channel)
// slot has one writer, and the 4 wave slots are added in a fixed order -- deterministic.
template <class TX, class TY>
__device__ __forceinline__ void gn_bwd_flat(const GnBwdArgs& a, int bg, int bidx, int g, int cpg, int cpc,
                                            const TX* xp, const TY* gp, float mean, float rstd) {
    __shared__ float s_pa[4][GN_FLAT_MAX], s_pb[4][GN_FLAT_MAX], s_k[GN_FLAT_MAX];
    __shared__ float scratch[8];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int lg = __builtin_ctz(cpc);
    const long long nch = (long long)cpg * cpc;
    for (int i = threadIdx.x; i < 4 * GN_FLAT_MAX; i += NT) {
        (&s_pa[0][0])[i] = 0.f;
        (&s_pb[0][0])[i] = 0.f;
    }
    __syncthreads();
    const int seg = cpc < 64 ? cpc : 64;
    float sa = 0.f, sb = 0.f;
    // one chunk of lookahead: the next chunk's two 16-B loads are issued before this one is used (two chunks
    // ahead measured the same: the two passes together run at ~5.7 TB/s of actual reads + writes, r6bk)
    float xv[8], gv[8];
    if (threadIdx.x < nch) {
        load8(xp + threadIdx.x * 8, xv);
        load8(gp + threadIdx.x * 8, gv);
    }
    for (long long base = 0; base < nch; base += NT) {
        const long long i = base + threadIdx.x;
        float xn[8], gn[8];
        if (i + NT < nch) {
            load8(xp + (i + NT) * 8, xn);
            load8(gp + (i + NT) * 8, gn);
        }
        if (i < nch) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                sa = fmaf(gv[k], (xv[k] - mean) * rstd, sa);
                sb += gv[k];
            }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            xv[k] = xn[k];
            gv[k] = gn[k];
        }
        const long long w0 = base + 64 * wave;        // this wave's first chunk
        const bool flush = cpc < 64 || w0 + NT >= nch || ((w0 + NT) >> lg) != (w0 >> lg);
        if (flush) {                                  // wave-uniform
            for (int off = seg >> 1; off >= 1; off >>= 1) {
                sa += __shfl_xor(sa, off);
                sb += __shfl_xor(sb, off);
            }
            if ((lane & (seg - 1)) == 0 && i < nch) {
                const int cl = (int)(i >> lg);
                s_pa[wave][cl] = sa;
                s_pb[wave][cl] = sb;
            }
            sa = sb = 0.f;
        }
    }
    __syncthreads();
    float cx = 0.f, cxx = 0.f;
    for (int cl = threadIdx.x; cl < cpg; cl += NT) {
        const float A = (s_pa[0][cl] + s_pa[1][cl]) + (s_pa[2][cl] + s_pa[3][cl]);
        const float Bs = (s_pb[0][cl] + s_pb[1][cl]) + (s_pb[2][cl] + s_pb[3][cl]);
        const int c = g * cpg + cl;
        const float wc = a.w ? a.w[c] : 1.f;
        const float sc = a.s ? a.s[bidx * a.C + c] : 1.f;
        cx += sc * wc * Bs;
        cxx += sc * wc * A;
        s_k[cl] = wc * sc;
        a.dw_part[bidx * a.C + c] = sc * A;
        a.db_part[bidx * a.C + c] = sc * Bs;
        if (a.ds) a.ds[bidx * a.C + c] = wc * A + (a.b ? a.b[c] : 0.f) * Bs;
    }
    const float n = (float)nch * 8.f;
    const float m1 = block_sum(cx, scratch) / n, m2 = block_sum(cxx, scratch + 4) / n;
    TX* dxp = reinterpret_cast<TX*>(a.dx) + (long long)bg * nch * 8;
    // pass 2 walks the group backwards: its first reads are the chunks pass 1 read last, still in L2 / MALL
#pragma unroll 4
    for (long long base = (nch - 1) / NT * NT; base >= 0; base -= NT) {
        const long long i = base + threadIdx.x;
        if (i >= nch) continue;
        const float k = s_k[(int)(i >> lg)];
        float xv[8], gv[8], o[8];
        load8(xp + i * 8, xv);
        load8(gp + i * 8, gv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float xh = (xv[j] - mean) * rstd;
            o[j] = rstd * (gv[j] * k - m1 - xh * m2);
        }
        store8(dxp + i * 8, o);
    }
}

// Per (sample, group) workgroup. Pass 1: per-channel sums A_c = sum dy*xhat, B_c = sum dy
// (channel loop, one workgroup reduction per channel). Pass 2: dx.
template <class TX, class TY>
__global__ __launch_bounds__(NT) void gn_bwd(GnBwdArgs a) {
    __shared__ float scratch[8];
    const int bg = blockIdx.x;
    const int bidx = bg / a.G, g = bg - bidx * a.G;
    const int cpg = a.C / a.G;
    const long long n = (long long)cpg * a.HW;
    const TX* xp = reinterpret_cast<const TX*>(a.x) + (long long)bg * n;
    const TY* gp = reinterpret_cast<const TY*>(a.dy) + (long long)bg * n;
    const float mean = a.mean[bg], rstd = a.rstd[bg];
    const bool vec = (a.HW % 8) == 0;
    const int cpc = a.HW >> 3;
    if (vec && cpg <= GN_FLAT_MAX && (cpc & (cpc - 1)) == 0) {
        gn_bwd_flat<TX, TY>(a, bg, bidx, g, cpg, cpc, xp, gp, mean, rstd);
        return;
    }
    float sum_dxhat = 0.f, sum_dxhat_xhat = 0.f;   // group sums (block-uniform)
    for (int cl = 0; cl < cpg; ++cl) {
        const TX* xc = xp + (long long)cl * a.HW;
        const TY* gc = gp + (long long)cl * a.HW;
        float sa = 0.f, sb = 0.f;
        if (vec) {
            for (int i = threadIdx.x; i < a.HW / 8; i += NT) {
                float xv[8], gv[8];
                load8(xc + i * 8, xv);
                load8(gc + i * 8, gv);
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    sa = fmaf(gv[k], (xv[k] - mean) * rstd, sa);
                    sb += gv[k];
                }
            }
        } else {
            for (int i = threadIdx.x; i < a.HW; i += NT) {
                const float gv = ld(gc + i);
                sa = fmaf(gv, (ld(xc + i) - mean) * rstd, sa);
                sb += gv;
            }
        }
        sa = block_sum(sa, scratch);
        sb = block_sum(sb, scratch + 4);
        const int c = g * cpg + cl;
        const float wc = a.w ? a.w[c] : 1.f;
        const float sc = a.s ? a.s[bidx * a.C + c] : 1.f;
        sum_dxhat += sc * wc * sb;
        sum_dxhat_xhat += sc * wc * sa;
        if (threadIdx.x == 0) {
            a.dw_part[bidx * a.C + c] = sc * sa;
            a.db_part[bidx * a.C + c] = sc * sb;
            if (a.ds) a.ds[bidx * a.C + c] = wc * sa + (a.b ? a.b[c] : 0.f) * sb;
        }
    }
    const float m1 = sum_dxhat / (float)n, m2 = sum_dxhat_xhat / (float)n;
    TX* dxp = reinterpret_cast<TX*>(a.dx) + (long long)bg * n;
    for (int cl = 0; cl < cpg; ++cl) {
        const int c = g * cpg + cl;
        const float k = (a.w ? a.w[c] : 1.f) * (a.s ? a.s[bidx * a.C + c] : 1.f);
        const TX* xc = xp + (long long)cl * a.HW;
        const TY* gc = gp + (long long)cl * a.HW;
        TX* dc = dxp + (long long)cl * a.HW;
        if (vec) {
            for (int i = threadIdx.x; i < a.HW / 8; i += NT) {
                float xv[8], gv[8], o[8];
                load8(xc + i * 8, xv);
                load8(gc + i * 8, gv);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float xh = (xv[j] - mean) * rstd;
                    o[j] = rstd * (gv[j] * k - m1 - xh * m2);
                }
                store8(dc + i * 8, o);
            }
        } else {
            for (int i = threadIdx.x; i < a.HW; i += NT) {
                const float xh = (ld(xc + i) - mean) * rstd;
                st(dc + i, rstd * (ld(gc + i) * k - m1 - xh * m2));
            }
        }
    }
}

// -------------------------------------------------------------------------------------------
// Row kernels on [R rows, P] with one wave per row (P % 8 == 0 required by the host).

// Exact-erf GELU (torch nn.GELU()). erff() from the device math library branches on |x| and
// costs ~25 VALU ops; with the backward's exp that made the GELU row kernels VALU-bound
// rather than HBM-bound. Here Phi(z) comes from the branch-free Abramowitz-Stegun 7.1.26
// form, |erf error| <= 1.5e-7 (about 1 fp32 ulp at 1.0): one v_rcp, one v_exp, five FMAs,
// and the exp(-z^2/2) it needs is the same factor the derivative's z*phi(z) term uses.
__device__ __forceinline__ float gelu_erf(float z) { return z * vfm::gelu_parts(z).cdf; }
__device__ __forceinline__ float gelu_erf_grad(float z) {
    const vfm::GeluParts g = vfm::gelu_parts(z);
    return g.cdf + g.zpdf;
}

struct RowArgs {
    const void* in0;      // h (gelu) | y (residual)
    const void* in1;      // -      | x_in
    const void* dout;
    void* out0;           // g | out | dh | dy
    const float* rscale;  // per-row [R] (gelu: s[b,o]) or null
    const float* cvec0;   // per-channel [O]: bias / b2
    const float* cvec1;   // per-channel [O]: - / gamma
    float* rsum0;         // per-row partial sums [R]
    float* rsum1;         // per-row partial sums [R]
    int R, O, P;
    __hip_bfloat16* pc;   // fp32 out0 only: its exact bf16 pieces [3][R P] (the f32x6 GEMMs' planar operand
                          // split, split_planar_kernel's layout and arithmetic) written with it, or null
};


template <class T>
__global__ __launch_bounds__(NT) void gelu_fwd(RowArgs a) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= a.R) return;
    const int lane = threadIdx.x & 63;
    const int o = row % a.O;
    const float sc = a.rscale ? a.rscale[row] : 1.f;
    const float bi = a.cvec0 ? a.cvec0[o] : 0.f;
    const T* __restrict__ hp = reinterpret_cast<const T*>(a.in0) + (long long)row * a.P;
    T* __restrict__ gp = reinterpret_cast<T*>(a.out0) + (long long)row * a.P;
#pragma unroll 4
    for (int i = lane; i < a.P / 8; i += 64) {
        float v[8];
        load8(hp + i * 8, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = gelu_erf(fmaf(v[k], sc, bi));
        store8(gp + i * 8, v);
        if (std::is_same<T, float>::value && a.pc)
            store_pieces8(a.pc, (long long)a.R * a.P, (long long)row * a.P + i * 8, v);
    }
}

// dz = dg * gelu'(h*s+b); dh = dz * s; rsum0[row] = sum dz*h (-> d_scale); rsum1[row] = sum dz (-> d_bias)
template <class T>
__global__ __launch_bounds__(NT) void gelu_bwd(RowArgs a) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= a.R) return;
    const int lane = threadIdx.x & 63;
    const int o = row % a.O;
    const float sc = a.rscale ? a.rscale[row] : 1.f;
    const float bi = a.cvec0 ? a.cvec0[o] : 0.f;
    const T* __restrict__ hp = reinterpret_cast<const T*>(a.in0) + (long long)row * a.P;
    const T* __restrict__ gp = reinterpret_cast<const T*>(a.dout) + (long long)row * a.P;
    T* __restrict__ dp = reinterpret_cast<T*>(a.out0) + (long long)row * a.P;
    float s0 = 0.f, s1 = 0.f;
#pragma unroll 4
    for (int i = lane; i < a.P / 8; i += 64) {
        float h[8], g[8], d[8];
        load8(hp + i * 8, h);
        load8(gp + i * 8, g);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float dz = g[k] * gelu_erf_grad(fmaf(h[k], sc, bi));
            s0 = fmaf(dz, h[k], s0);
            s1 += dz;
            d[k] = dz * sc;
        }
        store8(dp + i * 8, d);
        if (std::is_same<T, float>::value && a.pc)
            store_pieces8(a.pc, (long long)a.R * a.P, (long long)row * a.P + i * 8, d);
    }
    s0 = wave_sum(s0);
    s1 = wave_sum(s1);
    if (lane == 0) {
        if (a.rsum0) a.rsum0[row] = s0;
        a.rsum1[row] = s1;
    }
}

// out = x_in + gamma[c] * (y + b[c]);  TY = dtype of y, TX = dtype of x_in / out
template <class TY, class TX>
__global__ __launch_bounds__(NT) void lsr_fwd(RowArgs a) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= a.R) return;
    const int lane = threadIdx.x & 63;
    const int c = row % a.O;
    const float b = a.cvec0 ? a.cvec0[c] : 0.f;
    const float gm = a.cvec1 ? a.cvec1[c] : 1.f;
    const TY* __restrict__ yp = reinterpret_cast<const TY*>(a.in0) + (long long)row * a.P;
    const TX* __restrict__ xp = reinterpret_cast<const TX*>(a.in1) + (long long)row * a.P;
    TX* __restrict__ op = reinterpret_cast<TX*>(a.out0) + (long long)row * a.P;
#pragma unroll 4
    for (int i = lane; i < a.P / 8; i += 64) {
        float y[8], x[8];
        load8(yp + i * 8, y);
        load8(xp + i * 8, x);
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = fmaf(gm, y[k] + b, x[k]);
        store8(op + i * 8, x);
    }
}

// dy = gamma*dout (dtype TY); rsum0[row] = sum (y+b)*dout (-> d_gamma); rsum1[row] = sum dout (-> d_b / gamma)
template <class TY, class TX>
__global__ __launch_bounds__(NT) void lsr_bwd(RowArgs a) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= a.R) return;
    const int lane = threadIdx.x & 63;
    const int c = row % a.O;
    const float b = a.cvec0 ? a.cvec0[c] : 0.f;
    const float gm = a.cvec1 ? a.cvec1[c] : 1.f;
    const TY* __restrict__ yp = reinterpret_cast<const TY*>(a.in0) + (long long)row * a.P;
    const TX* __restrict__ gp = reinterpret_cast<const TX*>(a.dout) + (long long)row * a.P;
    TY* __restrict__ dp = reinterpret_cast<TY*>(a.out0) + (long long)row * a.P;
    float s0 = 0.f, s1 = 0.f;
#pragma unroll 4
    for (int i = lane; i < a.P / 8; i += 64) {
        float y[8], g[8], d[8];
        load8(yp + i * 8, y);
        load8(gp + i * 8, g);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            s0 = fmaf(y[k] + b, g[k], s0);
            s1 += g[k];
            d[k] = gm * g[k];
        }
        store8(dp + i * 8, d);
        if (std::is_same<TY, float>::value && a.pc)
            store_pieces8(a.pc, (long long)a.R * a.P, (long long)row * a.P + i * 8, d);
    }
    s0 = wave_sum(s0);
    s1 = wave_sum(s1);
    if (lane == 0) {
        a.rsum0[row] = s0;
        a.rsum1[row] = s1;
    }
}

// -------------------------------------------------------------------------------------------
// PixelShuffle(r) + replicate pad + separable normalised blur (taps k, 1 <= K <= 8).

struct BlurArgs {
    const void* x;     // [B, C*r*r, H, W]  (pre-shuffle); r == 1: plain blur of [B, C, H, W]
    void* y;           // [B, C, H*r, W*r]
    int B, C, H, W, r, K, pad0;
    float k[8];        // normalised 1-D taps (2-D kernel = k x k)
    // Adjoint edge terms (replicate padding folds the pad taps onto the border sample):
    // dS[0]   += sum_{o < P}   clo[o] dy[o],       clo[o] = sum_{t <= P-1-o} k[t]
    // dS[n-1] += sum_{m < Q}   chi[m] dy[n-1-m],   chi[m] = sum_{t >= P+1+m} k[t]
    // with P = (K-1)/2 pad before, Q = K-1-P pad after; every other sample is interior.
    float clo[8];
    float chi[8];
};

// Tiled forms: one workgroup = one (sample, channel) plane x a 64 x 32 tile of the
// (shuffled, full-resolution) image. The separable blur runs as a row pass then a column
// pass through LDS, so every input element is read from HBM once per tile (plus halo).
//
// Vector form (source width W % 8 == 0, every shape of the decoder): global memory is touched
// only in 8-element chunks (16 B for 16-bit types): the staged rows are whole chunks, and the
// column pass gives each thread one row x 8 consecutive destination elements, stored with one
// 16-B store. In the backward the destination is the pre-shuffle layout, so the row pass writes
// its result de-interleaved by sub-pixel column (R = 2: [even X | odd X]) and a thread's 8
// outputs are contiguous in both LDS and its source plane. The scalar form (2-byte accesses)
// remains for other widths.
constexpr int BTW = 64, BTH = 32;
constexpr int SBW = BTW + 4;          // padded LDS row stride of the row-pass result

// R (shuffle factor) is a template constant: the sub-pixel plane / low-res coordinate of a
// full-resolution (Y, X) are shifts and masks, not integer divisions.
template <class T, int R, int K>
__global__ __launch_bounds__(NT) void blur_fwd(BlurArgs a) {
    constexpr int P = (K - 1) / 2;
    constexpr int LW = BTW + K - 1, LH = BTH + K - 1;
    constexpr int SC = BTW / R + 16;                 // source columns kept per plane (vector form)
    constexpr int NS = LH * R * SC > LH * LW ? LH * R * SC : LH * LW;
    // staged source: the vector form's raw chunks of the R sub-pixel planes (sS) or the scalar
    // form's clamped, shuffled window (sA); the row pass writes sB
    __shared__ __attribute__((aligned(16))) float sStage[NS];
    __shared__ __attribute__((aligned(16))) float sB[LH * SBW];
    float* sS = sStage;
    float* sA = sStage;
    const int Ho = a.H * R, Wo = a.W * R;
    const int tilesX = (Wo + BTW - 1) / BTW, tilesY = (Ho + BTH - 1) / BTH;
    int bid = blockIdx.x;
    const int tx = bid % tilesX; bid /= tilesX;
    const int ty = bid % tilesY; bid /= tilesY;
    const int c = bid % a.C, b = bid / a.C;
    const int X0 = tx * BTW, Y0 = ty * BTH;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long long plane = (long long)a.H * a.W;
    // the R*R source planes of output channel c of sample b
    const T* xb = reinterpret_cast<const T*>(a.x) + ((long long)b * a.C + c) * (R * R) * plane;
    float k[K];
#pragma unroll
    for (int t = 0; t < K; ++t) k[t] = a.k[t];
    const bool vec = (a.W & 7) == 0;
    if (vec) {
        // the window's source columns of the R sub-pixel planes of each staged row, as chunks
        const int c_lo = max(0, X0 / R - 8), c_hi = min(a.W, X0 / R + BTW / R + 8);
        const int nch = (c_hi - c_lo) >> 3;
        for (int i = threadIdx.x; i < LH * R * nch; i += NT) {
            const int ry = i / (R * nch), rem = i - ry * R * nch, pp = rem / nch, ch = rem - pp * nch;
            const int Y = min(max(Y0 + ry - P, 0), Ho - 1);
            const T* src = xb + ((Y % R) * R + pp) * plane + (long long)(Y / R) * a.W + c_lo + 8 * ch;
            float v[8];
            load8(src, v);
            float* d = sS + (ry * R + pp) * SC + 8 * ch;
#pragma unroll
            for (int e = 0; e < 8; ++e) d[e] = v[e];
        }
        __syncthreads();
        // row pass straight from the raw chunks: tap t of output column X0 + lane reads source
        // column clamp(X0 + lane + t - P) of its sub-pixel plane (offsets fixed per lane)
        int idx[K];
#pragma unroll
        for (int t = 0; t < K; ++t) {
            const int X = min(max(X0 + lane + t - P, 0), Wo - 1);
            idx[t] = (X % R) * SC + X / R - c_lo;
        }
        for (int r = wave; r < LH; r += 4) {
            const float* row = sS + r * R * SC;
            float acc = 0.f;
#pragma unroll
            for (int t = 0; t < K; ++t) acc = fmaf(k[t], row[idx[t]], acc);
            sB[r * SBW + lane] = acc;
        }
    } else {
        // Stage the replicate-clamped source window, one row per wave-iteration.
        for (int ry = wave; ry < LH; ry += 4) {
            const int Y = min(max(Y0 + ry - P, 0), Ho - 1);
            const T* src = xb + (Y % R) * R * plane + (long long)(Y / R) * a.W;
            for (int rx = lane; rx < LW; rx += 64) {
                const int X = min(max(X0 + rx - P, 0), Wo - 1);
                sA[ry * LW + rx] = ld(src + (X % R) * plane + X / R);
            }
        }
        __syncthreads();
        for (int r = wave; r < LH; r += 4) {
            float acc = 0.f;
#pragma unroll
            for (int t = 0; t < K; ++t) acc = fmaf(k[t], sA[r * LW + lane + t], acc);
            sB[r * SBW + lane] = acc;
        }
    }
    __syncthreads();
    T* yb = reinterpret_cast<T*>(a.y) + ((long long)b * a.C + c) * Ho * Wo;
    if (vec) {
        const int ry = threadIdx.x >> 3, cx = 8 * (threadIdx.x & 7);
        const int Y = Y0 + ry, X = X0 + cx;
        if (Y < Ho && X < Wo) {
            float o[8] = {};
#pragma unroll
            for (int t = 0; t < K; ++t) {
                const float4 u0 = *reinterpret_cast<const float4*>(sB + (ry + t) * SBW + cx);
                const float4 u1 = *reinterpret_cast<const float4*>(sB + (ry + t) * SBW + cx + 4);
                const float u[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] = fmaf(k[t], u[e], o[e]);
            }
            store8(yb + (long long)Y * Wo + X, o);
        }
        return;
    }
    const int X = X0 + lane;
    if (X >= Wo) return;
#pragma unroll
    for (int i = 0; i < BTH / 4; ++i) {
        const int ry = wave * (BTH / 4) + i;
        const int Y = Y0 + ry;
        if (Y < Ho) {
            float acc = 0.f;
#pragma unroll
            for (int t = 0; t < K; ++t) acc = fmaf(k[t], sB[(ry + t) * SBW + lane], acc);
            st(yb + (long long)Y * Wo + X, acc);
        }
    }
}

// Vector form as a strip: one workgroup walks BSTRIP tiles down a 64-column strip of the plane with
// the next tile's source chunks loaded into registers while the current tile's row and column passes
// run (the one-tile form issues its ~2 loads per thread and then waits on them with nothing to overlap:
// 2.7 TB/s at the 256^2 bf16 blocks). Same arithmetic, same order of the taps, as blur_fwd's vector form.
constexpr int BSTRIP = 4;
#ifndef BLUR_STRIP
#define BLUR_STRIP 1
#endif
#ifndef BLUR_STRIP_BWD
#define BLUR_STRIP_BWD 1
#endif

template <class T, int R, int K>
__global__ __launch_bounds__(NT) void blur_fwd_strip(BlurArgs a) {
    constexpr int P = (K - 1) / 2;
    constexpr int LH = BTH + K - 1;
    constexpr int SC = BTW / R + 16;                 // source columns kept per sub-pixel plane
    constexpr int NL = (LH * R * (SC / 8) + NT - 1) / NT;
    __shared__ __attribute__((aligned(16))) float sS[LH * R * SC];
    __shared__ __attribute__((aligned(16))) float sB[LH * SBW];
    const int Ho = a.H * R, Wo = a.W * R;
    const int tilesX = (Wo + BTW - 1) / BTW, tilesY = (Ho + BTH - 1) / BTH;
    const int strips = (tilesY + BSTRIP - 1) / BSTRIP;
    int bid = blockIdx.x;
    const int tx = bid % tilesX; bid /= tilesX;
    const int sy = bid % strips; bid /= strips;
    const int c = bid % a.C, b = bid / a.C;
    const int X0 = tx * BTW;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long long plane = (long long)a.H * a.W;
    const T* xb = reinterpret_cast<const T*>(a.x) + ((long long)b * a.C + c) * (R * R) * plane;
    float k[K];
#pragma unroll
    for (int t = 0; t < K; ++t) k[t] = a.k[t];
    const int c_lo = max(0, X0 / R - 8), c_hi = min(a.W, X0 / R + BTW / R + 8);
    const int nch = (c_hi - c_lo) >> 3;
    const int total = LH * R * nch;
    int lry[NL], lpp[NL], lch[NL];
#pragma unroll
    for (int u = 0; u < NL; ++u) {
        const int i = threadIdx.x + u * NT;
        lry[u] = i / (R * nch);
        const int rem = i - lry[u] * R * nch;
        lpp[u] = rem / nch;
        lch[u] = rem - lpp[u] * nch;
    }
    float v[NL][8];
    auto fetch = [&](int Y0) {
#pragma unroll
        for (int u = 0; u < NL; ++u) {
            if (threadIdx.x + u * NT < total) {
                const int Y = min(max(Y0 + lry[u] - P, 0), Ho - 1);
                load8(xb + ((Y % R) * R + lpp[u]) * plane + (long long)(Y / R) * a.W + c_lo + 8 * lch[u], v[u]);
            }
        }
    };
    int idx[K];
#pragma unroll
    for (int t = 0; t < K; ++t) {
        const int X = min(max(X0 + lane + t - P, 0), Wo - 1);
        idx[t] = (X % R) * SC + X / R - c_lo;
    }
    T* yb = reinterpret_cast<T*>(a.y) + ((long long)b * a.C + c) * Ho * Wo;
    const int ty0 = sy * BSTRIP, ty1 = min(tilesY, ty0 + BSTRIP);
    fetch(ty0 * BTH);
    for (int ty = ty0; ty < ty1; ++ty) {
        const int Y0 = ty * BTH;
#pragma unroll
        for (int u = 0; u < NL; ++u) {
            if (threadIdx.x + u * NT < total) {
                float* d = sS + (lry[u] * R + lpp[u]) * SC + 8 * lch[u];
                *reinterpret_cast<float4*>(d) = make_float4(v[u][0], v[u][1], v[u][2], v[u][3]);
                *reinterpret_cast<float4*>(d + 4) = make_float4(v[u][4], v[u][5], v[u][6], v[u][7]);
            }
        }
        __syncthreads();
        if (ty + 1 < ty1) fetch(Y0 + BTH);
        for (int r = wave; r < LH; r += 4) {
            const float* row = sS + r * R * SC;
            float acc = 0.f;
#pragma unroll
            for (int t = 0; t < K; ++t) acc = fmaf(k[t], row[idx[t]], acc);
            sB[r * SBW + lane] = acc;
        }
        __syncthreads();
        const int ry = threadIdx.x >> 3, cx = 8 * (threadIdx.x & 7);
        const int Y = Y0 + ry, X = X0 + cx;
        if (Y < Ho && X < Wo) {
            float o[8] = {};
#pragma unroll
            for (int t = 0; t < K; ++t) {
                const float4 u0 = *reinterpret_cast<const float4*>(sB + (ry + t) * SBW + cx);
                const float4 u1 = *reinterpret_cast<const float4*>(sB + (ry + t) * SBW + cx + 4);
                const float w8[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] = fmaf(k[t], w8[e], o[e]);
            }
            store8(yb + (long long)Y * Wo + X, o);
        }
    }
}

// Adjoint, separable: along each axis dS[s] = sum_t k[t] dout[s + P - t] (zero outside the
// image) for every sample, plus the replicate-padding fold at the two border samples
// (BlurArgs::clo / chi). dS is written straight into the pre-shuffle layout of dx.
template <class T, int R, int K>
__global__ __launch_bounds__(NT) void blur_bwd(BlurArgs a, const void* dout, void* dx) {
    constexpr int P = (K - 1) / 2, Q = K - 1 - P;
    constexpr int LH = BTH + K - 1;
    constexpr int SW = BTW + 16;       // staged dout columns X0 - 8 .. X0 + BTW + 8 (K <= 8: Q <= 4, P <= 3)
    __shared__ __attribute__((aligned(16))) float sA[LH * SW];
    __shared__ __attribute__((aligned(16))) float sB[LH * SBW];
    const int Ho = a.H * R, Wo = a.W * R;
    const int tilesX = (Wo + BTW - 1) / BTW, tilesY = (Ho + BTH - 1) / BTH;
    int bid = blockIdx.x;
    const int tx = bid % tilesX; bid /= tilesX;
    const int ty = bid % tilesY; bid /= tilesY;
    const int c = bid % a.C, b = bid / a.C;
    const int X0 = tx * BTW, Y0 = ty * BTH;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const T* gp = reinterpret_cast<const T*>(dout) + ((long long)b * a.C + c) * Ho * Wo;
    const bool vec = (a.W & 7) == 0;
    // sA row ry, column 8 - Q + rx <-> dout (Y0 - Q + ry, X0 - Q + rx), zero outside the image
    if (vec) {
        constexpr int NCH = SW / 8;
        for (int i = threadIdx.x; i < LH * NCH; i += NT) {
            const int ry = i / NCH, ch = i - ry * NCH;
            const int y = Y0 + ry - Q, x = X0 - 8 + 8 * ch;
            float v[8];
            if (y >= 0 && y < Ho && x >= 0 && x < Wo) {
                load8(gp + (long long)y * Wo + x, v);
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = 0.f;
            }
            float* d = sA + ry * SW + 8 * ch;
            *reinterpret_cast<float4*>(d) = make_float4(v[0], v[1], v[2], v[3]);
            *reinterpret_cast<float4*>(d + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
    } else {
        constexpr int LW = BTW + K - 1;
        for (int ry = wave; ry < LH; ry += 4) {
            const int y = Y0 + ry - Q;
            const bool yok = y >= 0 && y < Ho;
            for (int rx = lane; rx < LW; rx += 64) {
                const int x = X0 + rx - Q;
                sA[ry * SW + 8 - Q + rx] = (yok && x >= 0 && x < Wo) ? ld(gp + (long long)y * Wo + x) : 0.f;
            }
        }
    }
    __syncthreads();
    float kr[K];
#pragma unroll
    for (int j = 0; j < K; ++j) kr[j] = a.k[K - 1 - j];
    const int X = X0 + lane;
    // vector form, R = 2: row-pass column of X is [X even | X odd] de-interleaved
    const int bcol = (vec && R == 2) ? ((lane & 1) * (BTW / 2) + (lane >> 1)) : lane;
    for (int r = wave; r < LH; r += 4) {
        const float* row = sA + r * SW + 8 - Q;
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < K; ++j) acc = fmaf(kr[j], row[lane + j], acc);
        if (X == 0)
            for (int o = 0; o < P && o < Wo; ++o) acc = fmaf(a.clo[o], row[o + Q], acc);
        if (X == Wo - 1)
            for (int m = 0; m < Q && m < Wo; ++m) acc = fmaf(a.chi[m], row[lane - m + Q], acc);
        sB[r * SBW + bcol] = acc;
    }
    __syncthreads();
    const long long plane = (long long)a.H * a.W;
    T* dxc = reinterpret_cast<T*>(dx) + ((long long)b * a.C + c) * (R * R) * plane;
    if (vec) {
        const int ry = threadIdx.x >> 3, ch = threadIdx.x & 7;
        const int Y = Y0 + ry;
        // destination: 8 consecutive source-plane columns of sub-pixel column pp
        const int pp = R == 2 ? ch >> 2 : 0;
        const int col = R == 2 ? X0 / 2 + 8 * (ch & 3) : X0 + 8 * ch;
        if (Y >= Ho || col >= a.W) return;
        float o[8] = {};
        auto fma_row = [&](float w, int rr) {
            const float4 u0 = *reinterpret_cast<const float4*>(sB + rr * SBW + 8 * ch);
            const float4 u1 = *reinterpret_cast<const float4*>(sB + rr * SBW + 8 * ch + 4);
            const float u[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = fmaf(w, u[e], o[e]);
        };
#pragma unroll
        for (int j = 0; j < K; ++j) fma_row(kr[j], ry + j);
        if (Y == 0)
            for (int q = 0; q < P && q < Ho; ++q) fma_row(a.clo[q], q + Q);
        if (Y == Ho - 1)
            for (int m = 0; m < Q && m < Ho; ++m) fma_row(a.chi[m], ry - m + Q);
        store8(dxc + ((Y % R) * R + pp) * plane + (long long)(Y / R) * a.W + col, o);
        return;
    }
    if (X >= Wo) return;
    T* dxb = dxc + (X % R) * plane + X / R;
    for (int i = 0; i < BTH / 4; ++i) {
        const int ry = wave * (BTH / 4) + i;
        const int Y = Y0 + ry;
        if (Y >= Ho) break;
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < K; ++j) acc = fmaf(kr[j], sB[(ry + j) * SBW + lane], acc);
        if (Y == 0)
            for (int o = 0; o < P && o < Ho; ++o) acc = fmaf(a.clo[o], sB[(o + Q) * SBW + lane], acc);
        if (Y == Ho - 1)
            for (int m = 0; m < Q && m < Ho; ++m) acc = fmaf(a.chi[m], sB[(ry - m + Q) * SBW + lane], acc);
        st(dxb + (Y % R) * R * plane + (long long)(Y / R) * a.W, acc);
    }
}

// blur_bwd's vector form as a strip of BSTRIP tiles with the next tile's dout chunks in flight
// (the same pipelining as blur_fwd_strip; same arithmetic and tap order as blur_bwd).
template <class T, int R, int K>
__global__ __launch_bounds__(NT) void blur_bwd_strip(BlurArgs a, const void* dout, void* dx) {
    constexpr int P = (K - 1) / 2, Q = K - 1 - P;
    constexpr int LH = BTH + K - 1;
    constexpr int SW = BTW + 16;
    constexpr int NCH = SW / 8;
    constexpr int NL = (LH * NCH + NT - 1) / NT;
    __shared__ __attribute__((aligned(16))) float sA[LH * SW];
    __shared__ __attribute__((aligned(16))) float sB[LH * SBW];
    const int Ho = a.H * R, Wo = a.W * R;
    const int tilesX = (Wo + BTW - 1) / BTW, tilesY = (Ho + BTH - 1) / BTH;
    const int strips = (tilesY + BSTRIP - 1) / BSTRIP;
    int bid = blockIdx.x;
    const int tx = bid % tilesX; bid /= tilesX;
    const int sy = bid % strips; bid /= strips;
    const int c = bid % a.C, b = bid / a.C;
    const int X0 = tx * BTW;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const T* gp = reinterpret_cast<const T*>(dout) + ((long long)b * a.C + c) * Ho * Wo;
    float v[NL][8];
    auto fetch = [&](int Y0) {
#pragma unroll
        for (int u = 0; u < NL; ++u) {
            const int i = threadIdx.x + u * NT;
            const int ry = i / NCH, ch = i - ry * NCH;
            const int y = Y0 + ry - Q, x = X0 - 8 + 8 * ch;
            if (i < LH * NCH && y >= 0 && y < Ho && x >= 0 && x < Wo) {
                load8(gp + (long long)y * Wo + x, v[u]);
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) v[u][e] = 0.f;
            }
        }
    };
    float kr[K];
#pragma unroll
    for (int j = 0; j < K; ++j) kr[j] = a.k[K - 1 - j];
    const int X = X0 + lane;
    const int bcol = R == 2 ? ((lane & 1) * (BTW / 2) + (lane >> 1)) : lane;
    const long long plane = (long long)a.H * a.W;
    T* dxc = reinterpret_cast<T*>(dx) + ((long long)b * a.C + c) * (R * R) * plane;
    const int cry = threadIdx.x >> 3, cch = threadIdx.x & 7;
    const int pp = R == 2 ? cch >> 2 : 0;
    const int col = R == 2 ? X0 / 2 + 8 * (cch & 3) : X0 + 8 * cch;
    const int ty0 = sy * BSTRIP, ty1 = min(tilesY, ty0 + BSTRIP);
    fetch(ty0 * BTH);
    for (int ty = ty0; ty < ty1; ++ty) {
        const int Y0 = ty * BTH;
#pragma unroll
        for (int u = 0; u < NL; ++u) {
            const int i = threadIdx.x + u * NT;
            if (i < LH * NCH) {
                const int ry = i / NCH, ch = i - ry * NCH;
                float* d = sA + ry * SW + 8 * ch;
                *reinterpret_cast<float4*>(d) = make_float4(v[u][0], v[u][1], v[u][2], v[u][3]);
                *reinterpret_cast<float4*>(d + 4) = make_float4(v[u][4], v[u][5], v[u][6], v[u][7]);
            }
        }
        __syncthreads();
        if (ty + 1 < ty1) fetch(Y0 + BTH);
        for (int r = wave; r < LH; r += 4) {
            const float* row = sA + r * SW + 8 - Q;
            float acc = 0.f;
#pragma unroll
            for (int j = 0; j < K; ++j) acc = fmaf(kr[j], row[lane + j], acc);
            if (X == 0)
                for (int o = 0; o < P && o < Wo; ++o) acc = fmaf(a.clo[o], row[o + Q], acc);
            if (X == Wo - 1)
                for (int m = 0; m < Q && m < Wo; ++m) acc = fmaf(a.chi[m], row[lane - m + Q], acc);
            sB[r * SBW + bcol] = acc;
        }
        __syncthreads();
        const int Y = Y0 + cry;
        if (Y < Ho && col < a.W) {
            float o[8] = {};
            auto fma_row = [&](float w, int rr) {
                const float4 u0 = *reinterpret_cast<const float4*>(sB + rr * SBW + 8 * cch);
                const float4 u1 = *reinterpret_cast<const float4*>(sB + rr * SBW + 8 * cch + 4);
                const float u[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] = fmaf(w, u[e], o[e]);
            };
#pragma unroll
            for (int j = 0; j < K; ++j) fma_row(kr[j], cry + j);
            if (Y == 0)
                for (int q = 0; q < P && q < Ho; ++q) fma_row(a.clo[q], q + Q);
            if (Y == Ho - 1)
                for (int m = 0; m < Q && m < Ho; ++m) fma_row(a.chi[m], cry - m + Q);
            store8(dxc + ((Y % R) * R + pp) * plane + (long long)(Y / R) * a.W + col, o);
        }
    }
}

template <class T, int R>
int blur_launch_r(BlurArgs& a, int mode, const void* dout, void* dx, const dim3& g, hipStream_t st) {
    const bool strip = (a.W & 7) == 0 && (mode == 0 ? BLUR_STRIP : BLUR_STRIP_BWD);
    const int tilesX = (a.W * R + BTW - 1) / BTW, tilesY = (a.H * R + BTH - 1) / BTH;
    const dim3 gs((unsigned)((long long)tilesX * ((tilesY + BSTRIP - 1) / BSTRIP) * a.B * a.C));
#define BLUR_CASE(KK)                                                                        \
    case KK:                                                                                 \
        if (strip && mode == 0) VFM_LAUNCH((blur_fwd_strip<T, R, KK>), gs, dim3(NT), 0, st, a);   \
        else if (strip) VFM_LAUNCH((blur_bwd_strip<T, R, KK>), gs, dim3(NT), 0, st, a, dout, dx); \
        else if (mode == 0) VFM_LAUNCH((blur_fwd<T, R, KK>), g, dim3(NT), 0, st, a); \
        else VFM_LAUNCH((blur_bwd<T, R, KK>), g, dim3(NT), 0, st, a, dout, dx);      \
        break;
    switch (a.K) {
        BLUR_CASE(1) BLUR_CASE(2) BLUR_CASE(3) BLUR_CASE(4) BLUR_CASE(5) BLUR_CASE(6) BLUR_CASE(7) BLUR_CASE(8)
    default: return VFM_ERR_ARGS;
    }
#undef BLUR_CASE
    return launch_status();
}

template <class T>
int blur_launch(BlurArgs& a, int mode, const void* dout, void* dx, long long grid, hipStream_t st) {
    const dim3 g((unsigned)grid);
    // edge-fold weights of the adjoint (see BlurArgs)
    const int P = (a.K - 1) / 2, Q = a.K - 1 - P;
    for (int o = 0; o < 8; ++o) {
        a.clo[o] = 0.f;
        for (int t = 0; o < P && t <= P - 1 - o; ++t) a.clo[o] += a.k[t];
        a.chi[o] = 0.f;
        for (int t = P + 1 + o; o < Q && t < a.K; ++t) a.chi[o] += a.k[t];
    }
    if (a.r == 1) return blur_launch_r<T, 1>(a, mode, dout, dx, g, st);
    if (a.r == 2) return blur_launch_r<T, 2>(a, mode, dout, dx, g, st);
    return VFM_ERR_ARGS;
}

// dw[c, t] = sum_r partial[r, c, t] (t < KK), db[c] = sum_r partial[r, c, KK]; rows in order
__global__ __launch_bounds__(256) void dw_wgrad_reduce(const float* __restrict__ partial, float* __restrict__ dw,
                                                       float* __restrict__ db, int rows, int C, int KK) {
    const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
    if (e >= (long long)C * (KK + 1)) return;
    const int c = (int)(e / (KK + 1)), t = (int)(e - (long long)c * (KK + 1));
    float s = 0.f;
    for (int r = 0; r < rows; ++r) s += partial[((long long)r * C + c) * (KK + 1) + t];
    if (t < KK) {
        if (dw) dw[(long long)c * KK + t] = s;
    } else if (db) {
        db[c] = s;
    }
}

// out_a[c] = scale_a[c] * sum_r a[r, c] (scale_a optional), out_b[c] = sum_r b[r, c] (b optional);
// rows summed in order (deterministic): the per-sample partials of the norm / layer-scale backward
__global__ __launch_bounds__(256) void colsum2(const float* __restrict__ a, const float* __restrict__ b,
                                               const float* __restrict__ scale_a, float* __restrict__ out_a,
                                               float* __restrict__ out_b, int rows, int cols) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= cols) return;
    float sa = 0.f, sb = 0.f;
    const bool wa = out_a != nullptr, wb = out_b != nullptr;
    // 16 rows' loads in flight per thread before they are summed (in row order): the loop was one
    // dependent L2 round trip per row
    for (int r0 = 0; r0 < rows; r0 += 16) {
        float va[16], vb[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const bool in = r0 + k < rows;
            const long long o = (long long)(r0 + k) * cols + c;
            va[k] = (wa && in) ? a[o] : 0.f;
            vb[k] = (wb && in) ? b[o] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            sa += va[k];
            sb += vb[k];
        }
    }
    if (wa) out_a[c] = scale_a ? sa * scale_a[c] : sa;
    if (wb) out_b[c] = sb;
}

}  // namespace

// ============================== C ABI ==========================================================

extern "C" int vfm_colsum2_f32(const float* a, const float* b, const float* scale_a, float* out_a, float* out_b,
                               int rows, int cols, void* stream) {
    if (rows <= 0 || cols <= 0 || (!out_a && !out_b) || (out_a && !a) || (out_b && !b)) return VFM_ERR_ARGS;
    VFM_LAUNCH(colsum2, dim3((cols + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a, b,
                       scale_a, out_a, out_b, rows, cols);
    return launch_status();
}

extern "C" int vfm_dwconv2d_wgrad_reduce(const float* partial, float* dw, float* db, int rows, int C, int KK,
                                         void* stream) {
    if (!partial || rows <= 0 || C <= 0 || KK <= 0 || (!dw && !db)) return VFM_ERR_ARGS;
    const long long n = (long long)C * (KK + 1);
    VFM_LAUNCH(dw_wgrad_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), partial, dw, db, rows, C, KK);
    return launch_status();
}

extern "C" int vfm_dwconv2d_fwd_res(const void* x, const float* w, const float* bias, const float* noise,
                                    const void* res, void* y, int dtype, int B, int C, int H, int W, int K, int pad,
                                    int flip, void* stream) {
    if (!x || !w || !y || B <= 0 || C <= 0 || H <= 0 || W <= 0 || pad < 0) return VFM_ERR_ARGS;
    DwArgs a{};
    a.x = x; a.w = w; a.bias = bias; a.noise = noise; a.res = res; a.y = y;
    a.B = B; a.C = C; a.H = H; a.W = W; a.pad = pad; a.flip = flip != 0;
    a.Ho = H + 2 * pad - K + 1; a.Wo = W + 2 * pad - K + 1;
    if (a.Ho <= 0 || a.Wo <= 0) return VFM_ERR_ARGS;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    DwRowArgs r{};
    r.x = x; r.w = w; r.bias = bias; r.noise = noise; r.res = res; r.y = y; r.B = B; r.C = C; r.H = H; r.W = W;
    r.flip = flip != 0;
    if (dwr_plan(r, K, pad)) {
        switch (dtype) {
        case VFM_F32: return dwr_launch<float>(r, K, 0, st);
        case VFM_F16: return dwr_launch<__half>(r, K, 0, st);
        case VFM_BF16: return dwr_launch<__hip_bfloat16>(r, K, 0, st);
        }
        return VFM_ERR_ARGS;
    }
    dw_plan(a);
    switch (dtype) {
    case VFM_F32: return dw_dispatch<float>(a, K, 0, nullptr, nullptr, st);
    case VFM_F16: return dw_dispatch<__half>(a, K, 0, nullptr, nullptr, st);
    case VFM_BF16: return dw_dispatch<__hip_bfloat16>(a, K, 0, nullptr, nullptr, st);
    }
    return VFM_ERR_ARGS;
}

extern "C" int vfm_dwconv2d_fwd_ex(const void* x, const float* w, const float* bias, const float* noise, void* y,
                                   int dtype, int B, int C, int H, int W, int K, int pad, int flip, void* stream) {
    return vfm_dwconv2d_fwd_res(x, w, bias, noise, nullptr, y, dtype, B, C, H, W, K, pad, flip, stream);
}

extern "C" int vfm_dwconv2d_fwd(const void* x, const float* w, const float* bias, const float* noise, void* y,
                                int dtype, int B, int C, int H, int W, int K, int pad, void* stream) {
    return vfm_dwconv2d_fwd_ex(x, w, bias, noise, y, dtype, B, C, H, W, K, pad, 0, stream);
}

extern "C" int vfm_dwconv2d_bwd_weight_tiles(int B, int C, int H, int W, int K, int pad) {
    DwArgs a{};
    a.B = B; a.C = C; a.H = H; a.W = W; a.pad = pad;
    a.Ho = H + 2 * pad - K + 1; a.Wo = W + 2 * pad - K + 1;
    if (a.Ho <= 0 || a.Wo <= 0) return VFM_ERR_ARGS;
    DwRowArgs r{};
    r.B = B; r.C = C; r.H = H; r.W = W;
    if (dwr_plan(r, K, pad)) return r.wpc;       // partial [wpc, C, K*K+1]
    dw_plan(a);
    return a.tilesX * B;                          // partial [tilesX][B][C][K*K+1] = [tilesX*B, C, K*K+1]
}

extern "C" int vfm_dwconv2d_bwd_weight(const void* x, const void* dy, float* partial, int dtype, int B, int C, int H,
                                       int W, int K, int pad, void* stream) {
    if (!x || !dy || !partial || B <= 0 || C <= 0 || H <= 0 || W <= 0 || pad < 0) return VFM_ERR_ARGS;
    DwArgs a{};
    a.x = x; a.B = B; a.C = C; a.H = H; a.W = W; a.pad = pad;
    a.Ho = H + 2 * pad - K + 1; a.Wo = W + 2 * pad - K + 1;
    if (a.Ho <= 0 || a.Wo <= 0) return VFM_ERR_ARGS;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    DwRowArgs r{};
    r.x = x; r.dy = dy; r.partial = partial; r.B = B; r.C = C; r.H = H; r.W = W;
    if (dwr_plan(r, K, pad)) {
        switch (dtype) {
        case VFM_F32: return dwr_launch<float>(r, K, 1, st);
        case VFM_F16: return dwr_launch<__half>(r, K, 1, st);
        case VFM_BF16: return dwr_launch<__hip_bfloat16>(r, K, 1, st);
        }
        return VFM_ERR_ARGS;
    }
    dw_plan(a);
    switch (dtype) {
    case VFM_F32: return dw_dispatch<float>(a, K, 1, dy, partial, st);
    case VFM_F16: return dw_dispatch<__half>(a, K, 1, dy, partial, st);
    case VFM_BF16: return dw_dispatch<__hip_bfloat16>(a, K, 1, dy, partial, st);
    }
    return VFM_ERR_ARGS;
}

template <class TI, class TO>
static int gn_fwd_launch(GnArgs& a, hipStream_t st) {
    VFM_LAUNCH((gn_fwd<TI, TO>), dim3(a.B * a.G), dim3(NT), 0, st, a);
    return launch_status();
}

extern "C" int vfm_group_norm_fwd_pc(const void* x, const float* w, const float* b, const float* s, void* y,
                                     void* y_pieces, float* mean, float* rstd, int dtype_in, int dtype_out, int B,
                                     int C, int G, int HW, float eps, void* stream) {
    if (!x || !y || !mean || !rstd || B <= 0 || C <= 0 || G <= 0 || C % G || HW <= 0) return VFM_ERR_ARGS;
    // pieces only on the vectorised paths (HW % 8 == 0) of an fp32 output
    if (y_pieces && (dtype_out != VFM_F32 || HW % 8 || (uintptr_t)y_pieces % 16)) return VFM_ERR_ARGS;
    GnArgs a{x, w, b, s, y, mean, rstd, B, C, G, HW, eps, nullptr, 0, (__hip_bfloat16*)y_pieces};
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define GN_CASE(DI, TI)                                                        \
    if (dtype_in == DI) {                                                      \
        if (dtype_out == VFM_F32) return gn_fwd_launch<TI, float>(a, st);      \
        if (dtype_out == VFM_BF16) return gn_fwd_launch<TI, __hip_bfloat16>(a, st); \
        if (dtype_out == VFM_F16) return gn_fwd_launch<TI, __half>(a, st);     \
    }
    GN_CASE(VFM_F32, float)
    GN_CASE(VFM_BF16, __hip_bfloat16)
    GN_CASE(VFM_F16, __half)
#undef GN_CASE
    return VFM_ERR_ARGS;
}

extern "C" int vfm_group_norm_fwd(const void* x, const float* w, const float* b, const float* s, void* y,
                                  float* mean, float* rstd, int dtype_in, int dtype_out, int B, int C, int G, int HW,
                                  float eps, void* stream) {
    return vfm_group_norm_fwd_pc(x, w, b, s, y, nullptr, mean, rstd, dtype_in, dtype_out, B, C, G, HW, eps, stream);
}

// vfm_group_norm_fwd with the statistics merged from a producer's per-wave partials (vfm_dwconv2d_fwd_mfma_gs:
// stats [B C upc][4]) instead of a first pass over x: x is read once.
extern "C" int vfm_group_norm_fwd_stats(const void* x, const float* w, const float* b, const float* s, void* y,
                                        float* mean, float* rstd, const float* stats, int upc, int dtype_in,
                                        int dtype_out, int B, int C, int G, int HW, float eps, void* stream) {
    if (!x || !y || !mean || !rstd || !stats || upc <= 0 || B <= 0 || C <= 0 || G <= 0 || C % G || HW <= 0)
        return VFM_ERR_ARGS;
    if ((uintptr_t)stats % 16) return VFM_ERR_ARGS;
    GnArgs a{x, w, b, s, y, mean, rstd, B, C, G, HW, eps, stats, upc};
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (HW % 8 == 0 && C / G <= GN_FLAT_MAX) {
        const long long nv = (long long)(C / G) * HW / 8;
        const dim3 grid(B * G, (unsigned)((nv + GN_APPLY_VEC - 1) / GN_APPLY_VEC));
        if (dtype_in == VFM_BF16 && dtype_out == VFM_BF16)
            VFM_LAUNCH((gn_apply<__hip_bfloat16, __hip_bfloat16>), grid, dim3(NT), 0, st, a);
        else if (dtype_in == VFM_BF16 && dtype_out == VFM_F32)
            VFM_LAUNCH((gn_apply<__hip_bfloat16, float>), grid, dim3(NT), 0, st, a);
        else
            return VFM_NO_KERNEL;
        return launch_status();
    }
    if (dtype_in == VFM_BF16 && dtype_out == VFM_BF16) return gn_fwd_launch<__hip_bfloat16, __hip_bfloat16>(a, st);
    if (dtype_in == VFM_BF16 && dtype_out == VFM_F32) return gn_fwd_launch<__hip_bfloat16, float>(a, st);
    return VFM_NO_KERNEL;
}

template <class TX, class TY>
static int gn_bwd_launch(GnBwdArgs& a, hipStream_t st) {
    VFM_LAUNCH((gn_bwd<TX, TY>), dim3(a.B * a.G), dim3(NT), 0, st, a);
    return launch_status();
}

extern "C" int vfm_group_norm_bwd(const void* x, const void* dy, const float* mean, const float* rstd, const float* w,
                                  const float* b, const float* s, void* dx, float* dw_part, float* db_part, float* ds,
                                  int dtype_x, int dtype_dy, int B, int C, int G, int HW, void* stream) {
    if (!x || !dy || !mean || !rstd || !dx || !dw_part || !db_part || B <= 0 || C % G || HW <= 0) return VFM_ERR_ARGS;
    GnBwdArgs a{x, dy, mean, rstd, w, b, s, dx, dw_part, db_part, ds, B, C, G, HW};
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define GNB_CASE(DX, TX)                                                         \
    if (dtype_x == DX) {                                                         \
        if (dtype_dy == VFM_F32) return gn_bwd_launch<TX, float>(a, st);         \
        if (dtype_dy == VFM_BF16) return gn_bwd_launch<TX, __hip_bfloat16>(a, st); \
        if (dtype_dy == VFM_F16) return gn_bwd_launch<TX, __half>(a, st);        \
    }
    GNB_CASE(VFM_F32, float)
    GNB_CASE(VFM_BF16, __hip_bfloat16)
    GNB_CASE(VFM_F16, __half)
#undef GNB_CASE
    return VFM_ERR_ARGS;
}

extern "C" int vfm_scale_bias_gelu_fwd_pc(const void* h, const float* scale, const float* bias, void* g,
                                          void* g_pieces, int dtype, int B, int O, int P, void* stream) {
    if (!h || !g || B <= 0 || O <= 0 || P <= 0 || P % 8) return VFM_ERR_ARGS;
    if (g_pieces && (dtype != VFM_F32 || (uintptr_t)g_pieces % 16)) return VFM_ERR_ARGS;
    RowArgs a{};
    a.in0 = h; a.out0 = g; a.rscale = scale; a.cvec0 = bias; a.R = B * O; a.O = O; a.P = P;
    a.pc = (__hip_bfloat16*)g_pieces;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    dim3 grid((a.R + 3) / 4);
    switch (dtype) {
    case VFM_F32: VFM_LAUNCH((gelu_fwd<float>), grid, dim3(NT), 0, st, a); break;
    case VFM_BF16: VFM_LAUNCH((gelu_fwd<__hip_bfloat16>), grid, dim3(NT), 0, st, a); break;
    case VFM_F16: VFM_LAUNCH((gelu_fwd<__half>), grid, dim3(NT), 0, st, a); break;
    default: return VFM_ERR_ARGS;
    }
    return launch_status();
}

extern "C" int vfm_scale_bias_gelu_fwd(const void* h, const float* scale, const float* bias, void* g, int dtype,
                                       int B, int O, int P, void* stream) {
    return vfm_scale_bias_gelu_fwd_pc(h, scale, bias, g, nullptr, dtype, B, O, P, stream);
}

extern "C" int vfm_scale_bias_gelu_bwd_pc(const void* h, const void* dg, const float* scale, const float* bias,
                                          void* dh, void* dh_pieces, float* d_scale_rows, float* d_bias_rows,
                                          int dtype, int B, int O, int P, void* stream) {
    if (!h || !dg || !dh || !d_bias_rows || B <= 0 || O <= 0 || P <= 0 || P % 8) return VFM_ERR_ARGS;
    if (dh_pieces && (dtype != VFM_F32 || (uintptr_t)dh_pieces % 16)) return VFM_ERR_ARGS;
    RowArgs a{};
    a.pc = (__hip_bfloat16*)dh_pieces;
    a.in0 = h; a.dout = dg; a.out0 = dh; a.rscale = scale; a.cvec0 = bias; a.rsum0 = d_scale_rows;
    a.rsum1 = d_bias_rows; a.R = B * O; a.O = O; a.P = P;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    dim3 grid((a.R + 3) / 4);
    switch (dtype) {
    case VFM_F32: VFM_LAUNCH((gelu_bwd<float>), grid, dim3(NT), 0, st, a); break;
    case VFM_BF16: VFM_LAUNCH((gelu_bwd<__hip_bfloat16>), grid, dim3(NT), 0, st, a); break;
    case VFM_F16: VFM_LAUNCH((gelu_bwd<__half>), grid, dim3(NT), 0, st, a); break;
    default: return VFM_ERR_ARGS;
    }
    return launch_status();
}

extern "C" int vfm_scale_bias_gelu_bwd(const void* h, const void* dg, const float* scale, const float* bias, void* dh,
                                       float* d_scale_rows, float* d_bias_rows, int dtype, int B, int O, int P,
                                       void* stream) {
    return vfm_scale_bias_gelu_bwd_pc(h, dg, scale, bias, dh, nullptr, d_scale_rows, d_bias_rows, dtype, B, O, P,
                                      stream);
}

#define LSR_DISPATCH(KERNEL)                                                                       \
    if (dtype_y == VFM_F32 && dtype_x == VFM_F32) VFM_LAUNCH((KERNEL<float, float>), grid, dim3(NT), 0, st, a); \
    else if (dtype_y == VFM_BF16 && dtype_x == VFM_BF16) VFM_LAUNCH((KERNEL<__hip_bfloat16, __hip_bfloat16>), grid, dim3(NT), 0, st, a); \
    else if (dtype_y == VFM_BF16 && dtype_x == VFM_F32) VFM_LAUNCH((KERNEL<__hip_bfloat16, float>), grid, dim3(NT), 0, st, a); \
    else if (dtype_y == VFM_F16 && dtype_x == VFM_F16) VFM_LAUNCH((KERNEL<__half, __half>), grid, dim3(NT), 0, st, a); \
    else if (dtype_y == VFM_F16 && dtype_x == VFM_F32) VFM_LAUNCH((KERNEL<__half, float>), grid, dim3(NT), 0, st, a); \
    else return VFM_ERR_ARGS;

extern "C" int vfm_layer_scale_residual_fwd(const void* y, const float* bias, const float* gamma, const void* x_in,
                                            void* out, int dtype_y, int dtype_x, int B, int C, int P, void* stream) {
    if (!y || !x_in || !out || B <= 0 || C <= 0 || P <= 0 || P % 8) return VFM_ERR_ARGS;
    RowArgs a{};
    a.in0 = y; a.in1 = x_in; a.out0 = out; a.cvec0 = bias; a.cvec1 = gamma; a.R = B * C; a.O = C; a.P = P;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    dim3 grid((a.R + 3) / 4);
    LSR_DISPATCH(lsr_fwd)
    return launch_status();
}

extern "C" int vfm_layer_scale_residual_bwd_pc(const void* y, const float* bias, const float* gamma,
                                               const void* dout, void* dy, void* dy_pieces, float* d_gamma_rows,
                                               float* d_sum_rows, int dtype_y, int dtype_x, int B, int C, int P,
                                               void* stream) {
    if (!y || !dout || !dy || !d_gamma_rows || !d_sum_rows || B <= 0 || C <= 0 || P <= 0 || P % 8) return VFM_ERR_ARGS;
    if (dy_pieces && (dtype_y != VFM_F32 || (uintptr_t)dy_pieces % 16)) return VFM_ERR_ARGS;
    RowArgs a{};
    a.pc = (__hip_bfloat16*)dy_pieces;
    a.in0 = y; a.dout = dout; a.out0 = dy; a.cvec0 = bias; a.cvec1 = gamma; a.rsum0 = d_gamma_rows;
    a.rsum1 = d_sum_rows; a.R = B * C; a.O = C; a.P = P;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    dim3 grid((a.R + 3) / 4);
    LSR_DISPATCH(lsr_bwd)
    return launch_status();
}
#undef LSR_DISPATCH

extern "C" int vfm_layer_scale_residual_bwd(const void* y, const float* bias, const float* gamma, const void* dout,
                                            void* dy, float* d_gamma_rows, float* d_sum_rows, int dtype_y, int dtype_x,
                                            int B, int C, int P, void* stream) {
    return vfm_layer_scale_residual_bwd_pc(y, bias, gamma, dout, dy, nullptr, d_gamma_rows, d_sum_rows, dtype_y,
                                           dtype_x, B, C, P, stream);
}

extern "C" int vfm_shuffle_blur_fwd(const void* x, void* y, const float* taps, int K, int dtype, int B, int C, int H,
                                    int W, int r, void* stream) {
    if (!x || !y || !taps || K < 1 || K > 8 || r < 1 || B <= 0 || C <= 0 || H <= 0 || W <= 0) return VFM_ERR_ARGS;
    BlurArgs a{};
    a.x = x; a.y = y; a.B = B; a.C = C; a.H = H; a.W = W; a.r = r; a.K = K; a.pad0 = (K - 1) / 2;
    for (int i = 0; i < K; ++i) a.k[i] = taps[i];
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const long long grid = (long long)((W * r + BTW - 1) / BTW) * ((H * r + BTH - 1) / BTH) * B * C;
    switch (dtype) {
    case VFM_F32: return blur_launch<float>(a, 0, nullptr, nullptr, grid, st);
    case VFM_BF16: return blur_launch<__hip_bfloat16>(a, 0, nullptr, nullptr, grid, st);
    case VFM_F16: return blur_launch<__half>(a, 0, nullptr, nullptr, grid, st);
    }
    return VFM_ERR_ARGS;
}

extern "C" int vfm_shuffle_blur_bwd(const void* dout, void* dx, const float* taps, int K, int dtype, int B, int C,
                                    int H, int W, int r, void* stream) {
    if (!dout || !dx || !taps || K < 1 || K > 8 || r < 1 || B <= 0 || C <= 0 || H <= 0 || W <= 0) return VFM_ERR_ARGS;
    BlurArgs a{};
    a.B = B; a.C = C; a.H = H; a.W = W; a.r = r; a.K = K; a.pad0 = (K - 1) / 2;
    for (int i = 0; i < K; ++i) a.k[i] = taps[i];
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const long long grid = (long long)((W * r + BTW - 1) / BTW) * ((H * r + BTH - 1) / BTH) * B * C;
    switch (dtype) {
    case VFM_F32: return blur_launch<float>(a, 1, dout, dx, grid, st);
    case VFM_BF16: return blur_launch<__hip_bfloat16>(a, 1, dout, dx, grid, st);
    case VFM_F16: return blur_launch<__half>(a, 1, dout, dx, grid, st);
    }
    return VFM_ERR_ARGS;
}
