// upfirdn2d for gfx950: zero-insert upsample -> pad/crop -> FIR -> downsample -> gain.
//
// Semantics follow `_upfirdn2d_ref` (reference torch_utils/ops/upfirdn2d.py:166-211):
//   y[o] = gain * sum_t g[t] * u[o*down + t - pad0],   g = flip(f) unless flip_filter,
//   u[j] = x[j/up] if j % up == 0 (and in range) else 0,     per axis, 2-D product.
// For output o, the taps that hit real samples are t = t0 + k*up with
//   m = o*down - pad0, base = ceil(m/up), t0 = base*up - m,   input index = base + k.
//
// Two kernels:
//  * `updn_tile`: planar (NCHW-like, W stride 1) path. One 256-thread workgroup owns a
//    64x16 output tile of one (n,c) plane; the input tile + halo is staged through LDS
//    with W-coalesced loads (fp32 in LDS), the flipped filter sits in LDS, each lane
//    produces 4 output rows. Template on (up, down) so the tap stride is compile time.
//  * `updn_generic`: any strides (channels-last included) and any up/down; one lane per
//    output element, channel-fastest lane order when C has unit stride (coalesced).
#include "vfm_common.h"

namespace {

using namespace vfm;

constexpr int TW = 64;   // output tile width  (one wave-row)
constexpr int TH = 16;   // output tile height (4 rows per lane)
constexpr int NT = 256;

struct UpfirdnArgs {
    const void* x;
    void* y;
    const float* f;
    int N, C, inH, inW, outH, outW;
    long long xs[4], ys[4];
    int fh, fw;
    long long fsh, fsw;
    int upx, upy, downx, downy, padx0, pady0;
    int flip;
    float gain;
    int tilesX, tilesY;
    int tinW, tinH;  // LDS input tile extents (upper bound)
};

template <class T, int UPX, int UPY, int DX, int DY>
__global__ __launch_bounds__(NT) void updn_tile(UpfirdnArgs a) {
    typedef typename Acc<T>::type A;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    A* sx = reinterpret_cast<A*>(smem_raw);           // [tinH][tinW]
    A* sg = sx + a.tinH * a.tinW;                     // [fh][fw], already "g" (conv-flipped)

    int bid = blockIdx.x;
    const int tx = bid % a.tilesX; bid /= a.tilesX;
    const int ty = bid % a.tilesY; bid /= a.tilesY;
    const int plane = bid;                            // n*C + c
    const int n = plane / a.C, c = plane - (plane / a.C) * a.C;
    const int ox0 = tx * TW, oy0 = ty * TH;

    // Filter -> LDS as g[t] so that y = sum g[t] * u[o*down + t - pad].
    const int ftaps = a.fh * a.fw;
    for (int i = threadIdx.x; i < ftaps; i += NT) {
        int fy = i / a.fw, fx = i - (i / a.fw) * a.fw;
        int sy = a.flip ? fy : a.fh - 1 - fy;
        int sxx = a.flip ? fx : a.fw - 1 - fx;
        sg[i] = (A)a.f[sy * a.fsh + sxx * a.fsw];
    }

    // Input tile origin (first input sample any output of the tile touches).
    const int inX0 = ceil_div(ox0 * DX - a.padx0, UPX);
    const int inY0 = ceil_div(oy0 * DY - a.pady0, UPY);
    const T* xp = reinterpret_cast<const T*>(a.x) + (long long)n * a.xs[0] + (long long)c * a.xs[1];
    const int tin = a.tinW * a.tinH;
    for (int i = threadIdx.x; i < tin; i += NT) {
        int ry = i / a.tinW, rx = i - ry * a.tinW;
        int ix = inX0 + rx, iy = inY0 + ry;
        A v = 0;
        if (ix >= 0 && ix < a.inW && iy >= 0 && iy < a.inH)
            v = (A)ld(xp + (long long)iy * a.xs[2] + (long long)ix * a.xs[3]);
        sx[i] = v;
    }
    __syncthreads();

    const int lx = threadIdx.x & 63;
    const int ly = threadIdx.x >> 6;
    const int ox = ox0 + lx;
    if (ox >= a.outW) return;
    const int mx = ox * DX - a.padx0;
    const int bx = ceil_div(mx, UPX);
    const int t0x = bx * UPX - mx;
    const int rbx = bx - inX0;
    T* yp = reinterpret_cast<T*>(a.y) + (long long)n * a.ys[0] + (long long)c * a.ys[1] + (long long)ox * a.ys[3];

#pragma unroll
    for (int r = 0; r < TH / 4; ++r) {
        const int oy = oy0 + ly + 4 * r;
        if (oy >= a.outH) break;
        const int my = oy * DY - a.pady0;
        const int by = ceil_div(my, UPY);
        const int t0y = by * UPY - my;
        const int rby = by - inY0;
        A acc = 0;
        for (int ky = 0, t_y = t0y; t_y < a.fh; ++ky, t_y += UPY) {
            const A* srow = sx + (rby + ky) * a.tinW + rbx;
            const A* grow = sg + t_y * a.fw;
            for (int kx = 0, t_x = t0x; t_x < a.fw; ++kx, t_x += UPX)
                acc += srow[kx] * grow[t_x];
        }
        st(yp + (long long)oy * a.ys[2], acc * (A)a.gain);
    }
}

template <class T>
__global__ __launch_bounds__(NT) void updn_generic(UpfirdnArgs a, long long total, int chan_fastest) {
    typedef typename Acc<T>::type A;
    const T* x = reinterpret_cast<const T*>(a.x);
    T* y = reinterpret_cast<T*>(a.y);
    for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < total; i += (long long)gridDim.x * NT) {
        long long r = i;
        int n, c, oy, ox;
        if (chan_fastest) {
            c = (int)(r % a.C); r /= a.C;
            ox = (int)(r % a.outW); r /= a.outW;
            oy = (int)(r % a.outH); r /= a.outH;
            n = (int)r;
        } else {
            ox = (int)(r % a.outW); r /= a.outW;
            oy = (int)(r % a.outH); r /= a.outH;
            c = (int)(r % a.C); r /= a.C;
            n = (int)r;
        }
        const int mx = ox * a.downx - a.padx0, my = oy * a.downy - a.pady0;
        const int bx = ceil_div(mx, a.upx), by = ceil_div(my, a.upy);
        const int t0x = bx * a.upx - mx, t0y = by * a.upy - my;
        const T* xp = x + (long long)n * a.xs[0] + (long long)c * a.xs[1];
        A acc = 0;
        for (int ky = 0, t_y = t0y; t_y < a.fh; ++ky, t_y += a.upy) {
            const int iy = by + ky;
            if (iy < 0 || iy >= a.inH) continue;
            const int fy = a.flip ? t_y : a.fh - 1 - t_y;
            for (int kx = 0, t_x = t0x; t_x < a.fw; ++kx, t_x += a.upx) {
                const int ix = bx + kx;
                if (ix < 0 || ix >= a.inW) continue;
                const int fx = a.flip ? t_x : a.fw - 1 - t_x;
                acc += (A)ld(xp + (long long)iy * a.xs[2] + (long long)ix * a.xs[3]) *
                       (A)a.f[fy * a.fsh + fx * a.fsw];
            }
        }
        st(y + (long long)n * a.ys[0] + (long long)c * a.ys[1] + (long long)oy * a.ys[2] + (long long)ox * a.ys[3],
           acc * (A)a.gain);
    }
}

template <class T, int UPX, int UPY, int DX, int DY>
int launch_tile(UpfirdnArgs& a, size_t lds, hipStream_t st) {
    long long blocks = (long long)a.tilesX * a.tilesY * a.N * a.C;
    VFM_LAUNCH((updn_tile<T, UPX, UPY, DX, DY>), dim3((unsigned)blocks), dim3(NT), lds, st, a);
    return launch_status();
}

template <class T>
int run(UpfirdnArgs& a, hipStream_t st) {
    typedef typename Acc<T>::type A;
    const bool planar = (a.xs[3] == 1 && a.ys[3] == 1);
    const bool small_ud = (a.upx == a.upy && a.downx == a.downy) &&
                          (a.upx == 1 || a.upx == 2 || a.upx == 4) &&
                          (a.downx == 1 || a.downx == 2 || a.downx == 4);
    if (planar && small_ud) {
        a.tilesX = (a.outW + TW - 1) / TW;
        a.tilesY = (a.outH + TH - 1) / TH;
        a.tinW = ((TW - 1) * a.downx + a.upx - 1) / a.upx + 1 + (a.fw + a.upx - 1) / a.upx;
        a.tinH = ((TH - 1) * a.downy + a.upy - 1) / a.upy + 1 + (a.fh + a.upy - 1) / a.upy;
        size_t lds = sizeof(A) * ((size_t)a.tinW * a.tinH + (size_t)a.fh * a.fw);
        long long blocks = (long long)a.tilesX * a.tilesY * a.N * a.C;
        if (lds <= 64 * 1024 && blocks < (1ll << 31)) {
            const int u = a.upx, d = a.downx;
#define VFM_UD(U, D) if (u == U && d == D) return launch_tile<T, U, U, D, D>(a, lds, st);
            VFM_UD(1, 1) VFM_UD(1, 2) VFM_UD(1, 4)
            VFM_UD(2, 1) VFM_UD(2, 2) VFM_UD(2, 4)
            VFM_UD(4, 1) VFM_UD(4, 2) VFM_UD(4, 4)
#undef VFM_UD
        }
    }
    const long long total = (long long)a.N * a.C * a.outH * a.outW;
    const int chan_fastest = (a.xs[1] == 1 && a.C > 1) ? 1 : 0;
    long long blocks = (total + NT - 1) / NT;
    if (blocks > 2048 * 8) blocks = 2048 * 8;
    VFM_LAUNCH((updn_generic<T>), dim3((unsigned)blocks), dim3(NT), 0, st, a, total, chan_fastest);
    return launch_status();
}

}  // namespace

extern "C" int vfm_upfirdn2d(const void* x, void* y, const float* f, int dtype,
                             int N, int C, int inH, int inW, const long long* xs,
                             int outH, int outW, const long long* ys,
                             int fh, int fw, long long fsh, long long fsw,
                             int upx, int upy, int downx, int downy, int padx0, int pady0,
                             int flip, float gain, void* stream) {
    if (!x || !y || !f || !xs || !ys) return VFM_ERR_ARGS;
    if (N <= 0 || C <= 0 || inH <= 0 || inW <= 0 || outH <= 0 || outW <= 0) return VFM_ERR_ARGS;
    if (fh <= 0 || fw <= 0 || upx < 1 || upy < 1 || downx < 1 || downy < 1) return VFM_ERR_ARGS;
    UpfirdnArgs a;
    a.x = x; a.y = y; a.f = f;
    a.N = N; a.C = C; a.inH = inH; a.inW = inW; a.outH = outH; a.outW = outW;
    for (int i = 0; i < 4; ++i) { a.xs[i] = xs[i]; a.ys[i] = ys[i]; }
    a.fh = fh; a.fw = fw; a.fsh = fsh; a.fsw = fsw;
    a.upx = upx; a.upy = upy; a.downx = downx; a.downy = downy;
    a.padx0 = padx0; a.pady0 = pady0; a.flip = flip; a.gain = gain;
    a.tilesX = a.tilesY = a.tinW = a.tinH = 0;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    VFM_DISPATCH_FLOAT(dtype, T, return run<T>(a, st));
    return VFM_ERR_ARGS;
}
