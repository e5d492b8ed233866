// im2col of a 2-D convolution (any kernel size, stride, zero padding; NCHW fp32) and its adjoint: the
// convolution of reference torch_utils/ops/conv2d_resample.py:46-141 (conv2d / conv_transpose2d through
// conv2d_gradfix.py:37-58, and the grouped per-sample form of generator.py:46-103 modulated_conv2d) as
// im2col + the exact-fp32 GEMM (csrc/sgemm.hip), instead of the library convolution:
//   cols[b, (c ky + ky) kw + kx, oy Wo + ox] = x[b, c, oy sy - py + ky, ox sx - px + kx]   (0 outside)
//   x[b, c, iy, ix]  = sum over (ky, kx, oy, ox) with oy sy - py + ky = iy, ox sx - px + kx = ix of cols[..]
// col2im is a gather (each image element sums the cols entries that read it): no atomics, deterministic.
// Rows of cols are (b, c, ky, kx) and run one wave each (the row's decomposition is wave-uniform); the
// lanes walk the row's Ho x Wo outputs with coalesced stores (reads strided by sx).
#include "vfm_common.h"

namespace {

using namespace vfm;

struct Geo {
    int B, C, H, W, kh, kw, sy, sx, py, px, Ho, Wo;
};

__global__ __launch_bounds__(256) void im2col2d_rows(const float* __restrict__ x, float* __restrict__ cols, Geo g,
                                                    long long rows) {
    const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);    // ((b C + c) kh + ky) kw + kx
    if (r >= rows) return;
    const int lane = threadIdx.x & 63;
    const int kx = (int)(r % g.kw);
    const long long r1 = r / g.kw;
    const int ky = (int)(r1 % g.kh);
    const long long bc = r1 / g.kh;
    const float* xp = x + bc * g.H * g.W;
    float* out = cols + r * (long long)g.Ho * g.Wo;
    const int P = g.Ho * g.Wo;
    for (int q = lane; q < P; q += 64) {
        const int oy = q / g.Wo, ox = q - oy * g.Wo;
        const int iy = oy * g.sy - g.py + ky, ix = ox * g.sx - g.px + kx;
        out[q] = (iy >= 0 && iy < g.H && ix >= 0 && ix < g.W) ? xp[iy * g.W + ix] : 0.f;
    }
}

__global__ __launch_bounds__(256) void col2im2d_rows(const float* __restrict__ cols, float* __restrict__ x, Geo g,
                                                    long long planes) {
    const long long bc = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);   // b C + c: one wave per image plane
    if (bc >= planes) return;
    const int lane = threadIdx.x & 63;
    const long long P = (long long)g.Ho * g.Wo;
    const float* cp = cols + bc * g.kh * g.kw * P;
    float* out = x + bc * g.H * g.W;
    const int HW = g.H * g.W;
    for (int t = lane; t < HW; t += 64) {
        const int iy = t / g.W, ix = t - iy * g.W;
        float acc = 0.f;
        for (int ky = 0; ky < g.kh; ++ky) {
            const int ny = iy + g.py - ky;                 // oy sy = ny
            if (ny < 0 || ny % g.sy) continue;
            const int oy = ny / g.sy;
            if (oy >= g.Ho) continue;
            for (int kx = 0; kx < g.kw; ++kx) {
                const int nx = ix + g.px - kx;
                if (nx < 0 || nx % g.sx) continue;
                const int ox = nx / g.sx;
                if (ox >= g.Wo) continue;
                acc += cp[(long long)(ky * g.kw + kx) * P + oy * g.Wo + ox];
            }
        }
        out[t] = acc;
    }
}

int geo_ok(const Geo& g) {
    return g.B > 0 && g.C > 0 && g.H > 0 && g.W > 0 && g.kh > 0 && g.kw > 0 && g.sy > 0 && g.sx > 0 && g.py >= 0 &&
           g.px >= 0 && g.Ho > 0 && g.Wo > 0 && g.Ho == (g.H + 2 * g.py - g.kh) / g.sy + 1 &&
           g.Wo == (g.W + 2 * g.px - g.kw) / g.sx + 1;
}

}  // namespace

// cols [B, C kh kw, Ho Wo] (fp32, contiguous) of x [B, C, H, W] (fp32, contiguous).
extern "C" int vfm_im2col2d_f32(const float* x, float* cols, int B, int C, int H, int W, int kh, int kw, int sy, int sx,
                                int py, int px, int Ho, int Wo, void* stream) {
    const Geo g{B, C, H, W, kh, kw, sy, sx, py, px, Ho, Wo};
    if (!x || !cols || !geo_ok(g)) return VFM_ERR_ARGS;
    const long long rows = (long long)B * C * kh * kw;
    VFM_LAUNCH(im2col2d_rows, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x, cols, g, rows);
    return launch_status();
}

// x [B, C, H, W] = the adjoint of vfm_im2col2d_f32 applied to cols [B, C kh kw, Ho Wo] (overwrites x).
extern "C" int vfm_col2im2d_f32(const float* cols, float* x, int B, int C, int H, int W, int kh, int kw, int sy, int sx,
                                int py, int px, int Ho, int Wo, void* stream) {
    const Geo g{B, C, H, W, kh, kw, sy, sx, py, px, Ho, Wo};
    if (!x || !cols || !geo_ok(g)) return VFM_ERR_ARGS;
    const long long planes = (long long)B * C;
    VFM_LAUNCH(col2im2d_rows, dim3((unsigned)((planes + 3) / 4)), dim3(256), 0, (hipStream_t)stream, cols, x, g,
               planes);
    return launch_status();
}
