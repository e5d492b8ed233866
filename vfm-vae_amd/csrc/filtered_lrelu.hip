// filtered_lrelu for gfx950: bias -> upsample FIR -> gain -> leaky ReLU -> clamp -> downsample FIR.
//
// Semantics = the reference's generic path (torch_utils/ops/filtered_lrelu.py:120-153 and
// :223-229): upfirdn2d(x + b, fu, up, pad, gain=up^2) -> act (gain, slope, clamp, 2-bit
// signs) -> upfirdn2d(., fd, down). Sign-tensor geometry follows filtered_lrelu.cpp:77-96
// (sh = yh*down-(down-1)+fdh-1 rows, width padded to 16 elements, 4 elements per byte,
// bit0 = negative, bit1 = clamped; bytes at/after ceil(sw_active/4) are don't-care).
//
// Fused design (not a translation of the reference's 27-row spec table): one 256-thread
// workgroup owns a TO x TO output tile of one (n,c) plane and keeps the whole chain in LDS:
//   input tile (+halo, bias added) -> intermediate tile (up-FIR, act, sign codes) -> output.
// Filters are passed as kernel arguments and staged per workgroup in LDS, so the op is
// stream-safe (the reference keeps them in a global __constant__ buffer, filtered_lrelu.cu:78,
// and warns about non-default streams, filtered_lrelu.py:215-216).
// Sign bytes are written only for the workgroup's *owned* intermediate rows/columns
// ([o0*down, (o0+TO)*down), the last tile owning the tail), so no two workgroups write one byte.
#include "vfm_common.h"

namespace {

using namespace vfm;

constexpr int NT = 256;

struct FlreluArgs {
    const void* x;
    const float* fu;
    const float* fd;
    const void* b;
    unsigned char* s;
    void* y;
    int N, C, xh, xw, yh, yw;
    long long xs[4], ys[4];
    int fuh, fuw, fdh, fdw;
    int px0, py0;
    int sh, swb, sx, sy;
    float gain, slope, clamp;
    int flip;
    int to;               // output tile edge
    int IW, IH, XW, XH;   // intermediate / input LDS tile extents
    int tilesX, tilesY;
};

template <class T, int UP, int DOWN, int MODE>
__global__ __launch_bounds__(NT) void flrelu_fused(FlreluArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    float* s_in = reinterpret_cast<float*>(smem_raw);          // [XH][XW]
    float* s_mid = s_in + a.XH * a.XW;                           // [IH][IW]
    float* s_gu = s_mid + a.IH * a.IW;                           // [fuh][fuw]
    float* s_gd = s_gu + a.fuh * a.fuw;                          // [fdh][fdw]
    unsigned char* s_code = reinterpret_cast<unsigned char*>(s_gd + a.fdh * a.fdw);  // [IH][IW]

    int bid = blockIdx.x;
    const int tx = bid % a.tilesX; bid /= a.tilesX;
    const int ty = bid % a.tilesY; bid /= a.tilesY;
    const int plane = bid;
    const int n = plane / a.C, c = plane - n * a.C;
    const int ox0 = tx * a.to, oy0 = ty * a.to;
    const int jx0 = ox0 * DOWN, jy0 = oy0 * DOWN;

    // Filters (conv orientation unless flip) -> LDS.
    for (int i = threadIdx.x; i < a.fuh * a.fuw; i += NT) {
        int fy = i / a.fuw, fx = i - fy * a.fuw;
        s_gu[i] = a.fu[(a.flip ? fy : a.fuh - 1 - fy) * a.fuw + (a.flip ? fx : a.fuw - 1 - fx)];
    }
    for (int i = threadIdx.x; i < a.fdh * a.fdw; i += NT) {
        int fy = i / a.fdw, fx = i - fy * a.fdw;
        s_gd[i] = a.fd[(a.flip ? fy : a.fdh - 1 - fy) * a.fdw + (a.flip ? fx : a.fdw - 1 - fx)];
    }

    // Input tile (+ bias) -> LDS.
    const int X0 = ceil_div(jx0 - a.px0, UP);
    const int Y0 = ceil_div(jy0 - a.py0, UP);
    const T* xp = reinterpret_cast<const T*>(a.x) + (long long)n * a.xs[0] + (long long)c * a.xs[1];
    const float bias = a.b ? (float)ld(reinterpret_cast<const T*>(a.b) + c) : 0.f;
    for (int i = threadIdx.x; i < a.XH * a.XW; i += NT) {
        int ry = i / a.XW, rx = i - ry * a.XW;
        int ix = X0 + rx, iy = Y0 + ry;
        float v = 0.f;
        if (ix >= 0 && ix < a.xw && iy >= 0 && iy < a.xh)
            v = (float)ld(xp + (long long)iy * a.xs[2] + (long long)ix * a.xs[3]) + bias;
        s_in[i] = v;
    }
    __syncthreads();

    // Intermediate tile: up-FIR (gain up^2), then gain / lrelu / clamp with sign handling.
    const float upg = (float)(UP * UP);
    const unsigned char* sp = a.s ? a.s + (long long)plane * a.sh * a.swb : nullptr;
    for (int i = threadIdx.x; i < a.IH * a.IW; i += NT) {
        int iy = i / a.IW, ix = i - iy * a.IW;
        int mx = jx0 + ix - a.px0, my = jy0 + iy - a.py0;
        int bx = ceil_div(mx, UP), by = ceil_div(my, UP);
        int t0x = bx * UP - mx, t0y = by * UP - my;
        int rbx = bx - X0, rby = by - Y0;
        float acc = 0.f;
        for (int ky = 0, tY = t0y; tY < a.fuh; ++ky, tY += UP) {
            const float* srow = s_in + (rby + ky) * a.XW + rbx;
            const float* grow = s_gu + tY * a.fuw;
            for (int kx = 0, tX = t0x; tX < a.fuw; ++kx, tX += UP) acc += srow[kx] * grow[tX];
        }
        float v = acc * upg * a.gain;
        unsigned char code = 0;
        if (MODE == 2) {
            int gx = jx0 + ix + a.sx, gy = jy0 + iy + a.sy;
            if ((unsigned)(gx >> 2) < (unsigned)a.swb && (unsigned)gy < (unsigned)a.sh) {
                int sc = sp[(long long)gy * a.swb + (gx >> 2)] >> ((gx & 3) << 1);
                if (sc & 1) v *= a.slope;
                if (sc & 2) v = 0.f;
            }
        } else {
            if (v < 0.f) { v *= a.slope; code = 1; }
            if (fabsf(v) > a.clamp) { v = fminf(fmaxf(v, -a.clamp), a.clamp); code = 2; }
        }
        s_mid[i] = v;
        if (MODE == 1) s_code[i] = code;
    }
    __syncthreads();

    // Sign bytes of the owned region.
    if (MODE == 1) {
        const bool lastX = (tx == a.tilesX - 1), lastY = (ty == a.tilesY - 1);
        const int ownWB = lastX ? (a.swb - jx0 / 4) : (a.to * DOWN) / 4;
        const int ownH = lastY ? (a.sh - jy0) : a.to * DOWN;
        unsigned char* wp = a.s + (long long)plane * a.sh * a.swb;
        for (int i = threadIdx.x; i < ownH * ownWB; i += NT) {
            int r = i / ownWB, q = i - r * ownWB;
            unsigned byte = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                int ix = 4 * q + e;
                if (ix < a.IW && r < a.IH) byte |= (unsigned)s_code[r * a.IW + ix] << (2 * e);
            }
            wp[(long long)(jy0 + r) * a.swb + (jx0 / 4 + q)] = (unsigned char)byte;
        }
    }

    // Down-FIR from the intermediate tile.
    T* yp = reinterpret_cast<T*>(a.y) + (long long)n * a.ys[0] + (long long)c * a.ys[1];
    for (int i = threadIdx.x; i < a.to * a.to; i += NT) {
        int ry = i / a.to, rx = i - ry * a.to;
        int ox = ox0 + rx, oy = oy0 + ry;
        if (ox >= a.yw || oy >= a.yh) continue;
        float acc = 0.f;
        for (int tY = 0; tY < a.fdh; ++tY) {
            const float* mrow = s_mid + (ry * DOWN + tY) * a.IW + rx * DOWN;
            const float* grow = s_gd + tY * a.fdw;
            for (int tX = 0; tX < a.fdw; ++tX) acc += mrow[tX] * grow[tX];
        }
        st(yp + (long long)oy * a.ys[2] + (long long)ox * a.ys[3], acc);
    }
}

template <class T, int UP, int DOWN>
int launch_ud(FlreluArgs& a, int mode, size_t lds, hipStream_t st) {
    long long blocks = (long long)a.tilesX * a.tilesY * a.N * a.C;
    dim3 g((unsigned)blocks), b(NT);
    if (mode == 0) VFM_LAUNCH((flrelu_fused<T, UP, DOWN, 0>), g, b, lds, st, a);
    else if (mode == 1) VFM_LAUNCH((flrelu_fused<T, UP, DOWN, 1>), g, b, lds, st, a);
    else VFM_LAUNCH((flrelu_fused<T, UP, DOWN, 2>), g, b, lds, st, a);
    return launch_status();
}

template <class T>
int run_fused(FlreluArgs& a, int up, int down, int mode, hipStream_t st) {
    a.to = (down == 4) ? 16 : 32;
    const int rw = ((a.to - 1) * down + a.fdw > a.to * down) ? (a.to - 1) * down + a.fdw : a.to * down;
    const int rh = ((a.to - 1) * down + a.fdh > a.to * down) ? (a.to - 1) * down + a.fdh : a.to * down;
    a.IW = (rw + 3) & ~3;
    a.IH = rh;
    a.XW = (a.IW + a.fuw - 1 + up - 1) / up + 1;
    a.XH = (a.IH + a.fuh - 1 + up - 1) / up + 1;
    a.tilesX = (a.yw + a.to - 1) / a.to;
    a.tilesY = (a.yh + a.to - 1) / a.to;
    size_t lds = 4 * ((size_t)a.XH * a.XW + (size_t)a.IH * a.IW + (size_t)a.fuh * a.fuw + (size_t)a.fdh * a.fdw) +
                 (mode == 1 ? (size_t)a.IH * a.IW : 0);
    if (lds > 64 * 1024) return VFM_NO_KERNEL;
    if ((long long)a.tilesX * a.tilesY * a.N * a.C >= (1ll << 31)) return VFM_NO_KERNEL;
#define VFM_UD(U, D) if (up == U && down == D) return launch_ud<T, U, D>(a, mode, lds, st);
    VFM_UD(1, 1) VFM_UD(1, 2) VFM_UD(1, 4)
    VFM_UD(2, 1) VFM_UD(2, 2) VFM_UD(2, 4)
    VFM_UD(4, 1) VFM_UD(4, 2) VFM_UD(4, 4)
#undef VFM_UD
    return VFM_NO_KERNEL;
}

// ---- in-place activation with sign write/read (generic path) ----

struct FlActArgs {
    void* x;
    unsigned char* s;
    int N, C, H, W;
    long long xs[4];
    int sh, swb, sx, sy;
    float gain, slope, clamp;
};

// One lane per element of the (sign-tensor or data) grid. In write mode each 4-lane
// group packs one byte with wave shuffles; the grid then spans the sign tensor so the
// padding columns are written as zero.
template <class T, int MODE>
__global__ __launch_bounds__(NT) void flrelu_act(FlActArgs a, int gridW, int gridH) {
    const long long total = (long long)a.N * a.C * gridH * gridW;
    for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i - (threadIdx.x & 63) < total;
         i += (long long)gridDim.x * NT) {
        const bool live = i < total;
        long long r = live ? i : 0;
        const int x = (int)(r % gridW); r /= gridW;
        const int y = (int)(r % gridH); r /= gridH;
        const int q = (int)r;
        const int n = q / a.C, c = q - n * a.C;
        unsigned code = 0;
        if (live && x < a.W && y < a.H) {
            T* p = reinterpret_cast<T*>(a.x) + (long long)n * a.xs[0] + (long long)c * a.xs[1] +
                   (long long)y * a.xs[2] + (long long)x * a.xs[3];
            typedef typename Acc<T>::type A;
            A v = (A)ld(p) * (A)a.gain;
            if (MODE == 2) {
                int gx = x + a.sx, gy = y + a.sy;
                if ((unsigned)(gx >> 2) < (unsigned)a.swb && (unsigned)gy < (unsigned)a.sh) {
                    int sc = a.s[((long long)q * a.sh + gy) * a.swb + (gx >> 2)] >> ((gx & 3) << 1);
                    if (sc & 1) v *= (A)a.slope;
                    if (sc & 2) v = 0;
                }
            } else {
                const A cl = (A)a.clamp;
                if (v < 0) { v *= (A)a.slope; code = 1; }
                if (fabs(v) > cl) { v = fmin(fmax(v, -cl), cl); code = 2; }
            }
            st(p, v);
        }
        if (MODE == 1) {
            // gridW is a multiple of 16 in write mode, so the 4 lanes of one byte are
            // consecutive lanes of one wave.
            unsigned packed = code << ((threadIdx.x & 3) << 1);
            packed |= __shfl_xor(packed, 1);
            packed |= __shfl_xor(packed, 2);
            if (live && (threadIdx.x & 3) == 0)
                a.s[((long long)q * a.sh + y) * a.swb + (x >> 2)] = (unsigned char)packed;
        }
    }
}

template <class T>
int run_act(FlActArgs& a, int mode, hipStream_t st) {
    const int gridW = (mode == 1) ? a.swb * 4 : a.W;
    const int gridH = (mode == 1) ? a.sh : a.H;
    const long long total = (long long)a.N * a.C * gridH * gridW;
    long long blocks = (total + NT - 1) / NT;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    dim3 g((unsigned)blocks), b(NT);
    if (mode == 0) VFM_LAUNCH((flrelu_act<T, 0>), g, b, 0, st, a, gridW, gridH);
    else if (mode == 1) VFM_LAUNCH((flrelu_act<T, 1>), g, b, 0, st, a, gridW, gridH);
    else VFM_LAUNCH((flrelu_act<T, 2>), g, b, 0, st, a, gridW, gridH);
    return launch_status();
}

}  // namespace

extern "C" int vfm_filtered_lrelu(const void* x, const float* fu, const float* fd, const void* b,
                                  unsigned char* s, void* y, int dtype,
                                  int N, int C, int xh, int xw, const long long* xs,
                                  int yh, int yw, const long long* ys,
                                  int fuh, int fuw, int fdh, int fdw,
                                  int up, int down, int px0, int py0,
                                  int sh, int sw_bytes, int sx, int sy, int sign_mode,
                                  float gain, float slope, float clamp, int flip, void* stream) {
    if (!x || !fu || !fd || !y || !xs || !ys) return VFM_ERR_ARGS;
    if (N <= 0 || C <= 0 || xh <= 0 || xw <= 0 || yh <= 0 || yw <= 0) return VFM_ERR_ARGS;
    if (fuh <= 0 || fuw <= 0 || fdh <= 0 || fdw <= 0 || up < 1 || down < 1) return VFM_ERR_ARGS;
    if (sign_mode < 0 || sign_mode > 2 || (sign_mode && (!s || sh <= 0 || sw_bytes <= 0))) return VFM_ERR_ARGS;
    if (dtype != VFM_F32 && dtype != VFM_F16 && dtype != VFM_BF16) return VFM_NO_KERNEL;
    if (!((up == 1 || up == 2 || up == 4) && (down == 1 || down == 2 || down == 4))) return VFM_NO_KERNEL;
    FlreluArgs a;
    a.x = x; a.fu = fu; a.fd = fd; a.b = b; a.s = s; a.y = y;
    a.N = N; a.C = C; a.xh = xh; a.xw = xw; a.yh = yh; a.yw = yw;
    for (int i = 0; i < 4; ++i) { a.xs[i] = xs[i]; a.ys[i] = ys[i]; }
    a.fuh = fuh; a.fuw = fuw; a.fdh = fdh; a.fdw = fdw;
    a.px0 = px0; a.py0 = py0;
    a.sh = sh; a.swb = sw_bytes; a.sx = sx; a.sy = sy;
    a.gain = gain; a.slope = slope; a.clamp = clamp; a.flip = flip;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    switch (dtype) {
    case VFM_F32: return run_fused<float>(a, up, down, sign_mode, st);
    case VFM_F16: return run_fused<__half>(a, up, down, sign_mode, st);
    case VFM_BF16: return run_fused<__hip_bfloat16>(a, up, down, sign_mode, st);
    }
    return VFM_NO_KERNEL;
}

extern "C" int vfm_filtered_lrelu_act(void* x, unsigned char* s, int dtype,
                                      int N, int C, int H, int W, const long long* xs,
                                      int sh, int sw_bytes, int sx, int sy, int sign_mode,
                                      float gain, float slope, float clamp, void* stream) {
    if (!x || !xs || N <= 0 || C <= 0 || H <= 0 || W <= 0) return VFM_ERR_ARGS;
    if (sign_mode < 0 || sign_mode > 2 || (sign_mode && (!s || sh <= 0 || sw_bytes <= 0))) return VFM_ERR_ARGS;
    FlActArgs a;
    a.x = x; a.s = s; a.N = N; a.C = C; a.H = H; a.W = W;
    for (int i = 0; i < 4; ++i) a.xs[i] = xs[i];
    a.sh = sh; a.swb = sw_bytes; a.sx = sx; a.sy = sy;
    a.gain = gain; a.slope = slope; a.clamp = clamp;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    switch (dtype) {
    case VFM_F32: return run_act<float>(a, sign_mode, st);
    case VFM_F16: return run_act<__half>(a, sign_mode, st);
    case VFM_BF16: return run_act<__hip_bfloat16>(a, sign_mode, st);
    case VFM_F64: return run_act<double>(a, sign_mode, st);
    }
    return VFM_ERR_ARGS;
}
