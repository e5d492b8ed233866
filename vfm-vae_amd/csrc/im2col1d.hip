// im2col of a 1-D convolution with zero or circular padding, and its adjoint, fp32 (the projected
// discriminator heads' k = 9 SpectralConv1d with padding_mode='circular', reference
// networks/discriminator.py DiscHead / make_block: F.pad(circular) + unfold + permute + reshape in the
// GEMM formulation, ~4 kernels forward and ~6 backward (CopySlices, slice / unfold backward)).
//   cols[b, c k + j, l] = x[b, c, s],  s = l + j - p  (circular: mod L; zeros: 0 outside [0, L))
//   dx[b, c, t]        = sum_j dcols[b, c k + j, l_j(t)]   over the l that read t
// CBL = 1: the batch folded into the columns, cols[c k + j, b, l] ([C k, B Lo]): the whole batch's
// convolution is then one GEMM W [O, C k] x cols with K = C k, and its weight gradient one GEMM
// dY [O, B Lo] x cols^T with the batch in the reduction (no per-sample [O, C k] products to sum).
#include <cstdlib>

#include "vfm_common.h"

namespace {

using namespace vfm;

// One wave per row: the row's (b, c, j) decomposition is wave-uniform (no per-element 64-bit
// divisions), and the lanes walk the row's Lo (or L) elements with coalesced loads and stores.
template <int CBL>
__global__ __launch_bounds__(256) void im2col1d_rows(const float* __restrict__ x, float* __restrict__ cols, int B, int C,
                                                int L, int k, int p, int Lo, int circ, long long rows) {
    const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);   // CBL ? (c k + j) B + b : (b C + c) k + j
    if (r >= rows) return;
    const int lane = threadIdx.x & 63;
    int j;
    long long bc;
    if (CBL) {
        const int b = (int)(r % B);
        const long long cj = r / B;
        j = (int)(cj % k);
        bc = (long long)b * C + cj / k;
    } else {
        j = (int)(r % k);
        bc = r / k;
    }
    const float* xr = x + bc * L;
    float* out = cols + r * Lo;
    for (int l = lane; l < Lo; l += 64) {
        int s = l + j - p;
        float v = 0.f;
        if (circ) {
            if (s < 0) s += L;
            else if (s >= L) s -= L;                 // p <= L: one wrap at most
            v = xr[s];
        } else if (s >= 0 && s < L) {
            v = xr[s];
        }
        out[l] = v;
    }
}

template <int CBL>
__global__ __launch_bounds__(256) void col2im1d_rows(const float* __restrict__ dcols, float* __restrict__ dx, int B, int C,
                                                int L, int k, int p, int Lo, int circ, long long rows) {
    const long long bc = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);  // b C + c
    if (bc >= rows) return;
    const int lane = threadIdx.x & 63;
    // row j of (b, c): CBL ? ((c k + j) B + b) Lo : ((b C + c) k + j) Lo
    const long long jstride = CBL ? (long long)B * Lo : Lo;
    const float* dr = CBL ? dcols + (((bc % C) * k) * B + bc / C) * Lo : dcols + bc * k * Lo;
    float* out = dx + bc * L;
    for (int t = lane; t < L; t += 64) {
        float acc = 0.f;
        for (int j = 0; j < k; ++j) {
            int l = t - j + p;
            if (circ) {                              // Lo == L: exactly one l per (t, j)
                if (l < 0) l += L;
                else if (l >= L) l -= L;
            } else if (l < 0 || l >= Lo) {
                continue;
            }
            acc += dr[(long long)j * jstride + l];
        }
        out[t] = acc;
    }
}


// One thread per element (VFM_IM2COL_ROWS=0; the one-wave-per-row form is the default).
template <int CBL>
__global__ __launch_bounds__(256) void im2col1d_el(const float* __restrict__ x, float* __restrict__ cols, int B, int C,
                                                int L, int k, int p, int Lo, int circ, long long n) {
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
        const int l = (int)(e % Lo);
        const long long r = e / Lo;                  // CBL ? (c k + j) B + b : (b C + c) k + j
        int j;
        long long bc;
        if (CBL) {
            const int b = (int)(r % B);
            const long long cj = r / B;
            j = (int)(cj % k);
            bc = (long long)b * C + cj / k;
        } else {
            j = (int)(r % k);
            bc = r / k;
        }
        int s = l + j - p;
        float v = 0.f;
        if (circ) {
            s %= L;
            if (s < 0) s += L;
            v = x[bc * L + s];
        } else if (s >= 0 && s < L) {
            v = x[bc * L + s];
        }
        cols[e] = v;
    }
}

template <int CBL>
__global__ __launch_bounds__(256) void col2im1d_el(const float* __restrict__ dcols, float* __restrict__ dx, int B, int C,
                                                int L, int k, int p, int Lo, int circ, long long n) {
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
        const int t = (int)(e % L);
        const long long bc = e / L;
        // row j of (b, c): CBL ? ((c k + j) B + b) Lo : ((b C + c) k + j) Lo
        const long long jstride = CBL ? (long long)B * Lo : Lo;
        const float* dr = CBL ? dcols + (((bc % C) * k) * B + bc / C) * Lo : dcols + bc * k * Lo;
        float acc = 0.f;
        for (int j = 0; j < k; ++j) {
            int l = t - j + p;
            if (circ) {                              // Lo == L: exactly one l per (t, j)
                l %= L;
                if (l < 0) l += L;
            } else if (l < 0 || l >= Lo) {
                continue;
            }
            acc += dr[(long long)j * jstride + l];
        }
        dx[e] = acc;
    }
}

int grid_of(long long n) { return (int)std::min<long long>((n + 255) / 256, 16384); }

bool rows_form() {
    static const bool on = [] {
        const char* e = getenv("VFM_IM2COL_ROWS");
        return !(e && e[0] == '0');
    }();
    return on;
}

int im2col_launch(const float* x, float* cols, int B, int C, int L, int k, int p, int circular, int cbl,
                  void* stream) {
    if (!x || !cols || B <= 0 || C <= 0 || L <= 0 || k <= 0 || p < 0) return VFM_ERR_ARGS;
    const int Lo = L + 2 * p - k + 1;
    if (Lo <= 0 || (circular && (Lo != L || p > L))) return VFM_NO_KERNEL;
    if (!rows_form()) {
        const long long n = (long long)B * C * k * Lo;
        if (cbl)
            VFM_LAUNCH(im2col1d_el<1>, dim3(grid_of(n)), dim3(256), 0, (hipStream_t)stream, x, cols, B, C, L, k, p, Lo,
                       circular ? 1 : 0, n);
        else
            VFM_LAUNCH(im2col1d_el<0>, dim3(grid_of(n)), dim3(256), 0, (hipStream_t)stream, x, cols, B, C, L, k, p, Lo,
                       circular ? 1 : 0, n);
        return launch_status();
    }
    const long long rows = (long long)B * C * k;
    if ((rows + 3) / 4 > 0x7fffffffLL) return VFM_ERR_ARGS;
    const dim3 grid((unsigned)((rows + 3) / 4));
    if (cbl)
        VFM_LAUNCH(im2col1d_rows<1>, grid, dim3(256), 0, (hipStream_t)stream, x, cols, B, C, L, k, p, Lo,
                   circular ? 1 : 0, rows);
    else
        VFM_LAUNCH(im2col1d_rows<0>, grid, dim3(256), 0, (hipStream_t)stream, x, cols, B, C, L, k, p, Lo,
                   circular ? 1 : 0, rows);
    return launch_status();
}

int col2im_launch(const float* dcols, float* dx, int B, int C, int L, int k, int p, int circular, int cbl,
                  void* stream) {
    if (!dcols || !dx || B <= 0 || C <= 0 || L <= 0 || k <= 0 || p < 0) return VFM_ERR_ARGS;
    const int Lo = L + 2 * p - k + 1;
    if (Lo <= 0 || (circular && (Lo != L || p > L))) return VFM_NO_KERNEL;
    if (!rows_form()) {
        const long long n = (long long)B * C * L;
        if (cbl)
            VFM_LAUNCH(col2im1d_el<1>, dim3(grid_of(n)), dim3(256), 0, (hipStream_t)stream, dcols, dx, B, C, L, k, p,
                       Lo, circular ? 1 : 0, n);
        else
            VFM_LAUNCH(col2im1d_el<0>, dim3(grid_of(n)), dim3(256), 0, (hipStream_t)stream, dcols, dx, B, C, L, k, p,
                       Lo, circular ? 1 : 0, n);
        return launch_status();
    }
    const long long rows = (long long)B * C;
    if ((rows + 3) / 4 > 0x7fffffffLL) return VFM_ERR_ARGS;
    const dim3 grid((unsigned)((rows + 3) / 4));
    if (cbl)
        VFM_LAUNCH(col2im1d_rows<1>, grid, dim3(256), 0, (hipStream_t)stream, dcols, dx, B, C, L, k, p, Lo,
                   circular ? 1 : 0, rows);
    else
        VFM_LAUNCH(col2im1d_rows<0>, grid, dim3(256), 0, (hipStream_t)stream, dcols, dx, B, C, L, k, p, Lo,
                   circular ? 1 : 0, rows);
    return launch_status();
}

}  // namespace

// cols [B, C k, Lo] from x [B, C, L], Lo = L + 2 p - k + 1; circular padding needs Lo == L.
extern "C" int vfm_im2col1d_f32(const float* x, float* cols, int B, int C, int L, int k, int p, int circular,
                                void* stream) {
    return im2col_launch(x, cols, B, C, L, k, p, circular, 0, stream);
}

// dx [B, C, L] = the adjoint of vfm_im2col1d_f32 applied to dcols [B, C k, Lo].
extern "C" int vfm_col2im1d_f32(const float* dcols, float* dx, int B, int C, int L, int k, int p, int circular,
                                void* stream) {
    return col2im_launch(dcols, dx, B, C, L, k, p, circular, 0, stream);
}

// the same with the batch folded into the columns: cols [C k, B, Lo]
extern "C" int vfm_im2col1d_cbl_f32(const float* x, float* cols, int B, int C, int L, int k, int p, int circular,
                                    void* stream) {
    return im2col_launch(x, cols, B, C, L, k, p, circular, 1, stream);
}

extern "C" int vfm_col2im1d_cbl_f32(const float* dcols, float* dx, int B, int C, int L, int k, int p, int circular,
                                    void* stream) {
    return col2im_launch(dcols, dx, B, C, L, k, p, circular, 1, stream);
}
