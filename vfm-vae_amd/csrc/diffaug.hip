// DiffAugment's random translation (reference training/diffaug.py rand_translation: the image is
// zero-padded by one pixel and gathered at clamp(i + t + 1, 0, H + 1), i.e. every sample shifted by
// its own integer (tx, ty) with zero fill) as a per-sample shift kernel. The gather is a bijection
// between the in-range pixels, so the backward is the same kernel with the shift negated (the
// reference's indexing backward accumulates each in-range gradient once into zeros: identical values)
// instead of torch's sort-based indexing_backward.
//   y[b, c, i, j] = x[b, c, i + s tx[b], j + s ty[b]] if inside the image, else 0   (s = +1 / -1)
#include "vfm_common.h"

namespace {

using namespace vfm;

template <class T>
__global__ __launch_bounds__(256) void shift2d_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                    const long long* __restrict__ tx,
                                                    const long long* __restrict__ ty, int C, int H, int W, int sign) {
    const int b = blockIdx.z;
    const int row = blockIdx.y;                       // c * H + i
    const int c = row / H, i = row - c * H;
    const int sx = sign * (int)tx[b], sy = sign * (int)ty[b];
    const int si = i + sx;
    const long long plane = ((long long)b * C + c) * H;
    T* yr = y + (plane + i) * W;
    const bool rin = si >= 0 && si < H;
    const T* xr = x + (plane + (rin ? si : 0)) * W;
    for (int j = blockIdx.x * 256 + threadIdx.x; j < W; j += gridDim.x * 256) {
        const int sj = j + sy;
        yr[j] = (rin && sj >= 0 && sj < W) ? xr[sj] : T(0.f);
    }
}

}  // namespace

extern "C" int vfm_shift2d(const void* x, void* y, const long long* tx, const long long* ty, int dtype, int B, int C,
                           int H, int W, int sign, void* stream) {
    if (!x || !y || !tx || !ty || B <= 0 || C <= 0 || H <= 0 || W <= 0 || (sign != 1 && sign != -1)) return VFM_ERR_ARGS;
    if (B > 65535 || (long long)C * H > 65535) return VFM_NO_KERNEL;
    const dim3 grid((W + 255) / 256, C * H, B);
    hipStream_t st = (hipStream_t)stream;
    switch (dtype) {
    case VFM_F32:
        VFM_LAUNCH(shift2d_kernel<float>, grid, dim3(256), 0, st, (const float*)x, (float*)y, tx, ty, C, H, W,
                           sign);
        break;
    case VFM_BF16:
        VFM_LAUNCH(shift2d_kernel<__hip_bfloat16>, grid, dim3(256), 0, st, (const __hip_bfloat16*)x,
                           (__hip_bfloat16*)y, tx, ty, C, H, W, sign);
        break;
    default:
        return VFM_ERR_ARGS;
    }
    return launch_status();
}
