// TORCH_LIBRARY(vfmvae, ...) registration of the plugin ops the reference binds through pybind11
// (torch_utils/custom_ops.py:59-155 building upfirdn2d_plugin / bias_act_plugin /
// filtered_lrelu_plugin), with the reference's schemas and argument checks, over the extern "C"
// launchers of include/vfmvae.h (libvfmvae_hip.so). Host code only: no kernels live here.
//
//   torch.ops.vfmvae.upfirdn2d(x, f, upx, upy, downx, downy, padx0, padx1, pady0, pady1, flip, gain)
//       replaces upfirdn2d.cpp:16-98 (reference); output in x's suggested memory format
//   torch.ops.vfmvae.bias_act(x, b, xref, yref, dy, grad, dim, act, alpha, gain, clamp)
//       replaces bias_act.cpp:32-90; empty tensors = absent, output empty_like(x)
//   torch.ops.vfmvae.filtered_lrelu(x, fu, fd, b, si, up, down, px0, px1, py0, py1, sx, sy, gain,
//       slope, clamp, flip_filters, writeSigns) -> (y, so, rc)
//       replaces filtered_lrelu.cpp:16-204; rc = -1 with empty tensors when no fused kernel exists
//       (the caller then takes the generic path, filtered_lrelu.py:223-229 of the reference)
//   torch.ops.vfmvae.filtered_lrelu_act_(x, si, sx, sy, gain, slope, clamp, writeSigns) -> so
//       replaces filtered_lrelu.cpp:208-290; x is modified in place
// Errors: TORCH_CHECK -> RuntimeError for the reference's argument violations; a launcher error code
// -> RuntimeError naming the launcher. Kernels are enqueued on the current HIP stream, no host sync.
#include <torch/library.h>
#include <ATen/ATen.h>
// ROCm builds of PyTorch present HIP devices as DeviceType::CUDA: the guard and stream types are the
// "masquerading" ones (c10::hip::HIPGuardImpl would reject a cuda device)
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <climits>
#include <tuple>

#include "../../include/vfmvae.h"

namespace {

int dtype_code(const at::Tensor& t) {
    switch (t.scalar_type()) {
    case at::kFloat: return VFM_F32;
    case at::kHalf: return VFM_F16;
    case at::kBFloat16: return VFM_BF16;
    case at::kDouble: return VFM_F64;
    default: TORCH_CHECK(false, "unsupported dtype ", t.scalar_type());
    }
    return -1;
}

void* stream_of(const at::Tensor& t) {
    return (void*)c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

void check_rc(int rc, const char* name) { TORCH_CHECK(rc == VFM_OK, name, " failed with code ", rc); }

bool has_same_layout(const at::Tensor& a, const at::Tensor& b) {
    if (a.dim() != b.dim()) return false;
    for (int64_t i = 0; i < a.dim(); ++i) {
        if (a.size(i) != b.size(i)) return false;
        if (a.size(i) >= 2 && a.stride(i) != b.stride(i)) return false;
    }
    return true;
}

int64_t footprint(const at::Tensor& t) {
    int64_t s = 0;
    for (int64_t i = 0; i < t.dim(); ++i) s += (t.size(i) - 1) * t.stride(i);
    return s;
}

// separable [k] filters are run as their [k, k] outer product (identical math)
at::Tensor as_2d(const at::Tensor& f) { return f.dim() == 1 ? at::outer(f, f).contiguous() : f.contiguous(); }

at::Tensor upfirdn2d(const at::Tensor& x, const at::Tensor& f, int64_t upx, int64_t upy, int64_t downx, int64_t downy,
                     int64_t padx0, int64_t padx1, int64_t pady0, int64_t pady1, bool flip, double gain) {
    TORCH_CHECK(x.is_cuda(), "x must reside on CUDA device");
    TORCH_CHECK(f.device() == x.device(), "f must reside on the same device as x");
    TORCH_CHECK(f.dtype() == at::kFloat, "f must be float32");
    TORCH_CHECK(x.numel() <= INT_MAX, "x is too large");
    TORCH_CHECK(f.numel() <= INT_MAX, "f is too large");
    TORCH_CHECK(x.numel() > 0, "x has zero size");
    TORCH_CHECK(f.numel() > 0, "f has zero size");
    TORCH_CHECK(x.dim() == 4, "x must be rank 4");
    TORCH_CHECK(f.dim() == 2, "f must be rank 2");
    TORCH_CHECK(footprint(x) <= INT_MAX, "x memory footprint is too large");
    TORCH_CHECK(f.size(0) >= 1 && f.size(1) >= 1, "f must be at least 1x1");
    TORCH_CHECK(upx >= 1 && upy >= 1, "upsampling factor must be at least 1");
    TORCH_CHECK(downx >= 1 && downy >= 1, "downsampling factor must be at least 1");
    const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
    const int outW = ((int)x.size(3) * (int)upx + (int)padx0 + (int)padx1 - (int)f.size(1) + (int)downx) / (int)downx;
    const int outH = ((int)x.size(2) * (int)upy + (int)pady0 + (int)pady1 - (int)f.size(0) + (int)downy) / (int)downy;
    TORCH_CHECK(outW >= 1 && outH >= 1, "output must be at least 1x1");
    at::Tensor y = at::empty({x.size(0), x.size(1), outH, outW}, x.options(), x.suggest_memory_format());
    TORCH_CHECK(y.numel() <= INT_MAX, "output is too large");
    TORCH_CHECK(footprint(y) <= INT_MAX, "output memory footprint is too large");
    const long long xs[4] = {x.stride(0), x.stride(1), x.stride(2), x.stride(3)};
    const long long ys[4] = {y.stride(0), y.stride(1), y.stride(2), y.stride(3)};
    check_rc(vfm_upfirdn2d(x.data_ptr(), y.data_ptr(), f.data_ptr<float>(), dtype_code(x), (int)x.size(0),
                           (int)x.size(1), (int)x.size(2), (int)x.size(3), xs, outH, outW, ys, (int)f.size(0),
                           (int)f.size(1), f.stride(0), f.stride(1), (int)upx, (int)upy, (int)downx, (int)downy,
                           (int)padx0, (int)pady0, flip ? 1 : 0, (float)gain, stream_of(x)),
             "vfm_upfirdn2d");
    return y;
}

at::Tensor bias_act(const at::Tensor& x, const at::Tensor& b, const at::Tensor& xref, const at::Tensor& yref,
                    const at::Tensor& dy, int64_t grad, int64_t dim, int64_t act, double alpha, double gain,
                    double clamp) {
    TORCH_CHECK(x.is_cuda(), "x must reside on CUDA device");
    TORCH_CHECK(b.numel() == 0 || (b.dtype() == x.dtype() && b.device() == x.device()),
                "b must have the same dtype and device as x");
    TORCH_CHECK(xref.numel() == 0 || (xref.sizes() == x.sizes() && xref.dtype() == x.dtype() && xref.device() == x.device()),
                "xref must have the same shape, dtype, and device as x");
    TORCH_CHECK(yref.numel() == 0 || (yref.sizes() == x.sizes() && yref.dtype() == x.dtype() && yref.device() == x.device()),
                "yref must have the same shape, dtype, and device as x");
    TORCH_CHECK(dy.numel() == 0 || (dy.sizes() == x.sizes() && dy.dtype() == x.dtype() && dy.device() == x.device()),
                "dy must have the same dtype and device as x");
    TORCH_CHECK(x.numel() <= INT_MAX, "x is too large");
    TORCH_CHECK(b.dim() == 1, "b must have rank 1");
    TORCH_CHECK(b.numel() == 0 || (dim >= 0 && dim < x.dim()), "dim is out of bounds");
    TORCH_CHECK(b.numel() == 0 || b.numel() == x.size(dim), "b has wrong number of elements");
    TORCH_CHECK(grad >= 0, "grad must be non-negative");
    TORCH_CHECK(x.is_non_overlapping_and_dense(), "x must be non-overlapping and dense");
    TORCH_CHECK(b.is_contiguous(), "b must be contiguous");
    TORCH_CHECK(xref.numel() == 0 || has_same_layout(xref, x), "xref must have the same layout as x");
    TORCH_CHECK(yref.numel() == 0 || has_same_layout(yref, x), "yref must have the same layout as x");
    TORCH_CHECK(dy.numel() == 0 || has_same_layout(dy, x), "dy must have the same layout as x");
    const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
    at::Tensor y = at::empty_like(x);
    TORCH_CHECK(has_same_layout(y, x), "y must have the same layout as x");
    if (x.numel() == 0) return y;
    const long long stepB = b.numel() ? x.stride(dim) : 1;
    const int rc = vfm_bias_act(x.data_ptr(), b.numel() ? b.data_ptr() : nullptr, xref.numel() ? xref.data_ptr() : nullptr,
                                yref.numel() ? yref.data_ptr() : nullptr, dy.numel() ? dy.data_ptr() : nullptr,
                                y.data_ptr(), dtype_code(x), x.numel(), (int)grad, (int)act, (float)alpha, (float)gain,
                                (float)clamp, stepB, (int)b.numel(), stream_of(x));
    TORCH_CHECK(rc != VFM_ERR_ARGS, "vfm_bias_act: no kernel for these arguments (activation code ", act, ")");
    check_rc(rc, "vfm_bias_act");
    return y;
}

std::tuple<at::Tensor, at::Tensor, int64_t> filtered_lrelu(const at::Tensor& x, const at::Tensor& fu,
                                                           const at::Tensor& fd, const at::Tensor& b,
                                                           const at::Tensor& si, int64_t up, int64_t down, int64_t px0,
                                                           int64_t px1, int64_t py0, int64_t py1, int64_t sx,
                                                           int64_t sy, double gain, double slope, double clamp,
                                                           bool flip_filters, bool writeSigns) {
    TORCH_CHECK(x.is_cuda(), "x must reside on CUDA device");
    const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
    TORCH_CHECK(fu.device() == x.device() && fd.device() == x.device() && b.device() == x.device(),
                "all input tensors must reside on the same device");
    TORCH_CHECK(fu.dtype() == at::kFloat && fd.dtype() == at::kFloat, "fu and fd must be float32");
    TORCH_CHECK(b.dtype() == x.dtype(), "x and b must have the same dtype");
    TORCH_CHECK(x.dtype() == at::kHalf || x.dtype() == at::kFloat || x.dtype() == at::kBFloat16,
                "x and b must be float16, bfloat16 or float32");
    TORCH_CHECK(x.dim() == 4, "x must be rank 4");
    TORCH_CHECK(x.size(0) * x.size(1) <= INT_MAX && x.size(2) <= INT_MAX && x.size(3) <= INT_MAX, "x is too large");
    TORCH_CHECK(x.numel() > 0, "x is empty");
    TORCH_CHECK((fu.dim() == 1 || fu.dim() == 2) && (fd.dim() == 1 || fd.dim() == 2), "fu and fd must be rank 1 or 2");
    TORCH_CHECK(fu.numel() > 0, "fu is empty");
    TORCH_CHECK(fd.numel() > 0, "fd is empty");
    TORCH_CHECK(b.dim() == 1 && b.size(0) == x.size(1), "b must be a vector with the same number of channels as x");
    TORCH_CHECK(up >= 1 && down >= 1, "up and down must be at least 1");
    const at::Tensor fu2 = as_2d(fu), fd2 = as_2d(fd);
    const int64_t fuh = fu2.size(0), fuw = fu2.size(1), fdh = fd2.size(0), fdw = fd2.size(1);
    const int64_t cw = x.size(3) * up + (px0 + px1) - (fuw - 1), ch = x.size(2) * up + (py0 + py1) - (fuh - 1);
    TORCH_CHECK(cw > fdw - 1 && ch > fdh - 1, "upsampled buffer must be at least the size of downsampling filter");
    const int64_t yw = (cw - (fdw - 1) + (down - 1)) / down, yh = (ch - (fdh - 1) + (down - 1)) / down;
    TORCH_CHECK(yw > 0 && yh > 0, "output must be at least 1x1");
    at::Tensor y = at::empty({x.size(0), x.size(1), yh, yw}, x.options(), x.suggest_memory_format());
    at::Tensor so, s;
    int mode = 0;
    if (writeSigns) {
        const int64_t sw_active = yw * down - (down - 1) + (fdw - 1), sh = yh * down - (down - 1) + (fdh - 1);
        const int64_t sw = (sw_active + 15) & ~15;
        so = s = at::empty({x.size(0), x.size(1), sh, sw >> 2}, x.options().dtype(at::kByte), at::MemoryFormat::Contiguous);
        mode = 1;
    } else if (si.numel()) {
        TORCH_CHECK(si.is_contiguous() && si.dtype() == at::kByte && si.dim() == 4 && si.size(0) == x.size(0) &&
                        si.size(1) == x.size(1),
                    "signs must be a contiguous uint8 [N, C, sh, sw/4] tensor");
        s = si;
        mode = 2;
    }
    const long long xs[4] = {x.stride(0), x.stride(1), x.stride(2), x.stride(3)};
    const long long ys[4] = {y.stride(0), y.stride(1), y.stride(2), y.stride(3)};
    const at::Tensor bb = b.contiguous();
    const int rc = vfm_filtered_lrelu(
        x.data_ptr(), fu2.data_ptr<float>(), fd2.data_ptr<float>(), bb.data_ptr(),
        mode ? s.data_ptr<unsigned char>() : nullptr, y.data_ptr(), dtype_code(x), (int)x.size(0), (int)x.size(1),
        (int)x.size(2), (int)x.size(3), xs, (int)yh, (int)yw, ys, (int)fuh, (int)fuw, (int)fdh, (int)fdw, (int)up,
        (int)down, (int)px0, (int)py0, mode ? (int)s.size(2) : 0, mode ? (int)s.size(3) : 0, (int)sx, (int)sy, mode,
        (float)gain, (float)slope, (float)clamp, flip_filters ? 1 : 0, stream_of(x));
    if (rc == VFM_NO_KERNEL) return std::make_tuple(at::Tensor(), at::Tensor(), (int64_t)-1);
    check_rc(rc, "vfm_filtered_lrelu");
    return std::make_tuple(y, writeSigns ? so : at::empty({0}, x.options().dtype(at::kByte)), (int64_t)0);
}

at::Tensor filtered_lrelu_act(const at::Tensor& x, const at::Tensor& si, int64_t sx, int64_t sy, double gain,
                              double slope, double clamp, bool writeSigns) {
    TORCH_CHECK(x.is_cuda(), "x must reside on CUDA device");
    const c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
    TORCH_CHECK(x.dim() == 4, "x must be rank 4");
    TORCH_CHECK(x.size(0) * x.size(1) <= INT_MAX && x.size(2) <= INT_MAX && x.size(3) <= INT_MAX, "x is too large");
    TORCH_CHECK(x.numel() > 0, "x is empty");
    TORCH_CHECK(x.dtype() == at::kHalf || x.dtype() == at::kFloat || x.dtype() == at::kDouble || x.dtype() == at::kBFloat16,
                "x must be float16, bfloat16, float32 or float64");
    at::Tensor so, s = si;
    const bool readSigns = si.numel() > 0;
    if (writeSigns) {
        const int64_t sw = (x.size(3) + 15) & ~15;
        s = so = at::empty({x.size(0), x.size(1), x.size(2), sw >> 2}, x.options().dtype(at::kByte),
                           at::MemoryFormat::Contiguous);
    }
    if (readSigns || writeSigns) {
        TORCH_CHECK(s.is_contiguous(), "signs must be contiguous");
        TORCH_CHECK(s.dtype() == at::kByte, "signs must be uint8");
        TORCH_CHECK(s.device() == x.device(), "signs must reside on the same device as x");
        TORCH_CHECK(s.dim() == 4, "signs must be rank 4");
        TORCH_CHECK(s.size(0) == x.size(0) && s.size(1) == x.size(1), "signs must have same batch & channels as x");
        TORCH_CHECK(s.size(2) <= INT_MAX && (s.size(3) << 2) <= INT_MAX, "signs tensor is too large");
    }
    const int mode = writeSigns ? 1 : (readSigns ? 2 : 0);
    const long long xs[4] = {x.stride(0), x.stride(1), x.stride(2), x.stride(3)};
    check_rc(vfm_filtered_lrelu_act(x.data_ptr(), mode ? s.data_ptr<unsigned char>() : nullptr, dtype_code(x),
                                    (int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3), xs,
                                    mode ? (int)s.size(2) : 0, mode ? (int)s.size(3) : 0, (int)sx, (int)sy, mode,
                                    (float)gain, (float)slope, (float)clamp, stream_of(x)),
             "vfm_filtered_lrelu_act");
    return writeSigns ? so : at::empty({0}, x.options().dtype(at::kByte));
}

}  // namespace

TORCH_LIBRARY(vfmvae, m) {
    m.def("upfirdn2d(Tensor x, Tensor f, int upx, int upy, int downx, int downy, int padx0, int padx1, int pady0, "
          "int pady1, bool flip, float gain) -> Tensor");
    m.def("bias_act(Tensor x, Tensor b, Tensor xref, Tensor yref, Tensor dy, int grad, int dim, int act, float alpha, "
          "float gain, float clamp) -> Tensor");
    m.def("filtered_lrelu(Tensor x, Tensor fu, Tensor fd, Tensor b, Tensor si, int up, int down, int px0, int px1, "
          "int py0, int py1, int sx, int sy, float gain, float slope, float clamp, bool flip_filters, bool writeSigns) "
          "-> (Tensor, Tensor, int)");
    m.def("filtered_lrelu_act_(Tensor(a!) x, Tensor si, int sx, int sy, float gain, float slope, float clamp, "
          "bool writeSigns) -> Tensor");
}

TORCH_LIBRARY_IMPL(vfmvae, CUDA, m) {
    m.impl("upfirdn2d", &upfirdn2d);
    m.impl("bias_act", &bias_act);
    m.impl("filtered_lrelu", &filtered_lrelu);
    m.impl("filtered_lrelu_act_", &filtered_lrelu_act);
}
