"""2-D convolution with integrated FIR up/downsampling.

Drop-in for reference `torch_utils/ops/conv2d_resample.py:46-141`. The
resampling steps run on the HIP `upfirdn2d` kernels; on ROCm tensors the
convolution itself (plain, strided, transposed, grouped -- modulated_conv2d's
per-sample groups) runs on our kernels too: im2col / col2im (csrc/im2col2d.hip)
around the exact-fp32 GEMM (csrc/sgemm.hip), conv2d_hip. CPU tensors take
conv2d_gradfix (torch.nn.functional), as the reference does. Padding is applied
once, before any resampling.
"""
import torch

from .. import misc
from . import conv2d_gradfix
from . import upfirdn2d
from .upfirdn2d import _get_filter_size, _parse_padding


def _conv(x, w, stride=1, padding=0, groups=1, transpose=False, flip_weight=True):
    kh, kw = int(w.shape[2]), int(w.shape[3])
    # conv2d correlates; flip_weight=False requests true convolution.
    if not flip_weight and (kh > 1 or kw > 1):
        w = w.flip([2, 3])
    from . import conv2d_hip
    if conv2d_hip.supported(x, w):
        if transpose:
            return conv2d_hip.conv_transpose2d(x, w, stride=stride, padding=padding, groups=groups)
        return conv2d_hip.conv2d(x, w, stride=stride, padding=padding, groups=groups)
    if transpose:
        return conv2d_gradfix.conv_transpose2d(x, w, stride=stride, padding=padding, groups=groups)
    return conv2d_gradfix.conv2d(x, w, stride=stride, padding=padding, groups=groups)


@misc.profiled_function
def conv2d_resample(x, w, f=None, up=1, down=1, padding=0, groups=1, flip_weight=True, flip_filter=False):
    """Convolve x [N, Cin, H, W] with w [Cout, Cin/groups, kh, kw], upsampling by
    `up` and/or downsampling by `down` with the prepared FIR filter `f`
    (`upfirdn2d.setup_filter`). flip_weight=True means correlation (conv2d)."""
    assert isinstance(x, torch.Tensor) and x.ndim == 4
    assert isinstance(w, torch.Tensor) and w.ndim == 4 and w.dtype == x.dtype
    assert f is None or (isinstance(f, torch.Tensor) and f.ndim in (1, 2) and f.dtype == torch.float32)
    assert isinstance(up, int) and up >= 1 and isinstance(down, int) and down >= 1
    assert isinstance(groups, int) and groups >= 1
    cout, cin_g, kh, kw = (int(s) for s in w.shape)
    fw, fh = _get_filter_size(f)
    px0, px1, py0, py1 = _parse_padding(padding)

    # Padding needed by the FIR resampling filter itself.
    if up > 1:
        px0 += (fw + up - 1) // 2
        px1 += (fw - up) // 2
        py0 += (fh + up - 1) // 2
        py1 += (fh - up) // 2
    if down > 1:
        px0 += (fw - down + 1) // 2
        px1 += (fw - down) // 2
        py0 += (fh - down + 1) // 2
        py1 += (fh - down) // 2
    pads = [px0, px1, py0, py1]
    pointwise = (kw == 1 and kh == 1)

    if pointwise and down > 1 and up == 1:   # decimate first, then 1x1
        x = upfirdn2d.upfirdn2d(x=x, f=f, down=down, padding=pads, flip_filter=flip_filter)
        return _conv(x, w, groups=groups, flip_weight=flip_weight)

    if pointwise and up > 1 and down == 1:   # 1x1 first, then interpolate
        x = _conv(x, w, groups=groups, flip_weight=flip_weight)
        return upfirdn2d.upfirdn2d(x=x, f=f, up=up, padding=pads, gain=up ** 2, flip_filter=flip_filter)

    if down > 1 and up == 1:                 # blur, then strided conv
        x = upfirdn2d.upfirdn2d(x=x, f=f, padding=pads, flip_filter=flip_filter)
        return _conv(x, w, stride=down, groups=groups, flip_weight=flip_weight)

    if up > 1:                               # transposed strided conv, then blur
        if groups == 1:
            wt = w.transpose(0, 1)
        else:
            wt = w.reshape(groups, cout // groups, cin_g, kh, kw).transpose(1, 2)
            wt = wt.reshape(groups * cin_g, cout // groups, kh, kw)
        px0 -= kw - 1
        px1 -= kw - up
        py0 -= kh - 1
        py1 -= kh - up
        pxt = max(min(-px0, -px1), 0)
        pyt = max(min(-py0, -py1), 0)
        x = _conv(x, wt, stride=up, padding=[pyt, pxt], groups=groups, transpose=True, flip_weight=not flip_weight)
        x = upfirdn2d.upfirdn2d(x=x, f=f, padding=[px0 + pxt, px1 + pxt, py0 + pyt, py1 + pyt], gain=up ** 2,
                                flip_filter=flip_filter)
        if down > 1:
            x = upfirdn2d.upfirdn2d(x=x, f=f, down=down, flip_filter=flip_filter)
        return x

    if up == 1 and down == 1 and px0 == px1 and py0 == py1 and px0 >= 0 and py0 >= 0:
        return _conv(x, w, padding=[py0, px0], groups=groups, flip_weight=flip_weight)

    # General case: explicit pad/upsample, conv, then decimate.
    x = upfirdn2d.upfirdn2d(x=x, f=(f if up > 1 else None), up=up, padding=pads, gain=up ** 2, flip_filter=flip_filter)
    x = _conv(x, w, groups=groups, flip_weight=flip_weight)
    if down > 1:
        x = upfirdn2d.upfirdn2d(x=x, f=f, down=down, flip_filter=flip_filter)
    return x
