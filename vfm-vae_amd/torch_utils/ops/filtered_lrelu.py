"""Filtered leaky ReLU: bias -> upsample FIR -> gain -> lrelu -> clamp -> downsample FIR.

Drop-in for the reference `torch_utils/ops/filtered_lrelu.py` (API :56-116,
autograd :159-272). `impl='cuda'` on a ROCm device runs the fused LDS kernel of
`csrc/filtered_lrelu.hip` (`vfm_filtered_lrelu`); when that kernel reports
VFM_NO_KERNEL the generic HIP chain upfirdn2d -> `vfm_filtered_lrelu_act` ->
upfirdn2d is used, exactly like the reference's return-code fallback
(filtered_lrelu.py:223-229). Only the 2-bit sign tensor is kept for backward.
"""
import warnings

import numpy as np
import torch

from .. import custom_ops
from .. import misc
from . import bias_act
from . import upfirdn2d


def _get_filter_size(f):
    if f is None:
        return 1, 1
    assert isinstance(f, torch.Tensor) and 1 <= f.ndim <= 2
    return int(f.shape[-1]), int(f.shape[0])  # width, height


def _parse_padding(padding):
    if isinstance(padding, int):
        padding = [padding, padding]
    assert isinstance(padding, (list, tuple)) and all(isinstance(p, (int, np.integer)) for p in padding)
    padding = [int(p) for p in padding]
    if len(padding) == 2:
        px, py = padding
        padding = [px, px, py, py]
    px0, px1, py0, py1 = padding
    return px0, px1, py0, py1


def filtered_lrelu(x, fu=None, fd=None, b=None, up=1, down=1, padding=0, gain=np.sqrt(2), slope=0.2,
                   clamp=None, flip_filter=False, impl='cuda'):
    """Per channel: add bias b, upsample by `up` with FIR `fu` (padding is w.r.t.
    the upsampled image), multiply by `gain`, leaky ReLU with `slope`, clamp to
    [-clamp, clamp], filter with `fd` and keep every `down`-th pixel.
    Same contract as reference filtered_lrelu.py:56-116."""
    assert isinstance(x, torch.Tensor)
    assert impl in ('ref', 'cuda')
    if impl == 'cuda' and x.device.type == 'cuda':
        cfg = _make_cfg(up, down, padding, gain, slope, clamp, flip_filter)
        return _FilteredLReluHip.apply(x, fu, fd, b, None, 0, 0, cfg)
    return _filtered_lrelu_ref(x, fu=fu, fd=fd, b=b, up=up, down=down, padding=padding, gain=gain,
                               slope=slope, clamp=clamp, flip_filter=flip_filter)


@misc.profiled_function
def _filtered_lrelu_ref(x, fu=None, fd=None, b=None, up=1, down=1, padding=0, gain=np.sqrt(2), slope=0.2,
                        clamp=None, flip_filter=False):
    """Composition of the reference ops (reference filtered_lrelu.py:120-153)."""
    assert isinstance(x, torch.Tensor) and x.ndim == 4
    fu_w, fu_h = _get_filter_size(fu)
    fd_w, fd_h = _get_filter_size(fd)
    if b is not None:
        assert isinstance(b, torch.Tensor) and b.dtype == x.dtype
        misc.assert_shape(b, [x.shape[1]])
    assert isinstance(up, int) and up >= 1 and isinstance(down, int) and down >= 1
    px0, px1, py0, py1 = _parse_padding(padding)
    assert gain == float(gain) and gain > 0
    assert slope == float(slope) and slope >= 0
    assert clamp is None or (clamp == float(clamp) and clamp >= 0)
    n, c, h, w = x.shape
    out_w = (w * up + (px0 + px1) - (fu_w - 1) - (fd_w - 1) + (down - 1)) // down
    out_h = (h * up + (py0 + py1) - (fu_h - 1) - (fd_h - 1) + (down - 1)) // down
    dtype = x.dtype
    x = bias_act.bias_act(x=x, b=b, impl='ref')
    x = upfirdn2d.upfirdn2d(x=x, f=fu, up=up, padding=[px0, px1, py0, py1], gain=up ** 2, flip_filter=flip_filter, impl='ref')
    x = bias_act.bias_act(x=x, act='lrelu', alpha=slope, gain=gain, clamp=clamp, impl='ref')
    x = upfirdn2d.upfirdn2d(x=x, f=fd, down=down, flip_filter=flip_filter, impl='ref')
    misc.assert_shape(x, [n, c, out_h, out_w])
    assert x.dtype == dtype
    return x


# ---------------------------------------------------------------------------
# HIP path.


def _make_cfg(up, down, padding, gain, slope, clamp, flip_filter):
    assert isinstance(up, int) and up >= 1 and isinstance(down, int) and down >= 1
    px0, px1, py0, py1 = _parse_padding(padding)
    assert gain == float(gain) and gain > 0
    assert slope == float(slope) and slope >= 0
    assert clamp is None or (clamp == float(clamp) and clamp >= 0)
    clamp = float(clamp) if clamp is not None else float('inf')
    return (up, down, px0, px1, py0, py1, float(gain), float(slope), clamp, bool(flip_filter))


def _as_2d(f):
    """Separable [k] filters are run as their [k, k] outer product (identical math)."""
    return torch.outer(f, f).contiguous() if f.ndim == 1 else f.contiguous()


def _filtered_lrelu_native(x, fu, fd, b, si, sx, sy, cfg, write_signs):
    """Fused kernel launch through torch.ops.vfmvae.filtered_lrelu (csrc/torch_ops.cpp over
    vfm_filtered_lrelu, the reference plugin's schema, filtered_lrelu.cpp:16-204). Returns
    (y, signs_out or None) or None when no kernel exists (the op's return code -1)."""
    up, down, px0, px1, py0, py1, gain, slope, clamp, flip = cfg
    if x.dtype not in (torch.float16, torch.float32, torch.bfloat16):
        return None
    e8 = torch.empty([0], dtype=torch.uint8, device=x.device)
    bb = b if b is not None else torch.zeros([x.shape[1]], dtype=x.dtype, device=x.device)
    y, so, rc = custom_ops.get_torch_ops().filtered_lrelu(
        x, fu, fd, bb, si if (si is not None and si.numel()) else e8, int(up), int(down), int(px0), int(px1),
        int(py0), int(py1), int(sx), int(sy), float(gain), float(slope), float(clamp), bool(flip), bool(write_signs))
    if rc == custom_ops.VFM_NO_KERNEL:
        return None
    return y, (so if write_signs else None)


def filtered_lrelu_act_(x, si, sx, sy, gain, slope, clamp, write_signs):
    """In-place gain/lrelu/clamp with sign write or read (reference plugin
    `filtered_lrelu_act_`, filtered_lrelu.cpp:213-290) through torch.ops.vfmvae.filtered_lrelu_act_.
    Returns the new sign tensor [N, C, H, round16(W)/4] when writing, else an empty tensor."""
    e8 = torch.empty([0], dtype=torch.uint8, device=x.device)
    return custom_ops.get_torch_ops().filtered_lrelu_act_(x, si if (si is not None and si.numel()) else e8, int(sx),
                                                          int(sy), float(gain), float(slope), float(clamp),
                                                          bool(write_signs))


class _FilteredLReluHip(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, x, fu, fd, b, si, sx, sy, cfg):
        assert isinstance(x, torch.Tensor) and x.ndim == 4
        up, down, px0, px1, py0, py1, gain, slope, clamp, flip = cfg
        if fu is None:
            fu = torch.ones([1, 1], dtype=torch.float32, device=x.device)
        if fd is None:
            fd = torch.ones([1, 1], dtype=torch.float32, device=x.device)
        assert 1 <= fu.ndim <= 2 and 1 <= fd.ndim <= 2
        if up == 1 and fu.ndim == 1 and fu.shape[0] == 1:
            fu = fu.square()[None]
        if down == 1 and fd.ndim == 1 and fd.shape[0] == 1:
            fd = fd.square()[None]
        if si is None:
            si = torch.empty([0])
        if b is None:
            b = torch.zeros([x.shape[1]], dtype=x.dtype, device=x.device)
        write_signs = (si.numel() == 0) and (x.requires_grad or b.requires_grad)

        strides = [x.stride(i) for i in range(x.ndim) if x.size(i) > 1]
        if any(s0 < s1 for s0, s1 in zip(strides[:-1], strides[1:])):
            warnings.warn("low-performance memory layout detected in filtered_lrelu input", RuntimeWarning)

        res = _filtered_lrelu_native(x, fu, fd, b, si, sx, sy, cfg, write_signs)
        if res is not None:
            y, so = res
        else:
            y = x.add(b.unsqueeze(-1).unsqueeze(-1))
            y = upfirdn2d.upfirdn2d(x=y, f=fu, up=up, padding=[px0, px1, py0, py1], gain=up ** 2, flip_filter=flip)
            so = filtered_lrelu_act_(y, si, sx, sy, gain, slope, clamp, write_signs)
            y = upfirdn2d.upfirdn2d(x=y, f=fd, down=down, flip_filter=flip)
        if so is None:
            so = torch.empty([0], dtype=torch.uint8, device=x.device)

        ctx.save_for_backward(fu, fd, si if si.numel() else so)
        ctx.x_shape = x.shape
        ctx.y_shape = y.shape
        ctx.s_ofs = (sx, sy)
        ctx.cfg = cfg
        return y

    @staticmethod
    def backward(ctx, dy):
        fu, fd, si = ctx.saved_tensors
        up, down, px0, px1, py0, py1, gain, slope, clamp, flip = ctx.cfg
        _, _, xh, xw = ctx.x_shape
        _, _, yh, yw = ctx.y_shape
        sx, sy = ctx.s_ofs
        for i in (1, 2, 4, 5, 6):
            assert not ctx.needs_input_grad[i]
        dx = db = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[3]:
            pp = [(fu.shape[-1] - 1) + (fd.shape[-1] - 1) - px0,
                  xw * up - yw * down + px0 - (up - 1),
                  (fu.shape[0] - 1) + (fd.shape[0] - 1) - py0,
                  xh * up - yh * down + py0 - (up - 1)]
            gg = gain * (up ** 2) / (down ** 2)
            bcfg = _make_cfg(down, up, pp, gg, slope, None, not flip)
            bsx = sx - (fu.shape[-1] - 1) + px0
            bsy = sy - (fu.shape[0] - 1) + py0
            dx = _FilteredLReluHip.apply(dy, fd, fu, None, si, bsx, bsy, bcfg)
        if ctx.needs_input_grad[3]:
            db = dx.sum([0, 2, 3])
        return dx, None, None, db, None, None, None, None
