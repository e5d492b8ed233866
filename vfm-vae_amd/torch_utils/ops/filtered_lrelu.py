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
    """Fused kernel launch. Returns (y, signs_out) or None when no kernel exists."""
    up, down, px0, px1, py0, py1, gain, slope, clamp, flip = cfg
    if x.dtype not in (torch.float16, torch.float32, torch.bfloat16):
        return None
    lib = custom_ops.get_native()
    fu2, fd2 = _as_2d(fu), _as_2d(fd)
    n, c, xh, xw = x.shape
    fuh, fuw = fu2.shape
    fdh, fdw = fd2.shape
    cw = xw * up + (px0 + px1) - (fuw - 1)
    ch = xh * up + (py0 + py1) - (fuh - 1)
    if not (cw > fdw - 1 and ch > fdh - 1):
        raise RuntimeError("upsampled buffer must be at least the size of downsampling filter")
    yw = (cw - (fdw - 1) + (down - 1)) // down
    yh = (ch - (fdh - 1) + (down - 1)) // down
    if yw <= 0 or yh <= 0:
        raise RuntimeError("output must be at least 1x1")
    y = torch.empty([n, c, yh, yw], dtype=x.dtype, device=x.device,
                    memory_format=upfirdn2d._memory_format(x))
    so = None
    if write_signs:
        sw_active = yw * down - (down - 1) + (fdw - 1)
        sh = yh * down - (down - 1) + (fdh - 1)
        sw = (sw_active + 15) & ~15
        so = torch.empty([n, c, sh, sw >> 2], dtype=torch.uint8, device=x.device)
        s, mode = so, 1
    elif si is not None and si.numel():
        if not si.is_contiguous() or si.dtype != torch.uint8 or si.ndim != 4 or si.shape[:2] != x.shape[:2]:
            raise RuntimeError("signs must be a contiguous uint8 [N, C, sh, sw/4] tensor")
        s, mode = si, 2
    else:
        s, mode = None, 0
    sh_, swb = (s.shape[2], s.shape[3]) if s is not None else (0, 0)
    bb = b.contiguous() if b is not None else None
    rc = lib.vfm_filtered_lrelu(x.data_ptr(), fu2.data_ptr(), fd2.data_ptr(), custom_ops.ptr(bb),
                                custom_ops.ptr(s), y.data_ptr(), custom_ops.dtype_code(x),
                                n, c, xh, xw, custom_ops.strides(x), yh, yw, custom_ops.strides(y),
                                fuh, fuw, fdh, fdw, up, down, px0, py0, sh_, swb, sx, sy, mode,
                                gain, slope, clamp, int(flip), custom_ops.stream_ptr(x.device))
    if custom_ops.check(rc, "vfm_filtered_lrelu", allow_no_kernel=True) == custom_ops.VFM_NO_KERNEL:
        return None
    return y, so


def filtered_lrelu_act_(x, si, sx, sy, gain, slope, clamp, write_signs):
    """In-place gain/lrelu/clamp with sign write or read (reference plugin
    `filtered_lrelu_act_`, filtered_lrelu.cpp:213-290). Returns the new sign
    tensor [N, C, H, round16(W)/4] when writing, else an empty tensor."""
    lib = custom_ops.get_native()
    n, c, h, w = x.shape
    so = torch.empty([0], dtype=torch.uint8, device=x.device)
    if write_signs:
        so = torch.empty([n, c, h, ((w + 15) & ~15) >> 2], dtype=torch.uint8, device=x.device)
        s, mode = so, 1
    elif si is not None and si.numel():
        s, mode = si, 2
    else:
        s, mode = None, 0
    sh_, swb = (s.shape[2], s.shape[3]) if s is not None else (0, 0)
    rc = lib.vfm_filtered_lrelu_act(x.data_ptr(), custom_ops.ptr(s), custom_ops.dtype_code(x), n, c, h, w,
                                    custom_ops.strides(x), sh_, swb, sx, sy, mode, float(gain), float(slope),
                                    float(clamp), custom_ops.stream_ptr(x.device))
    custom_ops.check(rc, "vfm_filtered_lrelu_act")
    return so


class _FilteredLReluHip(torch.autograd.Function):
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
