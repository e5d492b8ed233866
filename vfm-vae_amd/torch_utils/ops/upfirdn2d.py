"""Up/FIR/down resampling of image batches: `upfirdn2d`, `filter2d`, `upsample2d`,
`downsample2d`, `setup_filter`.

Drop-in for the reference module `torch_utils/ops/upfirdn2d.py` (API :70-387).
`impl='cuda'` on a ROCm device runs the gfx950 kernels of `csrc/upfirdn2d.hip`
through the C ABI `vfm_upfirdn2d` (include/vfmvae.h); `impl='ref'` (or a CPU
tensor) runs the pure-torch restatement `_upfirdn2d_ref`.

Per axis the op computes  y[o] = gain * sum_t g[t] * u[o*down + t - pad0],
with u the zero-inserted (x `up` times) signal and g = flip(f) for convolution
(flip_filter=False) or g = f for correlation.
"""
import numpy as np
import torch

from .. import custom_ops
from .. import misc
from . import conv2d_gradfix

# ---------------------------------------------------------------------------
# Argument parsing (same accepted forms as upfirdn2d.py:36-65).


def _parse_scaling(scaling):
    if isinstance(scaling, int):
        return scaling, scaling
    assert isinstance(scaling, (list, tuple)) and len(scaling) == 2
    sx, sy = scaling
    assert isinstance(sx, int) and isinstance(sy, int) and sx >= 1 and sy >= 1
    return sx, sy


def _parse_padding(padding):
    if isinstance(padding, int):
        return padding, padding, padding, padding
    assert isinstance(padding, (list, tuple)) and all(isinstance(p, (int, np.integer)) for p in padding)
    padding = [int(p) for p in padding]
    if len(padding) == 2:
        px, py = padding
        return px, px, py, py
    assert len(padding) == 4
    return tuple(padding)


def _get_filter_size(f):
    """(width, height) of a 1-D (separable) or 2-D filter; (1, 1) for None."""
    if f is None:
        return 1, 1
    assert isinstance(f, torch.Tensor) and f.ndim in (1, 2)
    fw = int(f.shape[-1])
    fh = int(f.shape[0])
    assert fw >= 1 and fh >= 1
    return fw, fh


# ---------------------------------------------------------------------------


def setup_filter(f, device=torch.device('cpu'), normalize=True, flip_filter=False, gain=1, separable=None):
    """Build an fp32 FIR filter for `upfirdn2d()`.

    f: list / array / tensor of shape [taps] (separable candidate), [fh, fw],
       [] (impulse) or None (identity). A 1-D filter with fewer than 8 taps is
       expanded to its 2-D outer product unless `separable` says otherwise
       (reference behaviour, upfirdn2d.py:91-111). The filter is normalised to
       unit DC gain, optionally flipped, and scaled by gain^(ndim/2).
    """
    if f is None:
        f = 1
    f = torch.as_tensor(f, dtype=torch.float32)
    assert f.ndim in (0, 1, 2) and f.numel() > 0
    if f.ndim == 0:
        f = f.reshape(1)
    if separable is None:
        separable = f.ndim == 1 and f.numel() >= 8
    if f.ndim == 1 and not separable:
        f = torch.outer(f, f)
    assert f.ndim == (1 if separable else 2)
    if normalize:
        f = f / f.sum()
    if flip_filter:
        f = f.flip(list(range(f.ndim)))
    f = f * (gain ** (f.ndim / 2))
    return f.to(device=device)


# ---------------------------------------------------------------------------


def upfirdn2d(x, f, up=1, down=1, padding=0, flip_filter=False, gain=1, impl='cuda'):
    """Upsample (zero insertion), pad (negative = crop), FIR-filter and downsample
    a [N, C, H, W] batch; same contract as reference upfirdn2d.py:118-162.
    Supports fp32/fp16/bf16/fp64 inputs, contiguous or channels-last, and
    gradients of any order on the HIP path."""
    assert isinstance(x, torch.Tensor)
    assert impl in ('ref', 'cuda')
    if impl == 'cuda' and x.device.type == 'cuda':
        upx, upy = _parse_scaling(up)
        downx, downy = _parse_scaling(down)
        pads = _parse_padding(padding)
        return _Upfirdn2dHip.apply(x, f, (upx, upy), (downx, downy), pads, bool(flip_filter), float(gain))
    return _upfirdn2d_ref(x, f, up=up, down=down, padding=padding, flip_filter=flip_filter, gain=gain)


@misc.profiled_function
def _upfirdn2d_ref(x, f, up=1, down=1, padding=0, flip_filter=False, gain=1):
    """Pure-torch restatement (reference _upfirdn2d_ref, upfirdn2d.py:166-211):
    zero-insert, pad/crop, depthwise conv with the (flipped) filter, decimate."""
    assert isinstance(x, torch.Tensor) and x.ndim == 4
    if f is None:
        f = torch.ones([1, 1], dtype=torch.float32, device=x.device)
    assert isinstance(f, torch.Tensor) and f.ndim in (1, 2)
    assert f.dtype == torch.float32 and not f.requires_grad
    n, c, h, w = x.shape
    upx, upy = _parse_scaling(up)
    downx, downy = _parse_scaling(down)
    px0, px1, py0, py1 = _parse_padding(padding)
    assert w * upx + px0 + px1 >= f.shape[-1] and h * upy + py0 + py1 >= f.shape[0]

    # Zero insertion: place samples at multiples of `up`.
    if upx > 1 or upy > 1:
        u = x.new_zeros([n, c, h * upy, w * upx])
        u[:, :, ::upy, ::upx] = x
        x = u
    # Pad positive sides, crop negative ones.
    x = torch.nn.functional.pad(x, [max(px0, 0), max(px1, 0), max(py0, 0), max(py1, 0)])
    x = x[:, :, max(-py0, 0): x.shape[2] - max(-py1, 0), max(-px0, 0): x.shape[3] - max(-px1, 0)]

    g = (f * (gain ** (f.ndim / 2))).to(x.dtype)
    if not flip_filter:
        g = g.flip(list(range(g.ndim)))  # conv2d correlates; flip for convolution
    if g.ndim == 2:
        wgt = g[None, None].expand(c, 1, *g.shape)
        x = conv2d_gradfix.conv2d(input=x, weight=wgt, groups=c)
    else:
        x = conv2d_gradfix.conv2d(input=x, weight=g[None, None, None, :].expand(c, 1, 1, g.numel()), groups=c)
        x = conv2d_gradfix.conv2d(input=x, weight=g[None, None, :, None].expand(c, 1, g.numel(), 1), groups=c)
    return x[:, :, ::downy, ::downx]


# ---------------------------------------------------------------------------
# HIP path.


def _out_size(size, up, pad0, pad1, taps, down):
    return (size * up + pad0 + pad1 - taps + down) // down


def _launch(x, f2, up, down, pads, flip, gain):
    """One kernel launch with a 2-D filter f2 (already shaped [fh, fw]) through the registered op
    torch.ops.vfmvae.upfirdn2d (csrc/torch_ops.cpp over vfm_upfirdn2d; the reference plugin's
    schema and checks, upfirdn2d.cpp:16-98)."""
    upx, upy = up
    downx, downy = down
    px0, px1, py0, py1 = pads
    return custom_ops.get_torch_ops().upfirdn2d(x, f2, upx, upy, downx, downy, px0, px1, py0, py1, bool(flip),
                                                float(gain))


def _memory_format(x):
    return torch.channels_last if (x.ndim == 4 and x.stride(1) == 1 and x.shape[1] > 1) else torch.contiguous_format


def _upfirdn2d_hip_forward(x, f, up, down, pads, flip, gain):
    if f is None:
        f = torch.ones([1, 1], dtype=torch.float32, device=x.device)
    if f.ndim == 1 and f.shape[0] == 1:
        f = f.square().unsqueeze(0)  # separable 1-tap -> 1x1
    if f.ndim == 2:
        return _launch(x, f, up, down, pads, flip, gain)
    # Separable: horizontal pass, then vertical pass carrying the gain.
    px0, px1, py0, py1 = pads
    y = _launch(x, f.unsqueeze(0), (up[0], 1), (down[0], 1), (px0, px1, 0, 0), flip, 1.0)
    return _launch(y, f.unsqueeze(1), (1, up[1]), (1, down[1]), (0, 0, py0, py1), flip, gain)


class _Upfirdn2dHip(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, x, f, up, down, pads, flip, gain):
        assert x.ndim == 4
        y = _upfirdn2d_hip_forward(x, f, up, down, pads, flip, gain)
        ff = f if f is not None else torch.ones([1, 1], dtype=torch.float32, device=x.device)
        if ff.ndim == 1 and ff.shape[0] == 1:
            ff = ff.square().unsqueeze(0)
        ctx.save_for_backward(ff)
        ctx.cfg = (up, down, pads, flip, gain, tuple(x.shape))
        return y

    @staticmethod
    def backward(ctx, dy):
        (f,) = ctx.saved_tensors
        up, down, pads, flip, gain, xshape = ctx.cfg
        assert not ctx.needs_input_grad[1], "filter gradients are not supported (as in the reference)"
        dx = None
        if ctx.needs_input_grad[0]:
            _, _, ih, iw = xshape
            _, _, oh, ow = dy.shape
            fw, fh = _get_filter_size(f)
            px0, px1, py0, py1 = pads
            # Adjoint: swap up/down, flip the filter, pad so that the output is x-shaped.
            p = (fw - px0 - 1,
                 iw * up[0] - ow * down[0] + px0 - up[0] + 1,
                 fh - py0 - 1,
                 ih * up[1] - oh * down[1] + py0 - up[1] + 1)
            dx = _Upfirdn2dHip.apply(dy, f, down, up, p, not flip, gain)
        return dx, None, None, None, None, None, None


# ---------------------------------------------------------------------------
# Convenience wrappers (padding relative to the output, as upfirdn2d.py:277-387).


def filter2d(x, f, padding=0, flip_filter=False, gain=1, impl='cuda'):
    """Same-size FIR filtering; extra padding (negative = crop) on top."""
    px0, px1, py0, py1 = _parse_padding(padding)
    fw, fh = _get_filter_size(f)
    p = [px0 + fw // 2, px1 + (fw - 1) // 2, py0 + fh // 2, py1 + (fh - 1) // 2]
    return upfirdn2d(x, f, padding=p, flip_filter=flip_filter, gain=gain, impl=impl)


def upsample2d(x, f, up=2, padding=0, flip_filter=False, gain=1, impl='cuda'):
    """Upsample by `up` with FIR interpolation; output is `up` times the input."""
    upx, upy = _parse_scaling(up)
    px0, px1, py0, py1 = _parse_padding(padding)
    fw, fh = _get_filter_size(f)
    p = [px0 + (fw + upx - 1) // 2, px1 + (fw - upx) // 2, py0 + (fh + upy - 1) // 2, py1 + (fh - upy) // 2]
    return upfirdn2d(x, f, up=up, padding=p, flip_filter=flip_filter, gain=gain * upx * upy, impl=impl)


def downsample2d(x, f, down=2, padding=0, flip_filter=False, gain=1, impl='cuda'):
    """Low-pass and decimate by `down`; output is 1/`down` of the input."""
    downx, downy = _parse_scaling(down)
    px0, px1, py0, py1 = _parse_padding(padding)
    fw, fh = _get_filter_size(f)
    p = [px0 + (fw - downx + 1) // 2, px1 + (fw - downx) // 2, py0 + (fh - downy + 1) // 2, py1 + (fh - downy) // 2]
    return upfirdn2d(x, f, down=down, padding=p, flip_filter=flip_filter, gain=gain, impl=impl)
