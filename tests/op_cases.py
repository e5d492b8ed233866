"""Shared helpers that turn golden-vector metadata into op calls."""
import numpy as np


def parse_scaling(s):
    return (s, s) if isinstance(s, int) else tuple(s)


def parse_padding(p):
    if isinstance(p, int):
        return p, p, p, p
    if len(p) == 2:
        return p[0], p[0], p[1], p[1]
    return tuple(p)


def upfirdn_params(api, f, kw):
    """Restate the wrapper padding/gain rules (reference upfirdn2d.py:277-387) as a
    plain upfirdn2d call: returns dict(up, down, padding, flip_filter, gain)."""
    if f is None:
        fw = fh = 1
    else:
        fw, fh = f.shape[-1], f.shape[0]
    flip = kw.get("flip_filter", False)
    gain = kw.get("gain", 1)
    if api == "upfirdn2d":
        return dict(up=parse_scaling(kw.get("up", 1)), down=parse_scaling(kw.get("down", 1)),
                    padding=parse_padding(kw.get("padding", 0)), flip_filter=flip, gain=gain)
    px0, px1, py0, py1 = parse_padding(kw.get("padding", 0))
    if api == "filter2d":
        return dict(up=(1, 1), down=(1, 1), flip_filter=flip, gain=gain,
                    padding=(px0 + fw // 2, px1 + (fw - 1) // 2, py0 + fh // 2, py1 + (fh - 1) // 2))
    if api == "upsample2d":
        ux, uy = parse_scaling(kw.get("up", 2))
        return dict(up=(ux, uy), down=(1, 1), flip_filter=flip, gain=gain * ux * uy,
                    padding=(px0 + (fw + ux - 1) // 2, px1 + (fw - ux) // 2, py0 + (fh + uy - 1) // 2, py1 + (fh - uy) // 2))
    if api == "downsample2d":
        dx, dy = parse_scaling(kw.get("down", 2))
        return dict(up=(1, 1), down=(dx, dy), flip_filter=flip, gain=gain,
                    padding=(px0 + (fw - dx + 1) // 2, px1 + (fw - dx) // 2, py0 + (fh - dy + 1) // 2, py1 + (fh - dy) // 2))
    raise ValueError(api)


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / (np.max(np.abs(b)) + 1e-30))
