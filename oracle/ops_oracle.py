"""ctypes wrapper over oracle/ops_oracle.c — TEST INFRASTRUCTURE ONLY.

Double-precision CPU restatements of upfirdn2d / bias_act / filtered_lrelu
(reference torch_utils/ops/{upfirdn2d,bias_act,filtered_lrelu}.py `_ref`
paths) and the fp32 codebook lookup (networks/utils/quant_utils.py:84-86).
See ops_oracle.c for the file:line each function follows.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "_build", "libops_oracle.so")
_lib = None

_dp = ctypes.POINTER(ctypes.c_double)
_ci, _cd, _cll = ctypes.c_int, ctypes.c_double, ctypes.c_longlong


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        lib = ctypes.CDLL(_LIB)
        lib.oracle_upfirdn2d.argtypes = [_dp, _ci, _ci, _ci, _ci, _dp, _ci, _ci, _ci, _ci, _ci, _ci, _ci, _ci,
                                         _ci, _cd, _dp, _ci, _ci]
        lib.oracle_bias_act.argtypes = [_dp, _dp, _cll, _cll, _ci, _ci, _cd, _cd, _cd, _dp]
        lib.oracle_filtered_lrelu.argtypes = [_dp, _dp, _ci, _ci, _ci, _ci, _dp, _ci, _ci, _dp, _ci, _ci,
                                              _ci, _ci, _ci, _ci, _ci, _ci, _cd, _cd, _cd, _ci,
                                              _dp, _ci, _ci, ctypes.POINTER(ctypes.c_ubyte), _ci, _ci]
        lib.oracle_codebook_argmax.argtypes = [ctypes.c_void_p, _cll, ctypes.c_void_p, _ci, _ci, _ci, ctypes.c_void_p]
        for fn in (lib.oracle_upfirdn2d, lib.oracle_bias_act, lib.oracle_filtered_lrelu, lib.oracle_codebook_argmax):
            fn.restype = None
        _lib = lib
    return _lib


def _d(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data_as(_dp)


def _pads(padding):
    if isinstance(padding, int):
        return padding, padding, padding, padding
    if len(padding) == 2:
        return padding[0], padding[0], padding[1], padding[1]
    return tuple(padding)


def upfirdn2d(x, f, up=1, down=1, padding=0, flip_filter=False, gain=1.0):
    """x: [N,C,H,W]; f: [fh,fw] or separable [k] (applied as outer product, as the
    reference's two 1-D passes with gain**0.5 each)."""
    x, xp = _d(x)
    f = np.asarray(f, dtype=np.float64)
    if f.ndim == 1:
        f = np.outer(f, f)
    f, fp = _d(f)
    upx, upy = (up, up) if isinstance(up, int) else up
    dx, dy = (down, down) if isinstance(down, int) else down
    px0, px1, py0, py1 = _pads(padding)
    n, c, h, w = x.shape
    fh, fw = f.shape
    oh = (h * upy + py0 + py1 - fh + dy) // dy
    ow = (w * upx + px0 + px1 - fw + dx) // dx
    y = np.zeros((n, c, oh, ow))
    _load().oracle_upfirdn2d(xp, n, c, h, w, fp, fh, fw, upx, upy, dx, dy, px0, py0, int(flip_filter), gain,
                             y.ctypes.data_as(_dp), oh, ow)
    return y


ACT_CODES = {'linear': 1, 'relu': 2, 'lrelu': 3, 'tanh': 4, 'sigmoid': 5, 'elu': 6, 'selu': 7, 'softplus': 8,
             'swish': 9}
DEF_GAIN = {'linear': 1.0, 'relu': 2 ** 0.5, 'lrelu': 2 ** 0.5, 'tanh': 1.0, 'sigmoid': 1.0, 'elu': 1.0,
            'selu': 1.0, 'softplus': 1.0, 'swish': 2 ** 0.5}


def bias_act(x, b=None, dim=1, act='linear', alpha=None, gain=None, clamp=None):
    x, xp = _d(x)
    alpha = 0.2 if (alpha is None and act == 'lrelu') else (alpha or 0.0)
    gain = DEF_GAIN[act] if gain is None else gain
    clamp = -1.0 if clamp is None else clamp
    step = int(np.prod(x.shape[dim + 1:])) if b is not None else 1
    bp = None
    if b is not None:
        b, bp = _d(b)
    y = np.zeros_like(x)
    _load().oracle_bias_act(xp, bp, x.size, step, b.size if b is not None else 0, ACT_CODES[act], alpha, gain,
                            clamp, y.ctypes.data_as(_dp))
    return y


def filtered_lrelu(x, fu=None, fd=None, b=None, up=1, down=1, padding=0, gain=2 ** 0.5, slope=0.2, clamp=None,
                   flip_filter=False):
    """Returns (y, codes) where codes[n,c,j,i] in {0,1,2} is the sign code of every
    element of the upsampled intermediate."""
    x, xp = _d(x)
    fu = np.ones((1, 1)) if fu is None else np.asarray(fu, dtype=np.float64)
    fd = np.ones((1, 1)) if fd is None else np.asarray(fd, dtype=np.float64)
    fu = np.outer(fu, fu) if fu.ndim == 1 else fu
    fd = np.outer(fd, fd) if fd.ndim == 1 else fd
    fu, fup = _d(fu)
    fd, fdp = _d(fd)
    bp = None
    if b is not None:
        b, bp = _d(b)
    px0, px1, py0, py1 = _pads(padding)
    n, c, h, w = x.shape
    cw = w * up + px0 + px1 - (fu.shape[1] - 1)
    ch = h * up + py0 + py1 - (fu.shape[0] - 1)
    ow = (cw - (fd.shape[1] - 1) + down - 1) // down
    oh = (ch - (fd.shape[0] - 1) + down - 1) // down
    y = np.zeros((n, c, oh, ow))
    codes = np.zeros((n, c, ch, cw), dtype=np.uint8)
    _load().oracle_filtered_lrelu(xp, bp, n, c, h, w, fup, fu.shape[0], fu.shape[1], fdp, fd.shape[0], fd.shape[1],
                                  up, down, px0, px1, py0, py1, gain, slope,
                                  float('inf') if clamp is None else clamp, int(flip_filter),
                                  y.ctypes.data_as(_dp), oh, ow,
                                  codes.ctypes.data_as(ctypes.POINTER(ctypes.c_ubyte)), ch, cw)
    return y, codes


def codebook_argmax(features, codebook):
    """features [N, C] fp32, codebook [V, C] fp32 -> int64 [N] (first maximal cosine)."""
    f = np.ascontiguousarray(features, dtype=np.float32)
    w = np.ascontiguousarray(codebook, dtype=np.float32)
    n, c = f.shape
    v, c2 = w.shape
    assert c == c2
    idx = np.zeros(n, dtype=np.int64)
    _load().oracle_codebook_argmax(f.ctypes.data, c, w.ctypes.data, n, c, v, idx.ctypes.data)
    return idx
