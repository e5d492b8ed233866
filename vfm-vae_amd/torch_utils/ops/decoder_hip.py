"""Autograd wrappers over the gfx950 decoder kernels (`csrc/decoder.hip`, C ABI in
include/vfmvae.h). Only reached through `decoder_ops.*` for ROCm tensors; the
library is loaded on import and a missing library raises (no silent fallback).

Shapes the kernels do not cover (spatial size not a multiple of 8 for the row
ops, kernel sizes outside {1,3,5,7}) are rejected by `supported()` and the
caller keeps the torch formulation for them — on the same device.

Every launch is bracketed by `kernel_timer.region(name, algorithmic_bytes)`
(inputs + outputs at the op boundary, each tensor counted once) so bench.py can
report the dominant kernel's roofline.
"""
import ctypes
import os
import threading
import weakref

import torch

from .. import custom_ops
from . import kernel_timer

_lib = custom_ops.get_native()
_F32 = 0


def _code(t):
    return custom_ops.dtype_code(t)


def _stream():
    return custom_ops.stream_ptr()


def _c(t):
    """Contiguous and 16-byte aligned (vector loads)."""
    t = t.contiguous()
    if t.data_ptr() % 16:
        t = t.clone()
    return t


def _f32(t):
    if t is None:
        return None
    if t.dtype == torch.float32 and t.is_contiguous():
        return t                      # only the device pointer crosses the ABI
    return t.detach().reshape(-1).float().contiguous()


def _p(t):
    return None if t is None else t.data_ptr()


_DT = {torch.float32: "f32", torch.bfloat16: "bf16", torch.float16: "f16", torch.float64: "f64"}


_RN = {}


def _rn(name, t, *extra):
    """kernel_timer region name: op + template parameters (dtype, tap count), so a timed
    entry maps onto one kernel instantiation of the rocprofv3 trace (memoised: this runs on every
    launch's host path)."""
    key = (name, t.dtype, extra)
    out = _RN.get(key)
    if out is None:
        out = _RN[key] = f"{name}<{','.join([_DT.get(t.dtype, str(t.dtype))] + [str(e) for e in extra])}>"
    return out


class _LazyBytes:
    """Algorithmic bytes of a launch's tensors, summed only when the timer samples the launch
    (kernel_timer calls int()) -- the sum is host work on every launch otherwise."""
    __slots__ = ("ts",)

    def __init__(self, ts):
        self.ts = ts

    def __int__(self):
        return sum(t.numel() * t.element_size() for t in self.ts if t is not None)

    def __add__(self, other):
        return int(self) + other

    __radd__ = __add__


def _nb(*ts):
    return _LazyBytes(ts)


def _check(rc, name):
    custom_ops.check(rc, name)


def _edges(ctx, *args):
    """Map forward-argument index -> index into ctx.next_functions (which has one entry per
    tensor argument, None/int arguments have no edge)."""
    n, edge = 0, []
    for a in args:
        edge.append(n if isinstance(a, torch.Tensor) else None)
        n += isinstance(a, torch.Tensor)
    ctx.edge = edge


def _wanted(ctx, i):
    """Input i needs a gradient in THIS backward pass: requires_grad at forward time AND the
    autograd engine will run the node that consumes it. `torch.autograd.grad(loss, inputs)`
    executes only the graph between loss and `inputs` -- e.g. the adaptive VF weight's
    grad(rec_loss, last_layer) (reference training/loss.py:262-271) runs the decoder backward
    for the data path only -- so parameter gradients are skipped there exactly as torch's
    built-in conv/matmul backward nodes skip them."""
    if not ctx.needs_input_grad[i]:
        return False
    fn = ctx.next_functions[ctx.edge[i]][0]
    if fn is None:
        return False
    try:
        return bool(torch._C._will_engine_execute_node(fn))
    except RuntimeError:          # not inside an engine-driven backward
        return True


def supported(op, x, **kw):
    if x.dtype not in (torch.float32, torch.float16, torch.bfloat16):
        return False
    if op == 'dwconv2d':
        return kw['k'] in (1, 3, 5, 7) and x.ndim == 4
    if op in ('scale_bias_gelu', 'layer_scale_residual'):
        return x.shape[-1] % 8 == 0 if x.ndim == 3 else (x.shape[-1] * x.shape[-2]) % 8 == 0
    if op == 'group_norm':
        return x.ndim >= 3 and x.shape[1] % kw['groups'] == 0
    if op == 'shuffle_blur':
        return 1 <= kw['k'] <= 8 and kw.get('r', 1) in (1, 2)
    return False


# ---------------------------------------------------------------------------
# 1x1 conv as a stride-0-batch GEMM (hipBLASLt through torch.bmm), no layout copies.


_NO_CAST_CACHE = os.environ.get("VFM_NO_CAST_CACHE", "0") == "1"


def _cast_cached(w, dtype):
    """w.detach().to(dtype), cached on the parameter until it changes (its version counter
    moves at every optimizer step): the D-phase and G-phase forwards of one iteration share
    one cast of each decoder weight. Not while a HIP graph is being captured (the cached tensor
would be baked into the graph and go stale after the next optimizer step)."""
    if w.dtype == dtype:
        return w.detach()
    if _NO_CAST_CACHE or torch.cuda.is_current_stream_capturing():
        return w.detach().to(dtype)     # a graph must recompute the cast at every replay
    base = w._base if w._base is not None else w
    key = (tuple(w.shape), w.stride(), w.storage_offset(), dtype, base._version)
    hit = getattr(base, "_vfm_cast", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    wc = w.detach().to(dtype)
    try:
        base._vfm_cast = (key, wc)
    except AttributeError:
        pass
    return wc


# The data gradients W^T dY of the fp32 1x1 convolutions read W^T as the GEMM's A operand: as a view it is
# M-contiguous, which gemm9 stages with transposed LDS reads (two ds_read_b64_tr_b16 per fragment); a row-major
# copy of W^T (K-contiguous A, its f32x6 pieces split once) runs the kernel's direct-read form: f32x6 data-gradient
# GEMM time 24.1 -> 19.9 ms/step (same-box A/B, profiles/r5_am_wt_copy_ab.txt). Not for bf16 weights (their (t, f)
# form measured 0.6 ms/step slower than the transposed reads). Weights change once per optimizer step, so the copy
# is cached on the weight until its version moves (not while a HIP graph is captured). VFM_WT_COPY=0: the view.
_WT_COPY = os.environ.get("VFM_WT_COPY", "1") == "1"


def _wt(w, contiguous=False):
    """W^T of a [O, I] fp32 weight as a contiguous [I, O] tensor (cached per weight version), else the view;
    contiguous=True: the cached contiguous copy for any dtype (kernels that take W^T as a plain row-major array)."""
    if not contiguous and (not _WT_COPY or not w.is_cuda or w.dim() != 2 or w.dtype != torch.float32):
        return w.t()
    if torch.cuda.is_current_stream_capturing():
        return w.t().contiguous()
    base = w._base if w._base is not None else w
    key = (w.data_ptr(), tuple(w.shape), w.stride(), w.dtype, base._version)
    hit = getattr(base, "_vfm_wt", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    wt = w.detach().t().contiguous()
    try:
        base._vfm_wt = (key, wt)
    except AttributeError:
        pass
    return wt


# Dense products of the decoder on the MFMA GEMM (csrc/gemm.hip: bf16, or fp32 operands with
# fp32-equivalent f32x6 products); VFM_GEMM=torch keeps hipBLASLt (A/B switch). Shapes the kernel does not
# cover fall back to torch.bmm explicitly.
_USE_HIP_GEMM = os.environ.get("VFM_GEMM", "hip") != "torch"


def _gemm(A, B, **kw):
    if not _USE_HIP_GEMM:
        return None
    from . import gemm_hip
    return gemm_hip.try_gemm(A, B, auto=True, **kw)


def _tn(t):
    return {torch.float32: "f32", torch.bfloat16: "bf16", torch.float16: "f16"}.get(t.dtype, str(t.dtype))


def weight_grad_1x1(dy, x, wdt):
    """sum_b dy[b] @ x[b]^T in fp32 -> wdt ([O, P] x [I, P] per sample). Planes whose P is not a
    multiple of the 64-deep K-tile (the 2x2 .. 12x12 maps: P = 4, 16, 36, 144) would fill a fraction
    P / 64 of every K-tile of the batch-reduced kernel (3-60 TF/s in the step, r4g shape table): those
    are gathered once into [O, B P] / [I, B P] (a few MB) and run as one product over K = B P."""
    B, O, P = dy.shape
    if dy.dtype == torch.float32 and P % 64 and (B * P) % 64 == 0 and _USE_HIP_GEMM:
        dyc = dy.permute(1, 0, 2).reshape(O, B * P)
        xc = x.permute(1, 0, 2).reshape(x.shape[1], B * P)
        dw = _gemm(dyc, xc.t(), out_dtype=torch.float32)
        if dw is not None:
            return dw.to(wdt)
    dw = _gemm(dy, x.transpose(1, 2), out_dtype=torch.float32, reduce_batch=True,
               splits=_splits(dy.shape[1], x.shape[1], dy.shape[2], dy.shape[0]))
    if dw is None:
        B, O, P = dy.shape
        with kernel_timer.vendor_gemm(f"{_tn(dy)},1x1_dw", O, x.shape[1], P, B, dy.element_size()):
            dw = torch.bmm(dy, x.transpose(1, 2), out_dtype=torch.float32) if dy.dtype != torch.float32 else \
                torch.bmm(dy, x.transpose(1, 2))
        dw = dw.sum(0)
    return dw.to(wdt)


def _splits(M, N, K, z):
    """K splits so that the grid has >= ~1024 workgroups (256 CUs x 4), each split >= 512 deep."""
    tiles = -(-M // 128) * -(-N // 128) * z
    want = -(-1024 // tiles)
    return max(1, min(want, K // 512, 64))


# The backward's weight-gradient and data-gradient GEMMs are independent; on the bf16 (hipBLASLt) path they
# are ridge-shaped (K = 512-2048 against 4096-65536-column planes: MFMA-bound K-loops, then output-write-
# bound epilogues in synchronized tile rounds). VFM_DW_STREAM=1 runs the weight gradient on a side stream
# next to the data gradient so one kernel's write phase can overlap the other's K-loop; measured slower
# (same-box A/B, profiles/r4_s_dw_stream_ab.txt: 95.95 / 95.61 img/s with it, 96.72 / 97.66 without), so
# it is off by default.
_DW_STREAM = os.environ.get("VFM_DW_STREAM", "0") == "1"
_side_streams = {}


def _overlapped(side_fn, main_fn, dev):
    """(side_fn(), main_fn()) with side_fn enqueued on a side stream of `dev` (after everything queued so
    far on the current stream) and the current stream waiting for it before anything later runs."""
    if not (_DW_STREAM and dev.type == 'cuda') or torch.cuda.is_current_stream_capturing():
        return side_fn(), main_fn()
    side = _side_streams.get(dev.index)
    if side is None:
        side = _side_streams[dev.index] = torch.cuda.Stream(device=dev)
    cur = torch.cuda.current_stream(dev)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        a = side_fn()
    b = main_fn()
    cur.wait_stream(side)
    return a, b


class _Pointwise(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, w, x):
        _edges(ctx, w, x)
        x = x.contiguous()
        B, I, P = x.shape
        O = w.shape[0]
        wc = _cast_cached(w, x.dtype)
        ctx.save_for_backward(wc, x)
        ctx.wdt = w.dtype
        y = _gemm(wc, x, cache_a=True)
        if y is None:
            with kernel_timer.vendor_gemm(f"{_tn(x)},1x1", O, P, I, B, x.element_size()):
                y = torch.bmm(wc.expand(B, O, I), x)
        return y

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dy):
        wc, x = ctx.saved_tensors
        B, I, P = x.shape
        O = wc.shape[0]
        dy = dy.contiguous()

        def wgrad():      # sum_b dy[b] @ x[b]^T with fp32 per-sample products, summed in fp32
            return weight_grad_1x1(dy, x, ctx.wdt)

        def dgrad():
            dx = _gemm(_wt(wc), dy, cache_a=True)
            if dx is None:
                with kernel_timer.vendor_gemm(f"{_tn(dy)},1x1_dx", I, P, O, B, dy.element_size()):
                    dx = torch.bmm(wc.t().expand(B, I, O), dy)
            return dx
        want_w, want_x = _wanted(ctx, 0), _wanted(ctx, 1)
        if want_w and want_x and dy.dtype != torch.float32:
            # (fp32 operands stay on one stream: their piece splits are shared between the two products)
            dw, dx = _overlapped(wgrad, dgrad, dy.device)
        else:
            dw = wgrad() if want_w else None
            dx = dgrad() if want_x else None
        return dw, dx


def pointwise(w, x):
    return _Pointwise.apply(w, x)


# ---------------------------------------------------------------------------
# Depthwise conv (reference convnext_utils.py:121-124 / :243: nn.Conv2d(groups=C)).


DW_MFMA = os.environ.get("VFM_DW_MFMA", "1") == "1"      # A/B switch for the banded-MFMA dwconv


GN_STATS = os.environ.get("VFM_GN_STATS", "1") == "1"      # A/B switch: GroupNorm statistics from the dwconv
# The handoff is per thread (threading.local) and keyed on the output tensor itself (weakref), its device, storage
# pointer, shape and version. Contract: nothing writes y in place between the dwconv and the GroupNorm that consumes
# it -- the one consumer is the next op of ConvNeXtSynthesisLayer.forward (networks/utils/convnext_utils.py), and a
# torch in-place write bumps y._version, which voids the handoff; a raw-pointer write by a native kernel would not,
# and none exists on that edge.
_gn_tls = threading.local()     # .e = (weakref of y, device, data_ptr, version, shape, partials, units per plane)


def _gn_stats_for(x):
    """The dwconv's GroupNorm partials when x is that dwconv's unchanged output (one consumer)."""
    e = getattr(_gn_tls, "e", None)
    _gn_tls.e = None
    if e is None:
        return None
    yref, dev, ptr, ver, shape, part, upc = e
    y = yref()
    if (y is None or x.data_ptr() != ptr or x.shape != shape or x.device != dev or x._version != ver
            or y._version != ver):
        return None
    return part, upc


def _dw_fwd(x, w3, bias, noise, pad, name, res=None, flip=False, nplane=None, gstat=False):
    """y = dwconv(x) (+ bias, + noise plane) (+ res, a tensor of y's shape: the residual-branch
    gradient added in the MFMA kernel's epilogue, else by a torch add); flip: taps rotated by 180
    degrees in the kernel (the data gradient). nplane ([H, W] fp32): also return sum x * nplane over
    (b, c, y, x) as a 0-d fp32 tensor -- from per-wave partials of the MFMA kernel when it runs, else
    by torch -- i.e. (y, dot). gstat: the MFMA kernel also writes y's GroupNorm partials, which the
    GroupNorm that consumes y picks up (_gn_stats_for) instead of its own statistics pass."""
    B, C, H, W = x.shape
    K = w3.shape[-1]
    Ho, Wo = H + 2 * pad - K + 1, W + 2 * pad - K + 1
    y = torch.empty([B, C, Ho, Wo], dtype=x.dtype, device=x.device)
    if res is not None:
        res = res.reshape(y.shape)            # handed over as the residual's [B, C, P] view
    if DW_MFMA and x.dtype == torch.bfloat16 and 2 * pad == K - 1:
        # bf16 planes: the banded-MFMA kernel (csrc/dwconv_mfma.hip); taps rounded to bf16 as
        # the reference's autocast conv does
        r = None if res is None else _c(res.to(torch.bfloat16))
        if gstat and GN_STATS and r is None and not flip and nplane is None and Ho == H and Wo == W:
            units = _lib.vfm_dwconv2d_fwd_mfma_units(B, C, H, W, K, pad)
            if units > 0:
                gs = torch.empty([units, 4], dtype=torch.float32, device=x.device)
                with kernel_timer.region(_rn(name.replace('dwconv2d', 'dwconv2d_mfma'), x, K), _nb(x, y)):
                    rc = _lib.vfm_dwconv2d_fwd_mfma_gs(x.data_ptr(), w3.data_ptr(), _p(bias), _p(noise),
                                                       y.data_ptr(), gs.data_ptr(), B, C, H, W, K, pad, _stream())
                if rc != custom_ops.VFM_NO_KERNEL:
                    _check(rc, name)
                    _gn_tls.e = (weakref.ref(y), y.device, y.data_ptr(), y._version, y.shape, gs, units // (B * C))
                    return y
        part = None
        if nplane is not None and Ho == H and Wo == W:
            units = _lib.vfm_dwconv2d_fwd_mfma_units(B, C, H, W, K, pad)
            part = torch.empty([units], dtype=torch.float32, device=x.device) if units > 0 else None
        with kernel_timer.region(_rn(name.replace('dwconv2d', 'dwconv2d_mfma'), x, K), _nb(x, y, r)):
            rc = _lib.vfm_dwconv2d_fwd_mfma_nz(x.data_ptr(), w3.data_ptr(), _p(bias), _p(noise), _p(r), y.data_ptr(),
                                               _p(nplane if part is not None else None), _p(part), B, C, H, W, K,
                                               pad, int(flip), _stream())
        if rc != custom_ops.VFM_NO_KERNEL:
            _check(rc, name)
            if nplane is None:
                return y
            return y, (part.sum() if part is not None else _plane_dot(x, nplane))
    r = None if res is None else _c(res.to(y.dtype))       # added in the kernel's store (no torch add)
    with kernel_timer.region(_rn(name, x, K), _nb(x, y, r)):
        _check(_lib.vfm_dwconv2d_fwd_res(x.data_ptr(), w3.data_ptr(), _p(bias), _p(noise), _p(r), y.data_ptr(),
                                         _code(x), B, C, H, W, K, pad, int(flip), _stream()), name)
    return y if nplane is None else (y, _plane_dot(x, nplane))


def _plane_dot(x, plane):
    """sum_{b, c, y, x} x * plane[y, x] (fp32 accumulation, no fp32 copy of x)."""
    return (x.sum(dim=(0, 1), dtype=torch.float32) * plane).sum()


RESIDUAL_FUSION = os.environ.get("VFM_RESIDUAL_FUSION", "1") == "1"     # A/B switch (tests, benches)


class ResidualSlot:
    """Hands a ConvNeXt layer's residual-branch gradient (d out / d x_in = d out) from the layer-scale
    residual's backward to the backward of the layer's depthwise conv, whose data-gradient kernel
    adds it in its epilogue: x feeds both the dwconv and the residual, and autograd would otherwise
    sum the two gradients in a separate full-tensor add. Used only when the dwconv input IS x_in
    (no cast in between) and the dwconv's backward node will run in the same engine pass."""
    __slots__ = ("node", "grad")

    def __init__(self):
        self.node = None
        self.grad = None


def _stash_residual(slot, dout):
    """True when the residual gradient was handed to the dwconv backward (return None for x_in)."""
    if slot is None or slot.node is None:
        return False
    try:
        if not torch._C._will_engine_execute_node(slot.node):
            return False
    except RuntimeError:
        return False
    slot.grad = dout
    return True


def _dw_wgrad(part, want_w, want_b, C, K, wshape, wdt, bdt):
    """(dw, db) from the weight-gradient partials [rows, C, K K + 1] in one reduce launch."""
    dw = torch.empty(wshape, dtype=torch.float32, device=part.device) if want_w else None
    db = torch.empty([C], dtype=torch.float32, device=part.device) if want_b else None
    _check(_lib.vfm_dwconv2d_wgrad_reduce(part.data_ptr(), _p(dw), _p(db), part.shape[0], C, K * K, _stream()),
           'vfm_dwconv2d_wgrad_reduce')
    return (None if dw is None else dw.to(wdt)), (None if db is None else db.to(bdt))


class _DwConv2d(custom_ops.FastFunction):
    """Depthwise conv (+ bias) (+ noise plane, or noise plane * strength for the legacy noise: then
    `noise` is the constant plane and the strength's gradient sum dY * plane comes out of the data-
    gradient kernel's pass over dY, decoder_hip._dw_fwd nplane)."""

    @staticmethod
    def forward(ctx, x, weight, bias, noise, pad, slot, strength=None):
        _edges(ctx, x, weight, bias, noise, pad, slot, strength)
        ctx.slot = slot
        x = _c(x)
        C, K = weight.shape[0], weight.shape[-1]
        w3 = weight.detach().reshape(C, K, K).float().contiguous()
        b = _f32(bias)
        n = None if noise is None else noise.detach().float().contiguous()
        plane = None
        ctx.strength = None
        if strength is not None:
            plane = n
            ctx.strength = strength.detach().float()
            n = (n * ctx.strength).contiguous()
        y = _dw_fwd(x, w3, b, n, pad, 'dwconv2d_fwd', gstat=True)
        ctx.save_for_backward(x, w3, plane)
        ctx.pad = pad
        ctx.meta = (weight.dtype, weight.shape, None if bias is None else bias.dtype,
                    None if noise is None else noise.dtype, None if strength is None else strength.dtype)
        return y

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dy):
        x, w3, plane = ctx.saved_tensors
        pad = ctx.pad
        wdt, wshape, bdt, ndt, sdt = ctx.meta
        dy = _c(dy.to(x.dtype))
        B, C, H, W = x.shape
        K = w3.shape[-1]
        dx = dw = db = dn = dstr = None
        want_w, want_b = _wanted(ctx, 1), _wanted(ctx, 2)
        want_s = plane is not None and _wanted(ctx, 6)
        res = None
        if ctx.slot is not None and ctx.slot.grad is not None:
            res, ctx.slot.grad = ctx.slot.grad, None
        if _wanted(ctx, 0):
            out = _dw_fwd(dy, w3, None, None, K - 1 - pad, 'dwconv2d_bwd_data', res, flip=True,
                          nplane=plane if want_s else None)
            dx, dstr = out if want_s else (out, None)
        # (res unused when dx is not wanted: then nothing consumes x's gradient in this pass)
        if (want_w or want_b) and DW_MFMA and x.dtype == torch.bfloat16 and \
                _lib.vfm_dwconv2d_bwd_weight_mfma_tiles(B, C, H, W, K, pad) > 0:
            # bf16 planes: the weight gradient as banded MFMA products (csrc/dwconv_mfma.hip)
            tiles = _lib.vfm_dwconv2d_bwd_weight_mfma_tiles(B, C, H, W, K, pad)
            part = torch.empty([tiles, C, K * K + 1], dtype=torch.float32, device=x.device)
            with kernel_timer.region(_rn('dwconv2d_mfma_bwd_weight', x, K), _nb(x, dy)):
                _check(_lib.vfm_dwconv2d_bwd_weight_mfma(x.data_ptr(), dy.data_ptr(), part.data_ptr(), B, C, H, W, K,
                                                         pad, _stream()), 'vfm_dwconv2d_bwd_weight_mfma')
            dw, db = _dw_wgrad(part, want_w, want_b, C, K, wshape, wdt, bdt)
        elif want_w or want_b:
            tiles = _lib.vfm_dwconv2d_bwd_weight_tiles(B, C, H, W, K, pad)
            if tiles <= 0:
                raise custom_ops.NativeError(f"vfm_dwconv2d_bwd_weight_tiles failed with code {tiles}")
            part = torch.empty([tiles, C, K * K + 1], dtype=torch.float32, device=x.device)
            with kernel_timer.region(_rn('dwconv2d_bwd_weight', x, K), _nb(x, dy)):
                _check(_lib.vfm_dwconv2d_bwd_weight(x.data_ptr(), dy.data_ptr(), part.data_ptr(), _code(x),
                                                    B, C, H, W, K, pad, _stream()), 'vfm_dwconv2d_bwd_weight')
            dw, db = _dw_wgrad(part, want_w, want_b, C, K, wshape, wdt, bdt)
        if want_s and dstr is None:
            dstr = _plane_dot(dy, plane)
        if _wanted(ctx, 3):
            dn = dy.sum(dim=(0, 1), dtype=torch.float32)                  # fp32 accumulation, no fp32 copy of dy
            dn = (dn if plane is None else dn * ctx.strength).to(ndt)      # d plane = strength * sum_{b,c} dy
        return dx, dw, db, dn, None, None, (None if dstr is None else dstr.reshape(()).to(sdt))


def dwconv2d(x, weight, bias, padding, noise, slot=None, noise_strength=None):
    y = _DwConv2d.apply(x, weight, bias, noise, int(padding), slot, noise_strength)
    if slot is not None:
        slot.node = y.grad_fn
    return y


# ---------------------------------------------------------------------------
# GroupNorm with fp32 statistics and the folded style scale
# (reference shared.py:165-167 GroupNorm32; convnext_utils.py:126-127).


def _colsum2(a, b, scale_a, want_a, want_b, rows, cols):
    """(scale_a * a.view(rows, cols).sum(0) if want_a, b.view(rows, cols).sum(0) if want_b) in one launch."""
    if not (want_a or want_b):
        return None, None
    oa = torch.empty([cols], dtype=torch.float32, device=a.device) if want_a else None
    ob = torch.empty([cols], dtype=torch.float32, device=a.device) if want_b else None
    sc = None if scale_a is None else _f32(scale_a)
    _check(_lib.vfm_colsum2_f32(a.data_ptr(), b.data_ptr(), _p(sc), _p(oa), _p(ob), rows, cols, _stream()),
           'vfm_colsum2_f32')
    return oa, ob


class _GroupNorm(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, x, weight, bias, style, groups, eps, out_dtype):
        _edges(ctx, x, weight, bias, style, groups, eps, out_dtype)
        x = _c(x)
        B, C = x.shape[:2]
        HW = x[0, 0].numel()
        w, b = _f32(weight), _f32(bias)
        s = None if style is None else style.detach().float().contiguous()
        y = torch.empty(x.shape, dtype=out_dtype, device=x.device)
        mean = torch.empty([B * groups], dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        st = _gn_stats_for(x) if x.dtype == torch.bfloat16 and y.dtype in (torch.bfloat16, torch.float32) else None
        if st is not None:
            # statistics merged from the producing dwconv's partials: x is read once
            with kernel_timer.region(_rn('group_norm_fwd_stats', x), _nb(x, y)):
                _check(_lib.vfm_group_norm_fwd_stats(x.data_ptr(), _p(w), _p(b), _p(s), y.data_ptr(), mean.data_ptr(),
                                                     rstd.data_ptr(), st[0].data_ptr(), st[1], _code(x), _code(y), B,
                                                     C, groups, HW, float(eps), _stream()), 'vfm_group_norm_fwd_stats')
        else:
            # the ConvNeXt layer's GN(d) * s (style given) feeds pwconv1's f32x6 product: pieces written here
            yp = _pieces_for(y, HW) if (s is not None and HW % 8 == 0) else None
            with kernel_timer.region(_rn('group_norm_fwd', x), _nb(x, y, yp)):
                _check(_lib.vfm_group_norm_fwd_pc(x.data_ptr(), _p(w), _p(b), _p(s), y.data_ptr(), _p(yp),
                                                  mean.data_ptr(), rstd.data_ptr(), _code(x), _code(y), B, C, groups,
                                                  HW, float(eps), _stream()), 'vfm_group_norm_fwd')
            _attach_pieces(y, yp)
        ctx.save_for_backward(x, w, b, s, mean, rstd)
        ctx.groups = groups
        ctx.meta = tuple(None if t is None else t.dtype for t in (weight, bias, style))
        return y

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dy):
        x, w, b, s, mean, rstd = ctx.saved_tensors
        B, C = x.shape[:2]
        HW = x[0, 0].numel()
        dy = _c(dy)
        dx = torch.empty_like(x)
        dwp = torch.empty([B, C], dtype=torch.float32, device=x.device)
        dbp = torch.empty_like(dwp)
        ds = torch.empty_like(dwp) if s is not None else None
        with kernel_timer.region(_rn('group_norm_bwd', x), _nb(x, dy, dx)):
            _check(_lib.vfm_group_norm_bwd(x.data_ptr(), dy.data_ptr(), mean.data_ptr(), rstd.data_ptr(), _p(w),
                                           _p(b), _p(s), dx.data_ptr(), dwp.data_ptr(), dbp.data_ptr(), _p(ds),
                                           _code(x), _code(dy), B, C, ctx.groups, HW, _stream()),
                   'vfm_group_norm_bwd')
        wdt, bdt, sdt = ctx.meta
        dw, db = _colsum2(dwp, dbp, None, _wanted(ctx, 1), _wanted(ctx, 2), B, C)
        dw = None if dw is None else dw.to(wdt)
        db = None if db is None else db.to(bdt)
        dst = ds.to(sdt) if _wanted(ctx, 3) else None
        return (dx if ctx.needs_input_grad[0] else None), dw, db, dst, None, None, None


def group_norm(x, num_groups, weight, bias, eps, out_dtype, style):
    return _GroupNorm.apply(x, weight, bias, style, int(num_groups), float(eps), out_dtype)


# ---------------------------------------------------------------------------
# Modulated pwconv1 epilogue: gelu(h * dcoef[b, o] + bias[o])
# (reference convnext_utils.py:60-66 demodulation, :129-130 bias + GELU).


PRODUCER_PIECES = os.environ.get("VFM_PRODUCER_PIECES", "1") == "1"


def _pieces_for(t, P):
    """A planar [3, numel] bf16 piece buffer for the fp32 output t of a row kernel that feeds the f32x6 GEMMs
    (planes of >= 64 pixels: narrower products go to the exact-fp32 GEMM, which takes no pieces), or None."""
    if not (PRODUCER_PIECES and t.dtype == torch.float32 and P >= 64 and gemm_pieces_mode() == 3) or \
            torch.cuda.is_current_stream_capturing():
        return None
    return torch.empty((3, t.numel()), dtype=torch.bfloat16, device=t.device)


def gemm_pieces_mode():
    return custom_ops.f32_precision()[1]


def _attach_pieces(t, pieces):
    """Hand the producer-written pieces to gemm_hip._planar's per-tensor cache (same key it computes), so the
    products of t skip their split pass."""
    if pieces is not None and not torch.cuda.is_current_stream_capturing():
        t._vfm_planar = ((t.data_ptr(), t.numel(), t._version, custom_ops.f32_precision()[0]), pieces)


class _ScaleBiasGelu(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, h, scale, bias):
        _edges(ctx, h, scale, bias)
        h = _c(h)
        B, O = h.shape[:2]
        P = h[0, 0].numel()
        s, b = _f32(scale), _f32(bias)
        g = torch.empty_like(h)
        gp = _pieces_for(g, P)
        with kernel_timer.region(_rn('scale_bias_gelu_fwd', h), _nb(h, g, gp)):
            _check(_lib.vfm_scale_bias_gelu_fwd_pc(h.data_ptr(), _p(s), _p(b), g.data_ptr(), _p(gp), _code(h), B, O, P,
                                                   _stream()), 'vfm_scale_bias_gelu_fwd')
        _attach_pieces(g, gp)
        ctx.save_for_backward(h, s, b)
        ctx.meta = (None if scale is None else scale.dtype, None if bias is None else bias.dtype)
        return g

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dg):
        h, s, b = ctx.saved_tensors
        B, O = h.shape[:2]
        P = h[0, 0].numel()
        dg = _c(dg)
        dh = torch.empty_like(h)
        want_s = s is not None and _wanted(ctx, 1)
        ds_rows = torch.empty([B * O], dtype=torch.float32, device=h.device) if want_s else None
        db_rows = torch.empty([B * O], dtype=torch.float32, device=h.device)
        dhp = _pieces_for(dh, P) if ctx.needs_input_grad[0] else None
        with kernel_timer.region(_rn('scale_bias_gelu_bwd', h), _nb(h, dg, dh, dhp)):
            _check(_lib.vfm_scale_bias_gelu_bwd_pc(h.data_ptr(), dg.data_ptr(), _p(s), _p(b), dh.data_ptr(), _p(dhp),
                                                   _p(ds_rows), db_rows.data_ptr(), _code(h), B, O, P, _stream()),
                   'vfm_scale_bias_gelu_bwd')
        _attach_pieces(dh, dhp)
        sdt, bdt = ctx.meta
        ds = ds_rows.view(B, O).to(sdt) if want_s else None
        db = db_rows.view(B, O).sum(0).to(bdt) if (b is not None and _wanted(ctx, 2)) else None
        return (dh if ctx.needs_input_grad[0] else None), ds, db


def scale_bias_gelu(h, scale, bias):
    return _ScaleBiasGelu.apply(h, scale, bias)


# ---------------------------------------------------------------------------
# pwconv2 bias + layer scale + residual (reference convnext_utils.py:131-142).


class _LayerScaleResidual(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, y, bias, gamma, x_in, slot=None):
        _edges(ctx, y, bias, gamma, x_in, slot)
        ctx.slot = slot
        y, x_in = _c(y), _c(x_in)
        B, C = y.shape[:2]
        P = y[0, 0].numel()
        b, g = _f32(bias), _f32(gamma)
        out = torch.empty(x_in.shape, dtype=x_in.dtype, device=x_in.device)
        with kernel_timer.region(_rn('layer_scale_residual_fwd', y), _nb(y, x_in, out)):
            _check(_lib.vfm_layer_scale_residual_fwd(y.data_ptr(), _p(b), _p(g), x_in.data_ptr(), out.data_ptr(),
                                                     _code(y), _code(x_in), B, C, P, _stream()),
                   'vfm_layer_scale_residual_fwd')
        ctx.save_for_backward(y, b, g)
        ctx.meta = (None if bias is None else bias.dtype, None if gamma is None else gamma.dtype, x_in.dtype)
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dout):
        y, b, g = ctx.saved_tensors
        bdt, gdt, xdt = ctx.meta
        B, C = y.shape[:2]
        P = y[0, 0].numel()
        dout = _c(dout.to(xdt))
        dy = torch.empty_like(y)
        r0 = torch.empty([B * C], dtype=torch.float32, device=y.device)
        r1 = torch.empty_like(r0)
        dyp = _pieces_for(dy, P) if ctx.needs_input_grad[0] else None
        with kernel_timer.region(_rn('layer_scale_residual_bwd', y), _nb(y, dout, dy, dyp)):
            _check(_lib.vfm_layer_scale_residual_bwd_pc(y.data_ptr(), _p(b), _p(g), dout.data_ptr(), dy.data_ptr(),
                                                        _p(dyp), r0.data_ptr(), r1.data_ptr(), _code(y), _code(dout),
                                                        B, C, P, _stream()), 'vfm_layer_scale_residual_bwd')
        _attach_pieces(dy, dyp)
        db, dg = _colsum2(r1, r0, g, b is not None and _wanted(ctx, 1), g is not None and _wanted(ctx, 2), B, C)
        db = None if db is None else db.to(bdt)
        dg = None if dg is None else dg.to(gdt)
        dx = dout if ctx.needs_input_grad[3] and not _stash_residual(ctx.slot, dout) else None
        return (dy if ctx.needs_input_grad[0] else None), db, dg, dx, None


def layer_scale_residual(y, bias, gamma, x_in, slot=None):
    if bias is not None:
        bias = bias.reshape(-1)
    if gamma is not None:
        gamma = gamma.reshape(-1)
    return _LayerScaleResidual.apply(y, bias, gamma, x_in, slot)


# ---------------------------------------------------------------------------
# Whole ConvNeXt MLP without autograd (reference convnext_utils.py:135-142): the D phase's
# no-grad generator pass keeps the 4C hidden tensor on chip (csrc/pwgemm.hip mlp_fwd).

# measured faster than the unfused chain only at C = 128 (b5 256^2); VFM_NO_FUSED_MLP=1 for A/B
MLP_CHANNELS = () if os.environ.get("VFM_NO_FUSED_MLP") else (128,)
# wider layers (b3: C = 512 at 64^2, b4: C = 256 at 128^2): the two 1x1s on the persistent 256-tile GEMM
# (csrc/gemm9.hip) with the GELU fused into pwconv1's epilogue (forward: h and g, or g alone without
# autograd) and into the 4C-wide data gradient's (backward: dh and the d_s / d_b1 row sums), no separate
# scale_bias_gelu passes; VFM_GEMM_MLP=0: the unfused chain (pointwise GEMMs + GELU row kernels, A/B)
GEMM_MLP_CHANNELS = () if os.environ.get("VFM_GEMM_MLP") == "0" else (256, 512)
# the backward's GELU' in the 4C-wide data gradient's epilogue (vfm_gemm9_gelu mode 2) instead of a plain
# GEMM + the GELU' row kernel: opt-in (VFM_GEMM_MLP_BWD=1), slower at one wave per SIMD (see backward)
GEMM_MLP_BWD_EPI = os.environ.get("VFM_GEMM_MLP_BWD") == "1"
GEMM_MLP_TESTED = (256, 512)


def convnext_mlp_supported(m, C, P):
    if not (m.is_cuda and m.dtype == torch.bfloat16):
        return False
    if C in MLP_CHANNELS:
        return P % 128 == 0
    return C in GEMM_MLP_CHANNELS and P % 8 == 0


def _g8(A, B, **kw):
    """bf16 product on the persistent 256-tile kernel (gemm_hip route ("g9", 0), csrc/gemm9.hip); raises if not
    covered."""
    from . import gemm_hip
    out = gemm_hip.try_gemm(A, B, route=("g9", 0), **kw)
    if out is None:
        raise custom_ops.NativeError(f"vfm_gemm9 does not cover {tuple(A.shape)} x {tuple(B.shape)}")
    return out


def gemm_gelu_fwd(w1c, m, s, b1, want_h=True):
    """(h, g): h = W1 m[b] (bf16 [B, O, P], None unless want_h) and g = GELU(h s[b] + b1) in one
    GEMM (vfm_gemm9_gelu mode 1). w1c bf16 [O, I] contiguous, m bf16 [B, I, P], s fp32 [B, O] or
    None, b1 fp32 [O] or None."""
    B, I, P = m.shape
    O = w1c.shape[0]
    g = torch.empty([B, O, P], dtype=torch.bfloat16, device=m.device)
    h = torch.empty_like(g) if want_h else None
    with kernel_timer.region('gemm9_gelu<1>', _nb(m, g, h) + w1c.numel() * 2, flops=2.0 * B * O * I * P, bound="mfma"):
        _check(_lib.vfm_gemm9_gelu(w1c.data_ptr(), m.data_ptr(), _p(h), g.data_ptr(), None, _p(s), _p(b1), None, None,
                                   1, O, P, I, B, w1c.stride(0), m.stride(1), m.stride(0), P, O * P, _stream()),
               'vfm_gemm9_gelu')
    return h, g


def gemm_gelu_bwd(w2t, dy, h, s, b1):
    """dh = (W2^T dy[b]) GELU'(h s + b1) s with the per-(b, o) sums for d_s ([B, O], None when s is
    None) and d_b1 ([O]) (vfm_gemm9_gelu mode 2). w2t bf16 [O, C] contiguous, dy bf16 [B, C, P]."""
    B, C, P = dy.shape
    O = w2t.shape[0]
    parts = _lib.vfm_gemm9_gelu_parts(P)
    dh = torch.empty_like(h)
    p1 = torch.empty([B, parts, O], dtype=torch.float32, device=dy.device)
    p0 = torch.empty_like(p1) if s is not None else None
    with kernel_timer.region('gemm9_gelu<2>', _nb(dy, h, dh) + w2t.numel() * 2, flops=2.0 * B * O * C * P,
                             bound="mfma"):
        _check(_lib.vfm_gemm9_gelu(w2t.data_ptr(), dy.data_ptr(), dh.data_ptr(), None, h.data_ptr(), _p(s), _p(b1),
                                   _p(p0), p1.data_ptr(), 2, O, P, C, B, w2t.stride(0), dy.stride(1), dy.stride(0), P,
                                   O * P, _stream()), 'vfm_gemm9_gelu')
    return dh, (p0.sum(1) if p0 is not None else None), p1.sum((0, 1))


class _ConvNeXtMLPGemm(custom_ops.FastFunction):
    """The ConvNeXt MLP of the wide bf16 blocks (reference convnext_utils.py:135-142) on the 256-tile
    GEMM: forward pwconv1 + scale/bias/GELU in one kernel (h and g written for the backward), pwconv2,
    the layer-scale residual kernel; backward: the residual kernel's dy, dW2 (batch-reduced fp32
    GEMM), the 4C-wide data gradient with GELU' and the d_s / d_b1 row sums in its epilogue, dW1 and
    dm. Same arithmetic and bf16 roundings as the unfused Functions above."""

    @staticmethod
    def forward(ctx, m, w1, dcoef, b1, w2, b2, gamma, x_in, slot=None):
        _edges(ctx, m, w1, dcoef, b1, w2, b2, gamma, x_in, slot)
        ctx.slot = slot
        m, x_in = _c(m), _c(x_in)
        B, C, P = m.shape
        w1c = _cast_cached(w1, torch.bfloat16).contiguous()
        w2c = _cast_cached(w2, torch.bfloat16).contiguous()
        s = None if dcoef is None else dcoef.detach().float().contiguous()
        fb1, fb2, fg = _f32(b1), _f32(b2), _f32(gamma)
        h, g = gemm_gelu_fwd(w1c, m, s, fb1, want_h=True)
        y = _g8(w2c, g)
        out = torch.empty_like(x_in)
        with kernel_timer.region(_rn('layer_scale_residual_fwd', y), _nb(y, x_in, out)):
            _check(_lib.vfm_layer_scale_residual_fwd(y.data_ptr(), _p(fb2), _p(fg), x_in.data_ptr(), out.data_ptr(),
                                                     _code(y), _code(x_in), B, C, P, _stream()),
                   'vfm_layer_scale_residual_fwd')
        ctx.save_for_backward(m, h, g, y, w1c, w2c, s, fb1, fb2, fg)
        ctx.meta = (w1.dtype, w2.dtype, None if dcoef is None else dcoef.dtype, None if b1 is None else b1.dtype,
                    None if b2 is None else b2.dtype, None if gamma is None else gamma.dtype)
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dout):
        m, h, g, y, w1c, w2c, s, fb1, fb2, fg = ctx.saved_tensors
        w1dt, w2dt, sdt, b1dt, b2dt, gdt = ctx.meta
        B, C, P = m.shape
        dout = _c(dout.to(torch.bfloat16))
        dy = torch.empty_like(y)
        r0 = torch.empty([B * C], dtype=torch.float32, device=m.device)
        r1 = torch.empty_like(r0)
        with kernel_timer.region(_rn('layer_scale_residual_bwd', y), _nb(y, dout, dy)):
            _check(_lib.vfm_layer_scale_residual_bwd(y.data_ptr(), _p(fb2), _p(fg), dout.data_ptr(), dy.data_ptr(),
                                                     r0.data_ptr(), r1.data_ptr(), _code(y), _code(dout), B, C, P,
                                                     _stream()), 'vfm_layer_scale_residual_bwd')
        dw1 = db1 = ds = dw2 = db2 = dgm = dm = None
        if fb2 is not None and _wanted(ctx, 5):
            s1 = r1.view(B, C).sum(0)
            db2 = (s1 * fg if fg is not None else s1).to(b2dt)
        if fg is not None and _wanted(ctx, 6):
            dgm = r0.view(B, C).sum(0).to(gdt)
        if _wanted(ctx, 4):
            dw2 = weight_grad_1x1(dy, g, w2dt)
        if GEMM_MLP_BWD_EPI:
            dh, sum_s, sum_b = gemm_gelu_bwd(w2c.t().contiguous(), dy, h, s, fb1)
        else:
            # dg = W2^T dy on the plain GEMM, then the HBM-bound GELU' row kernel: the GELU' epilogue's VALU
            # work (erf GELU + derivative per element) does not overlap the MFMAs at one wave per SIMD and
            # measured slower than this pass (profiles/r5_j_benchshape.txt: 17.6 ms/step vs ~3 + 7 ms/step)
            dg = _g8(_wt(w2c), dy)
            dh = torch.empty_like(h)
            O = h.shape[1]
            ds_rows = torch.empty([B * O], dtype=torch.float32, device=h.device) if s is not None else None
            db_rows = torch.empty([B * O], dtype=torch.float32, device=h.device)
            with kernel_timer.region(_rn('scale_bias_gelu_bwd', h), _nb(h, dg, dh)):
                _check(_lib.vfm_scale_bias_gelu_bwd(h.data_ptr(), dg.data_ptr(), _p(s), _p(fb1), dh.data_ptr(),
                                                    _p(ds_rows), db_rows.data_ptr(), _code(h), B, O, P, _stream()),
                       'vfm_scale_bias_gelu_bwd')
            sum_s = ds_rows.view(B, O) if s is not None else None
            sum_b = db_rows.view(B, O).sum(0)
        if s is not None and _wanted(ctx, 2):
            ds = sum_s.to(sdt)
        if fb1 is not None and _wanted(ctx, 3):
            db1 = sum_b.to(b1dt)
        if _wanted(ctx, 1):
            dw1 = weight_grad_1x1(dh, m, w1dt)
        if ctx.needs_input_grad[0]:
            dm = _g8(_wt(w1c), dh)
        dx = dout if ctx.needs_input_grad[7] and not _stash_residual(ctx.slot, dout) else None
        return dm, dw1, ds, db1, dw2, db2, dgm, dx, None


def _mlp_gemm_nograd(m, w1, dcoef, b1, w2, b2, gamma, x_in):
    B, C, P = m.shape
    w1c = _cast_cached(w1, torch.bfloat16).contiguous()
    w2c = _cast_cached(w2, torch.bfloat16).contiguous()
    s = None if dcoef is None else dcoef.detach().float().contiguous()
    _, g = gemm_gelu_fwd(w1c, m, s, _f32(b1), want_h=False)
    y = _g8(w2c, g)
    out = torch.empty_like(x_in)
    with kernel_timer.region(_rn('layer_scale_residual_fwd', y), _nb(y, x_in, out)):
        _check(_lib.vfm_layer_scale_residual_fwd(y.data_ptr(), _p(_f32(b2)), _p(_f32(gamma)), x_in.data_ptr(),
                                                 out.data_ptr(), _code(y), _code(x_in), B, C, P, _stream()),
               'vfm_layer_scale_residual_fwd')
    return out


class _ConvNeXtMLP(custom_ops.FastFunction):
    """pointwise(W1) -> GELU(h*s+b1) -> pointwise(W2) -> x_in + gamma*(y+b2) with autograd.
    Forward: one kernel that also writes h, g and y for the backward. Backward: the layer-
    scale residual kernel, then the 4C->C conv's data gradient with GELU' fused into its
    epilogue (vfm_pw_gemm_gelu mode 1), and hipBLASLt GEMMs for the two weight gradients
    and dm; the same arithmetic as the unfused Functions above (bf16 roundings included)."""

    @staticmethod
    def forward(ctx, m, w1, dcoef, b1, w2, b2, gamma, x_in, slot=None):
        _edges(ctx, m, w1, dcoef, b1, w2, b2, gamma, x_in, slot)
        ctx.slot = slot
        m, x_in = _c(m), _c(x_in)
        B, C, P = m.shape
        w1c = _cast_cached(w1, torch.bfloat16).contiguous()
        w2c = _cast_cached(w2, torch.bfloat16).contiguous()
        s = None if dcoef is None else dcoef.detach().float().contiguous()
        fb1, fb2, fg = _f32(b1), _f32(b2), _f32(gamma)
        out = torch.empty_like(x_in)
        h = torch.empty([B, 4 * C, P], dtype=torch.bfloat16, device=m.device)
        g = torch.empty_like(h)
        y = torch.empty_like(m)
        with kernel_timer.region(_rn('convnext_mlp_fwd', m, C, 'true'), _nb(m, x_in, out, h, g, y)):
            _check(_lib.vfm_convnext_mlp_fwd(w1c.data_ptr(), m.data_ptr(), _p(s), _p(fb1), w2c.data_ptr(), _p(fb2),
                                             _p(fg), x_in.data_ptr(), out.data_ptr(), h.data_ptr(), g.data_ptr(),
                                             y.data_ptr(), B, C, P, _stream()), 'vfm_convnext_mlp_fwd')
        ctx.save_for_backward(m, h, g, y, w1c, w2c, s, fb1, fb2, fg)
        ctx.meta = (w1.dtype, w2.dtype, None if dcoef is None else dcoef.dtype, None if b1 is None else b1.dtype,
                    None if b2 is None else b2.dtype, None if gamma is None else gamma.dtype)
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dout):
        m, h, g, y, w1c, w2c, s, fb1, fb2, fg = ctx.saved_tensors
        w1dt, w2dt, sdt, b1dt, b2dt, gdt = ctx.meta
        B, C, P = m.shape
        O = 4 * C
        dout = _c(dout.to(torch.bfloat16))
        # layer-scale residual: dy = gamma * dout, sums for d_b2 / d_gamma
        dy = torch.empty_like(y)
        r0 = torch.empty([B * C], dtype=torch.float32, device=m.device)
        r1 = torch.empty_like(r0)
        with kernel_timer.region(_rn('layer_scale_residual_bwd', y), _nb(y, dout, dy)):
            _check(_lib.vfm_layer_scale_residual_bwd(y.data_ptr(), _p(fb2), _p(fg), dout.data_ptr(), dy.data_ptr(),
                                                     r0.data_ptr(), r1.data_ptr(), _code(y), _code(dout), B, C, P,
                                                     _stream()), 'vfm_layer_scale_residual_bwd')
        dw1 = db1 = ds = dw2 = db2 = dgm = dm = None
        if fb2 is not None and _wanted(ctx, 5):
            s1 = r1.view(B, C).sum(0)
            db2 = (s1 * fg if fg is not None else s1).to(b2dt)
        if fg is not None and _wanted(ctx, 6):
            dgm = r0.view(B, C).sum(0).to(gdt)
        # dh = (W2^T dy) * GELU'(h*s+b1) * s, with the per-(b, o) sums for d_s and d_b1 (next to dW2 on
        # the side stream, _overlapped)
        tiles = _lib.vfm_pw_gemm_gelu_tiles(P)
        w2t = _wt(w2c, contiguous=True)         # vfm_pw_gemm_gelu reads W2^T as a row-major [C][O] array

        def dh_kernel():
            dh = torch.empty_like(h)
            p0 = torch.empty([B, tiles, O], dtype=torch.float32, device=m.device)
            p1 = torch.empty_like(p0)
            with kernel_timer.region(_rn('pw_gemm_gelu_bwd', h), _nb(dy, h, dh)):
                _check(_lib.vfm_pw_gemm_gelu(w2t.data_ptr(), dy.data_ptr(), _p(s), _p(fb1), h.data_ptr(),
                                             dh.data_ptr(), None, p0.data_ptr(), p1.data_ptr(), 1, B, O, C, P,
                                             _stream()), 'vfm_pw_gemm_gelu')
            return dh, p0, p1
        if _wanted(ctx, 4):
            dw2, (dh, p0, p1) = _overlapped(lambda: weight_grad_1x1(dy, g, w2dt), dh_kernel, dy.device)
        else:
            dh, p0, p1 = dh_kernel()
        if s is not None and _wanted(ctx, 2):
            ds = p0.sum(1).to(sdt)
        if fb1 is not None and _wanted(ctx, 3):
            db1 = p1.sum((0, 1)).to(b1dt)

        def dm_gemm():
            dm = _gemm(_wt(w1c), dh)
            if dm is None:
                with kernel_timer.vendor_gemm(f"{_tn(dh)},1x1_dx", C, dh.shape[2], O, B, dh.element_size()):
                    dm = torch.bmm(w1c.t().expand(B, C, O), dh)
            return dm
        want_w1, want_m = _wanted(ctx, 1), ctx.needs_input_grad[0]
        if want_w1 and want_m:
            dw1, dm = _overlapped(lambda: weight_grad_1x1(dh, m, w1dt), dm_gemm, dh.device)
        else:
            dw1 = weight_grad_1x1(dh, m, w1dt) if want_w1 else None
            dm = dm_gemm() if want_m else None
        dx = dout if ctx.needs_input_grad[7] and not _stash_residual(ctx.slot, dout) else None
        return dm, dw1, ds, db1, dw2, db2, dgm, dx, None


def convnext_mlp(m, w1, dcoef, b1, w2, b2, gamma, x_in, slot=None):
    """Autograd form of the fused MLP (same arguments as convnext_mlp_nograd): the whole-MLP kernel
    at C in MLP_CHANNELS, else the GELU-epilogue GEMM form."""
    if m.shape[1] not in MLP_CHANNELS:
        return _ConvNeXtMLPGemm.apply(m, w1, dcoef, b1, w2, b2, gamma, x_in, slot)
    return _ConvNeXtMLP.apply(m, w1, dcoef, b1, w2, b2, gamma, x_in, slot)


def convnext_mlp_nograd(m, w1, dcoef, b1, w2, b2, gamma, x_in):
    """m, x_in: bf16 [B, C, P]; w1 [4C, C], w2 [C, 4C] (any float dtype, cast to bf16);
    dcoef [B, 4C] fp32 or None; b1 [4C], b2, gamma [C] or None. Returns bf16 [B, C, P]."""
    m, x_in = _c(m), _c(x_in)
    B, C, P = m.shape
    if C not in MLP_CHANNELS:
        return _mlp_gemm_nograd(m, w1, dcoef, b1, w2, b2, gamma, x_in)
    w1c = _cast_cached(w1, torch.bfloat16).contiguous()
    w2c = _cast_cached(w2, torch.bfloat16).contiguous()
    s = None if dcoef is None else dcoef.detach().float().contiguous()
    out = torch.empty_like(x_in)
    with kernel_timer.region(_rn('convnext_mlp_fwd', m, C, 'false'), _nb(m, x_in, out), flops=4.0 * B * P * C * 4 * C,
                             bound="hbm"):
        _check(_lib.vfm_convnext_mlp_fwd(w1c.data_ptr(), m.data_ptr(), _p(s), _p(_f32(b1)), w2c.data_ptr(),
                                         _p(_f32(b2)), _p(_f32(gamma)), x_in.data_ptr(), out.data_ptr(), None, None, None, B, C, P,
                                         _stream()), 'vfm_convnext_mlp_fwd')
    return out


# ---------------------------------------------------------------------------
# PixelShuffle + replicate pad + fixed blur (reference convnext_utils.py:234-257).


def _taps(blur1d):
    k = [float(t) for t in blur1d]
    s = sum(k)
    k = [t / s for t in k]
    return (ctypes.c_float * 8)(*(k + [0.0] * (8 - len(k)))), len(k)


class _ShuffleBlur(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, x, blur1d, r):
        x = _c(x)
        B, Cr, H, W = x.shape
        C = Cr // (r * r)
        taps, K = _taps(blur1d)
        y = torch.empty([B, C, H * r, W * r], dtype=x.dtype, device=x.device)
        with kernel_timer.region(_rn('shuffle_blur_fwd', x, K), _nb(x, y)):
            _check(_lib.vfm_shuffle_blur_fwd(x.data_ptr(), y.data_ptr(), taps, K, _code(x), B, C, H, W, r, _stream()),
                   'vfm_shuffle_blur_fwd')
        ctx.cfg = (tuple(blur1d), r, (B, C, H, W))
        return y

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dy):
        blur1d, r, (B, C, H, W) = ctx.cfg
        dy = _c(dy)
        taps, K = _taps(blur1d)
        dx = torch.empty([B, C * r * r, H, W], dtype=dy.dtype, device=dy.device)
        with kernel_timer.region(_rn('shuffle_blur_bwd', dy, K), _nb(dy, dx)):
            _check(_lib.vfm_shuffle_blur_bwd(dy.data_ptr(), dx.data_ptr(), taps, K, _code(dy), B, C, H, W, r,
                                             _stream()), 'vfm_shuffle_blur_bwd')
        return dx, None, None


def shuffle_blur(x, blur1d, upscale):
    return _ShuffleBlur.apply(x, tuple(blur1d), int(upscale))


def blur_replicate(x, blur1d):
    return _ShuffleBlur.apply(x, tuple(blur1d), 1)


# ---------------------------------------------------------------------------
# ToRGB: modulated 1x1 to O <= 4 channels + bias (reference convnext_utils.py:145-187), one
# HBM pass per direction (csrc/torgb.hip); dstyle / dweight / dbias from the kernel's [B, O, C]
# partials on the host side (tiny).


class _ToRGB(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, x, w2, style, bias):
        _edges(ctx, x, w2, style, bias)
        B, C, H, W = x.shape
        O, P = w2.shape[0], H * W
        x = _c(x)
        s32, w32 = style.detach().float(), w2.detach().float()
        wm = (w32[None] * s32[:, None, :]).contiguous()                      # [B, O, C]
        b32 = bias.detach().reshape(-1).float().contiguous()
        y = torch.empty([B, O, H, W], dtype=torch.float32, device=x.device)
        with kernel_timer.region(_rn('torgb_fwd', x), _nb(x, y)):
            _check(_lib.vfm_torgb_fwd(x.data_ptr(), wm.data_ptr(), b32.data_ptr(), y.data_ptr(), _code(x), B, O, C, P,
                                      _stream()), 'vfm_torgb_fwd')
        ctx.save_for_backward(x, wm, s32, w32)
        ctx.meta = (w2.dtype, style.dtype, bias.dtype, bias.shape)
        return y

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dy):
        x, wm, s32, w32 = ctx.saved_tensors
        wdt, sdt, bdt, bshape = ctx.meta
        B, C, H, W = x.shape
        O, P = wm.shape[1], H * W
        dy = _c(dy.float())
        dx = dw = ds = db = None
        S = _lib.vfm_torgb_bwd_splits(B, C, P)
        dxt = torch.empty_like(x)
        tpart = torch.empty([B, S, O, C], dtype=torch.float32, device=x.device)
        with kernel_timer.region(_rn('torgb_bwd', x), _nb(x, dy, dxt)):
            _check(_lib.vfm_torgb_bwd(x.data_ptr(), dy.data_ptr(), wm.data_ptr(), dxt.data_ptr(), tpart.data_ptr(),
                                      _code(x), B, O, C, P, S, _stream()), 'vfm_torgb_bwd')
        T = tpart.sum(1)                                                        # [B, O, C]
        if _wanted(ctx, 0):
            dx = dxt
        if _wanted(ctx, 1):
            dw = (T * s32[:, None, :]).sum(0).to(wdt)
        if _wanted(ctx, 2):
            ds = (T * w32[None]).sum(1).to(sdt)
        if _wanted(ctx, 3):
            db = dy.sum((0, 2, 3)).reshape(bshape).to(bdt)
        return dx, dw, ds, db


def torgb_supported(x, O):
    B, C, H, W = x.shape
    return x.dtype in (torch.float32, torch.bfloat16) and 1 <= O <= 4 and (H * W) % 8 == 0 and C % 16 == 0


def torgb(x, w2, style, bias):
    """y = (w2 @ (style * x)) + bias in fp32: x [B, C, H, W], w2 [O, C], style [B, C], bias [1, O, 1, 1]."""
    return _ToRGB.apply(x, w2, style, bias)


# ---------------------------------------------------------------------------
# Channel RMS norm of the decoder attention blocks (csrc/rmsnorm.hip; reference
# networks/utils/gigagan_utils.py:31-39): one launch forward, one (+ the gamma row sum) backward.


class _ChannelRMSNorm(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, x, gamma, scale):
        _edges(ctx, x, gamma, scale)
        x = _c(x)
        B, C = x.shape[:2]
        P = x[0, 0].numel()
        g = _f32(gamma)
        y = torch.empty_like(x)
        rinv = torch.empty([B, P], dtype=torch.float32, device=x.device)
        with kernel_timer.region(_rn('channel_rms_norm_fwd', x), _nb(x, y)):
            _check(_lib.vfm_channel_rms_norm_fwd(x.data_ptr(), g.data_ptr(), y.data_ptr(), rinv.data_ptr(), B, C, P,
                                                 float(scale), _stream()), 'vfm_channel_rms_norm_fwd')
        ctx.save_for_backward(x, g, rinv)
        ctx.scale, ctx.gmeta = float(scale), (gamma.dtype, gamma.shape)
        return y

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dy):
        x, g, rinv = ctx.saved_tensors
        B, C = x.shape[:2]
        P = x[0, 0].numel()
        dy = _c(dy.float())
        dx = torch.empty_like(x)
        want_g = _wanted(ctx, 1)
        gpart = dg = None
        if want_g:
            gpart = torch.empty([_lib.vfm_channel_rms_norm_rows(B, C, P), C], dtype=torch.float32, device=x.device)
            dg = torch.empty([C], dtype=torch.float32, device=x.device)
        with kernel_timer.region(_rn('channel_rms_norm_bwd', x), _nb(x, dy, dx)):
            _check(_lib.vfm_channel_rms_norm_bwd(x.data_ptr(), g.data_ptr(), rinv.data_ptr(), dy.data_ptr(),
                                                 dx.data_ptr(), _p(gpart), _p(dg), B, C, P, ctx.scale, _stream()),
                   'vfm_channel_rms_norm_bwd')
        gdt, gshape = ctx.gmeta
        return (dx if ctx.needs_input_grad[0] else None), (dg.reshape(gshape).to(gdt) if want_g else None), None


def channel_rms_norm_supported(x):
    return x.is_cuda and x.dtype == torch.float32 and x.dim() >= 3 and x.numel() > 0


def channel_rms_norm(x, gamma, scale):
    """F.normalize(x, dim=1) * scale * gamma for fp32 [B, C, ...] (gamma [C] / [C, 1, 1])."""
    return _ChannelRMSNorm.apply(x, gamma, scale)


# ---------------------------------------------------------------------------
# Style affine + demodulation of a ConvNeXt synthesis layer (csrc/style.hip; reference
# networks/utils/shared.py StyleSplit / FullyConnectedLayer, convnext_utils.py:60-66):
# two launches forward, two backward, instead of ~9 / ~25 torch kernels per layer.


class _StyleDemod(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, w, A, ab, W1, wg, bg, eps):
        _edges(ctx, w, A, ab, W1, wg, bg, eps)
        wv = w.detach()
        if wv.dtype != torch.float32 or wv.stride(1) != 1 or wv.data_ptr() % 16:
            wv = wv.float().contiguous()
        B, WD = wv.shape
        C = A.shape[0] // 3
        A32, ab32 = _f32(A).reshape(3 * C, WD), _f32(ab)
        W132 = None if W1 is None else _f32(W1).reshape(W1.shape[0], C)
        O = 0 if W1 is None else W132.shape[0]
        dev = w.device
        m = torch.empty([B, 3 * C], dtype=torch.float32, device=dev)
        s = torch.empty([B, C], dtype=torch.float32, device=dev)
        d = torch.empty([B, O], dtype=torch.float32, device=dev) if W1 is not None else None
        with kernel_timer.region('style_demod_fwd<f32>', _nb(wv, A32, W132, m, s, d)):
            _check(_lib.vfm_style_demod_fwd(wv.data_ptr(), wv.stride(0), A32.data_ptr(), ab32.data_ptr(), _p(W132),
                                            float(wg), float(bg), float(eps), B, C, WD, O, m.data_ptr(), s.data_ptr(),
                                            _p(d), _stream()), 'vfm_style_demod_fwd')
        ctx.save_for_backward(wv, A32, W132, m, s, d)
        ctx.meta = (float(wg), float(bg), w.dtype, A.dtype, ab.dtype, None if W1 is None else W1.dtype)
        if d is None:
            return s
        return s, d

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, ds_in, dd=None):
        wv, A32, W132, m, s, d = ctx.saved_tensors
        wg, bg, wdt, adt, abdt, w1dt = ctx.meta
        B, WD = wv.shape
        C = s.shape[1]
        O = 0 if d is None else d.shape[1]
        dev = wv.device
        want_w, want_A, want_ab = _wanted(ctx, 0), _wanted(ctx, 1), _wanted(ctx, 2)
        want_W1 = d is not None and _wanted(ctx, 3)
        f32 = dict(dtype=torch.float32, device=dev)
        ds_in = _c(ds_in.float()) if ds_in is not None else torch.zeros([B, C], **f32)
        if d is not None:
            dd = _c(dd.float()) if dd is not None else torch.zeros([B, O], **f32)
        nws = _lib.vfm_style_demod_bwd_workspace_floats(B, C, WD, O)
        if nws < 0:
            raise custom_ops.NativeError(f"vfm_style_demod_bwd: workspace for B={B} C={C} WD={WD} O={O} exceeds 2^31 floats")
        ds_ws = torch.empty([max(1, nws)], **f32)
        dW1 = torch.empty([O, C], **f32) if want_W1 else None
        dA = torch.empty([3 * C, WD], **f32) if want_A else None
        dab = torch.empty([3 * C], **f32) if want_ab else None
        dw = torch.empty([B, WD], **f32) if want_w else None
        with kernel_timer.region('style_demod_bwd<f32>', _nb(wv, A32, W132, m, s, d, dW1, dA, dw)):
            _check(_lib.vfm_style_demod_bwd(wv.data_ptr(), wv.stride(0), A32.data_ptr(), _p(W132), m.data_ptr(),
                                            s.data_ptr(), _p(d), ds_in.data_ptr(), _p(dd if d is not None else None),
                                            wg, bg, B, C, WD, O, _p(ds_ws), _p(dW1), _p(dA), _p(dab), _p(dw),
                                            _stream()), 'vfm_style_demod_bwd')
        return (None if dw is None else dw.to(wdt), None if dA is None else dA.to(adt),
                None if dab is None else dab.to(abdt), None if dW1 is None else dW1.to(w1dt), None, None, None)


def style_demod(w, A, ab, W1, wg, bg, eps):
    """(s [B, C], d [B, O] or None): s = StyleSplit(FullyConnectedLayer(A, ab, gains wg / bg))(w),
    d = rsqrt(s^2 @ (W1^2)^T + eps) when W1 [O, C] is given. fp32."""
    out = _StyleDemod.apply(w, A, ab, W1, wg, bg, eps)
    return (out, None) if W1 is None else out
