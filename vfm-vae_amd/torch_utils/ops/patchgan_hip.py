"""Multi-scale PatchGAN discriminator on the gfx950 kernels (stage 3; reference
networks/discriminator.py:75-99 BatchNormLocal2d, :180-228 NLayerDiscriminator).

Activations are NHWC fp32 (channels_last views of the reference's NCHW tensors). A k4 conv is
im2col (csrc/patchgan.hip) + our MFMA GEMM (gemm_hip, fp32-equivalent f32x6 products) with the
bias fused into the GEMM epilogue; its weight gradient is the same GEMM (split-K over the pixels) and
its data gradient a GEMM followed by the col2im gather. The 1-channel logit layer uses a row dot /
column dot instead of a 1-wide GEMM. BatchNormLocal2d + LeakyReLU(0.2) run as one fused forward and
one fused backward (virtual-batch statistics, deterministic partial sums). Layer 0's bias + LeakyReLU
is the HIP bias_act kernel.

Only reached for ROCm fp32 tensors (`supported`); a missing kernel library raises.
"""
import os

import torch

from .. import custom_ops
from . import kernel_timer

_lib = custom_ops.get_native()


def _stream():
    return custom_ops.stream_ptr()


def _check(rc, name):
    custom_ops.check(rc, name)


def _c16(t):
    t = t.contiguous()
    return t if t.data_ptr() % 16 == 0 else t.clone()


def _gemm(A, B, **kw):
    from . import gemm_hip
    return gemm_hip.gemm(A, B, out_dtype=torch.float32, **kw)


def _gemm_or_mm(A, B, bias=None, **kw):
    """fp32 A @ B (+ bias[:, None]) for the D heads' 1-D convs: the exact-fp32 MFMA GEMM (csrc/sgemm.hip, the
    default: the reference's precision with TF32 off, no operand split), VFM_DHEAD_GEMM=hip our f32x6 GEMM,
    VFM_DHEAD_GEMM=torch hipBLASLt's exact fp32 (A/B); a layout neither kernel takes falls back to the library
    product, timed as a vendor region."""
    from . import gemm_hip
    if _DHEAD == "sgemm":
        out = gemm_hip.sgemm(A, B, bias=bias, bias_dim=None if bias is None else 0)
        if out is not None:
            return out
    elif _DHEAD == "hip":
        out = gemm_hip.try_gemm(A, B, out_dtype=torch.float32, bias=bias, bias_dim=None if bias is None else 0, **kw)
        if out is not None:
            return out
    with kernel_timer.vendor_gemm("f32,dhead", A.shape[0], B.shape[1], A.shape[1], esize=4):
        return torch.mm(A, B) if bias is None else torch.addmm(bias[:, None], A, B)


def _splits(M, N, K):
    tiles = -(-M // 128) * -(-N // 128)
    return max(1, min(-(-1024 // tiles), K // 512, 64))


def _im2col(xh, k, stride, pad, Ho, Wo):
    B, H, W, C = xh.shape
    K = k * k * C
    A = torch.empty([B * Ho * Wo, K], dtype=torch.float32, device=xh.device)
    with kernel_timer.region("im2col_nhwc<f32>", 4 * (xh.numel() + A.numel())):
        _check(_lib.vfm_im2col_nhwc_f32(xh.data_ptr(), A.data_ptr(), K, B, H, W, C, Ho, Wo, k, stride, pad, _stream()),
               "vfm_im2col_nhwc_f32")
    return A


class _ConvNHWC(custom_ops.FastFunction):
    """y[b, oy, ox, o] = sum_{ky, kx, c} x[b, s oy - p + ky, s ox - p + kx, c] w[o, c, ky, kx] (+ bias[o])."""

    @staticmethod
    def forward(ctx, xh, weight, bias, stride, pad):
        B, H, W, C = xh.shape
        O, _, k, _ = weight.shape
        Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
        xh = _c16(xh)
        A = _im2col(xh, k, stride, pad, Ho, Wo)
        Wm = weight.detach().permute(0, 2, 3, 1).reshape(O, k * k * C).float().contiguous()   # [O, K] tap-major
        b32 = None if bias is None else bias.detach().float().contiguous()
        M = B * Ho * Wo
        if O == 1:
            y = torch.empty([M], dtype=torch.float32, device=xh.device)
            with kernel_timer.region("rowdot<f32>", 4 * (A.numel() + M), flops=2.0 * A.numel(), bound="hbm"):
                _check(_lib.vfm_rowdot_f32(A.data_ptr(), A.shape[1], Wm.data_ptr(), custom_ops.ptr(b32), y.data_ptr(),
                                           M, A.shape[1], _stream()), "vfm_rowdot_f32")
        else:
            y = _gemm(A, Wm.t(), bias=b32, bias_dim=1)
        ctx.save_for_backward(A, Wm)
        ctx.geo = (B, H, W, C, Ho, Wo, k, stride, pad, O)
        ctx.meta = (weight.dtype, None if bias is None else bias.dtype)
        ctx.needs = (ctx.needs_input_grad[0], ctx.needs_input_grad[1], bias is not None and ctx.needs_input_grad[2])
        return y.reshape(B, Ho, Wo, O)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dy):
        A, Wm = ctx.saved_tensors
        B, H, W, C, Ho, Wo, k, stride, pad, O = ctx.geo
        wdt, bdt = ctx.meta
        nx, nw, nb = ctx.needs
        M, K = A.shape
        dy = _c16(dy.float().reshape(M, O))
        dx = dw = db = None
        if nb:
            db = dy.sum(0).to(bdt)
        if nw:
            if O == 1:
                S = _lib.vfm_coldot_splits(M, K)
                part = torch.empty([S, K], dtype=torch.float32, device=dy.device)
                with kernel_timer.region("coldot<f32>", 4 * (A.numel() + M + part.numel()), flops=2.0 * A.numel()):
                    _check(_lib.vfm_coldot_f32(A.data_ptr(), K, dy.data_ptr(), part.data_ptr(), M, K, S, _stream()),
                           "vfm_coldot_f32")
                dWm = part.sum(0, keepdim=True)
            else:
                dWm = _gemm(dy.t(), A, splits=_splits(O, K, M))
            dw = dWm.reshape(O, k, k, C).permute(0, 3, 1, 2).contiguous().to(wdt)
        if nx:
            dX = torch.empty([B, H, W, C], dtype=torch.float32, device=dy.device)
            if O == 1:
                dA, dy1, w1 = None, dy, Wm
            else:
                dA, dy1, w1 = _gemm(dy, Wm), None, None
            with kernel_timer.region("col2im_nhwc<f32>", 4 * (dX.numel() + (dA.numel() if dA is not None else M))):
                _check(_lib.vfm_col2im_nhwc_f32(custom_ops.ptr(dA), K, custom_ops.ptr(dy1), custom_ops.ptr(w1),
                                                dX.data_ptr(), B, H, W, C, Ho, Wo, k, stride, pad, _stream()),
                       "vfm_col2im_nhwc_f32")
            dx = dX
        return dx, dw, db, None, None


class _BnLocalLReLU(custom_ops.FastFunction):
    """lrelu(BatchNormLocal2d(x)) over NHWC x [B, H, W, C], G virtual batches."""

    @staticmethod
    def forward(ctx, xh, weight, bias, G, eps, slope):
        B, H, W, C = xh.shape
        P = H * W
        xh = _c16(xh)
        w32 = None if weight is None else weight.detach().float().contiguous()
        b32 = None if bias is None else bias.detach().float().contiguous()
        n = _lib.vfm_bnl_workspace_floats(B, P, C, G)
        ws = torch.empty([n], dtype=torch.float32, device=xh.device)
        mean = torch.empty([G, C], dtype=torch.float32, device=xh.device)
        rstd = torch.empty_like(mean)
        y = torch.empty_like(xh)
        with kernel_timer.region("bnl_lrelu_fwd<f32>", 4 * 4 * xh.numel()):
            _check(_lib.vfm_bnl_lrelu_fwd(xh.data_ptr(), custom_ops.ptr(w32), custom_ops.ptr(b32), y.data_ptr(),
                                          mean.data_ptr(), rstd.data_ptr(), ws.data_ptr(), B, P, C, G, float(eps),
                                          float(slope), _stream()), "vfm_bnl_lrelu_fwd")
        ctx.save_for_backward(xh, w32, b32, mean, rstd)
        ctx.cfg = (G, slope, None if weight is None else weight.dtype, None if bias is None else bias.dtype)
        return y

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dy):
        xh, w32, b32, mean, rstd = ctx.saved_tensors
        G, slope, wdt, bdt = ctx.cfg
        B, H, W, C = xh.shape
        P = H * W
        dy = _c16(dy.float())
        n = _lib.vfm_bnl_workspace_floats(B, P, C, G)
        ws = torch.empty([n], dtype=torch.float32, device=xh.device)
        dx = torch.empty_like(xh)
        dw = torch.empty([C], dtype=torch.float32, device=xh.device) if w32 is not None else None
        db = torch.empty([C], dtype=torch.float32, device=xh.device) if b32 is not None else None
        with kernel_timer.region("bnl_lrelu_bwd<f32>", 4 * 4 * xh.numel()):
            _check(_lib.vfm_bnl_lrelu_bwd(xh.data_ptr(), dy.data_ptr(), custom_ops.ptr(w32), custom_ops.ptr(b32),
                                          mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(), custom_ops.ptr(dw),
                                          custom_ops.ptr(db), ws.data_ptr(), B, P, C, G, float(slope), _stream()),
                   "vfm_bnl_lrelu_bwd")
        return (dx, None if dw is None else dw.to(wdt), None if db is None else db.to(bdt), None, None, None)


class _BnLocal1dLReLU(custom_ops.FastFunction):
    """lrelu(BatchNormLocal(x)) over [B, C, L] fp32, G virtual batches (the D heads' blocks)."""

    @staticmethod
    def forward(ctx, x, weight, bias, G, eps, slope):
        B, C, L = x.shape
        x = x.contiguous()
        w32 = None if weight is None else weight.detach().float().contiguous()
        b32 = None if bias is None else bias.detach().float().contiguous()
        mean = torch.empty([G, C], dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        y = torch.empty_like(x)
        with kernel_timer.region("bnl1d_lrelu_fwd<f32>", 4 * 3 * x.numel()):
            _check(_lib.vfm_bnl1d_lrelu_fwd(x.data_ptr(), custom_ops.ptr(w32), custom_ops.ptr(b32), y.data_ptr(),
                                            mean.data_ptr(), rstd.data_ptr(), B, C, L, G, float(eps), float(slope),
                                            _stream()), "vfm_bnl1d_lrelu_fwd")
        ctx.save_for_backward(x, w32, b32, mean, rstd)
        ctx.cfg = (G, slope, None if weight is None else weight.dtype, None if bias is None else bias.dtype)
        return y

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dy):
        x, w32, b32, mean, rstd = ctx.saved_tensors
        G, slope, wdt, bdt = ctx.cfg
        B, C, L = x.shape
        dy = dy.float().contiguous()
        dx = torch.empty_like(x)
        part = torch.empty([2, G, C], dtype=torch.float32, device=x.device)
        with kernel_timer.region("bnl1d_lrelu_bwd<f32>", 4 * 4 * x.numel()):
            _check(_lib.vfm_bnl1d_lrelu_bwd(x.data_ptr(), dy.data_ptr(), custom_ops.ptr(w32), custom_ops.ptr(b32),
                                            mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(), part.data_ptr(), B, C, L,
                                            G, float(slope), _stream()), "vfm_bnl1d_lrelu_bwd")
        dw = None if w32 is None else part[0].sum(0).to(wdt)
        db = None if b32 is None else part[1].sum(0).to(bdt)
        return dx, dw, db, None, None, None


def bn_local1d_lrelu(x, weight, bias, groups, eps, slope):
    return _BnLocal1dLReLU.apply(x, weight, bias, int(groups), float(eps), float(slope))


def supported(x):
    return x.is_cuda and x.dtype == torch.float32 and x.dim() == 4


def conv_nhwc(xh, weight, bias, stride, pad):
    return _ConvNHWC.apply(xh, weight, bias, int(stride), int(pad))


def bn_local_lrelu(xh, weight, bias, groups, eps, slope):
    return _BnLocalLReLU.apply(xh, weight, bias, int(groups), float(eps), float(slope))


def bias_lrelu(yh, bias, slope):
    """lrelu(y + bias[c]) over NHWC y (HIP bias_act, gain 1)."""
    from . import bias_act
    C = yh.shape[-1]
    y2 = bias_act.bias_act(yh.reshape(-1, C), bias, dim=1, act='lrelu', alpha=slope, gain=1.0)
    return y2.reshape(yh.shape)


# ---------------------------------------------------------------------------
# Spectral normalisation of the D heads' SpectralConv1d weights in training mode (csrc/specnorm.hip;
# torch.nn.utils.spectral_norm with one power iteration, dim 0): three launches forward, two backward.


class _SpectralNormWeight(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, weight, u, v, eps):
        O = weight.shape[0]
        W = weight.detach().reshape(O, -1)
        if W.dtype != torch.float32 or not W.is_contiguous():
            raise custom_ops.NativeError("spectral_norm_weight: fp32 contiguous weight expected")
        I = W.shape[1]
        dev = W.device
        ws = torch.empty([_lib.vfm_specnorm_workspace_floats(O, I)], dtype=torch.float32, device=dev)
        uc = torch.empty([O], dtype=torch.float32, device=dev)
        vc = torch.empty([I], dtype=torch.float32, device=dev)
        sigma = torch.empty([1], dtype=torch.float32, device=dev)
        wsn = torch.empty_like(weight)
        with kernel_timer.region('specnorm_fwd<f32>', 4 * (2 * O * I + O + I)):
            _check(_lib.vfm_specnorm_fwd(W.data_ptr(), u.data_ptr(), v.data_ptr(), uc.data_ptr(), vc.data_ptr(),
                                         sigma.data_ptr(), wsn.data_ptr(), ws.data_ptr(), O, I, float(eps), _stream()),
                   'vfm_specnorm_fwd')
        ctx.save_for_backward(W, uc, vc, sigma)
        return wsn

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g):
        W, uc, vc, sigma = ctx.saved_tensors
        O, I = W.shape
        g = _c16(g.float())
        ws = torch.empty([_lib.vfm_specnorm_workspace_floats(O, I)], dtype=torch.float32, device=W.device)
        dW = torch.empty_like(W)
        with kernel_timer.region('specnorm_bwd<f32>', 4 * 3 * O * I):
            _check(_lib.vfm_specnorm_bwd(g.data_ptr(), W.data_ptr(), uc.data_ptr(), vc.data_ptr(), sigma.data_ptr(),
                                         dW.data_ptr(), ws.data_ptr(), O, I, _stream()), 'vfm_specnorm_bwd')
        return dW.reshape(g.shape), None, None, None


def spectral_norm_weight(weight, u, v, eps):
    """W / sigma(W) with one in-place power iteration on (u, v) (training-mode torch spectral_norm, dim 0)."""
    return _SpectralNormWeight.apply(weight, u, v, eps)


# ---------------------------------------------------------------------------
# im2col of the D heads' 1-D convs (csrc/im2col1d.hip): zero or circular padding, one launch each way.


class _Im2col1d(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, x, k, p, circular):
        x = _c16(x)
        B, C, L = x.shape
        Lo = L + 2 * p - k + 1
        cols = torch.empty([B, C * k, Lo], dtype=torch.float32, device=x.device)
        with kernel_timer.region('im2col1d<f32>', 4 * (x.numel() + cols.numel())):
            _check(_lib.vfm_im2col1d_f32(x.data_ptr(), cols.data_ptr(), B, C, L, k, p, int(circular), _stream()),
                   'vfm_im2col1d_f32')
        ctx.meta = (B, C, L, k, p, circular)
        return cols

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dcols):
        B, C, L, k, p, circular = ctx.meta
        dcols = _c16(dcols.float())
        dx = torch.empty([B, C, L], dtype=torch.float32, device=dcols.device)
        with kernel_timer.region('col2im1d<f32>', 4 * (dx.numel() + dcols.numel())):
            _check(_lib.vfm_col2im1d_f32(dcols.data_ptr(), dx.data_ptr(), B, C, L, k, p, int(circular), _stream()),
                   'vfm_col2im1d_f32')
        return dx, None, None, None


def im2col1d_supported(x, k, p, circular):
    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 3 and x.numel() > 0
            and (not circular or (2 * p == k - 1 and p <= x.shape[2])))


def im2col1d(x, k, p, circular):
    """[B, C, L] -> [B, C k, Lo]: F.pad(x, (p, p), circular / zeros).unfold(2, k, 1) in the GEMM layout."""
    return _Im2col1d.apply(x, int(k), int(p), bool(circular))


# ---------------------------------------------------------------------------
# The D heads' SpectralConv1d over the whole batch as single GEMMs (reference networks/discriminator.py
# :39-42, 116-142: nn.Conv1d, k = 1 or 9 with circular padding). The columns are gathered with the batch
# folded in, cols [C k, B Lo] (vfm_im2col1d_cbl_f32), so
#   forward   y [O, B Lo] = W [O, C k] cols (+ bias), one [B, O, Lo] transpose copy of the small output;
#   backward  dW = dY [O, B Lo] cols^T  (the batch inside the reduction: no per-sample [O, C k] products
#             and no batch sum), dcols = W^T dY, dx = the folded col2im; db = row sums of dY.
# The products: the exact-fp32 MFMA GEMM (csrc/sgemm.hip) by default -- the reference's precision with TF32
# off, which matters here: the heads' BatchNormLocal over virtual batches of 8 samples amplifies GEMM rounding into
# the input gradient. VFM_DHEAD_GEMM=hip puts them on our f32x6 GEMM (three exact bf16 pieces per operand, six piece
# products; measured 13.7 ms/step slower than hipBLASLt in round 5, r5o), VFM_DHEAD_GEMM=torch on hipBLASLt's exact
# fp32 (round 5's default).
_DHEAD = os.environ.get("VFM_DHEAD_GEMM", "sgemm")


class _Conv1dFolded(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, x, w2, bias, k, p, circular):
        x = _c16(x.float())
        B, C, L = x.shape
        O = w2.shape[0]
        Lo = L + 2 * p - k + 1
        cols = torch.empty([C * k, B * Lo], dtype=torch.float32, device=x.device)
        with kernel_timer.region('im2col1d_cbl<f32>', 4 * (x.numel() + cols.numel())):
            _check(_lib.vfm_im2col1d_cbl_f32(x.data_ptr(), cols.data_ptr(), B, C, L, k, p, int(circular), _stream()),
                   'vfm_im2col1d_cbl_f32')
        w = w2.detach().float()
        y2 = _gemm_or_mm(w, cols, bias=None if bias is None else bias.detach().float())
        ctx.save_for_backward(cols, w)
        ctx.meta = (B, C, L, k, p, circular, w2.dtype, None if bias is None else bias.dtype)
        return y2.view(O, B, Lo).transpose(0, 1).contiguous()

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dy):
        cols, w = ctx.saved_tensors
        B, C, L, k, p, circular, wdt, bdt = ctx.meta
        O = w.shape[0]
        gy2 = dy.float().transpose(0, 1).reshape(O, -1)                       # [O, B Lo]
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dcols = _c16(_gemm_or_mm(w.t(), gy2))
            dx = torch.empty([B, C, L], dtype=torch.float32, device=dy.device)
            with kernel_timer.region('col2im1d_cbl<f32>', 4 * (dx.numel() + dcols.numel())):
                _check(_lib.vfm_col2im1d_cbl_f32(dcols.data_ptr(), dx.data_ptr(), B, C, L, k, p, int(circular),
                                                 _stream()), 'vfm_col2im1d_cbl_f32')
        if ctx.needs_input_grad[1]:
            # deep reduction over the batch-folded columns (own GEMM: K splits fill the chip)
            dw = _gemm_or_mm(gy2, cols.t(), splits=_splits(O, cols.shape[0], gy2.shape[1])).to(wdt)
        if ctx.needs_input_grad[2]:
            db = gy2.sum(1).to(bdt)
        return dx, dw, db, None, None, None


def conv1d_folded_supported(x, k, p, circular):
    return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 3 and x.numel() > 0
            and x.shape[2] + 2 * p - k + 1 > 0 and (not circular or (2 * p == k - 1 and p <= x.shape[2])))


def conv1d_folded(x, w2, bias, k, p, circular):
    """y [B, O, Lo] = conv1d(pad(x, p, circular / zeros), W) for x [B, C, L] fp32, w2 [O, C k] (the
    Conv1d weight reshaped), stride 1, one group."""
    return _Conv1dFolded.apply(x, w2, bias, int(k), int(p), bool(circular))
