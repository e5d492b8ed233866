"""2-D convolution and transposed convolution on our kernels (csrc/im2col2d.hip + the exact-fp32 GEMM
csrc/sgemm.hip), with autograd: the convolution inside reference torch_utils/ops/conv2d_resample.py:46-141
(conv2d_gradfix.conv2d / conv_transpose2d, reference conv2d_gradfix.py:37-58) and the grouped per-sample form
generator.py:46-103 modulated_conv2d uses (x reshaped [1, B Cin, H, W], groups = B).

  conv2d            y[b, g] = W_g cols_g[b] (+ bias),   cols = im2col(x)       (one GEMM per group, batched)
    backward        dcols_g[b] = W_g^T dy_g[b] -> dx = col2im(dcols);  dW_g = sum_b dy_g[b] cols_g[b]^T
  conv_transpose2d  the adjoint of conv2d(., W) on the output geometry: cols_g[b] = W_g^T x_g[b], y = col2im(cols)
    backward        dx = conv2d(dy, W): W_g im2col(dy)_g[b];  dW_g = sum_b x_g[b] im2col(dy)_g[b]^T

Products in exact fp32 (fp16 / bf16 inputs are computed in fp32 and rounded to their dtype at the output, the
precision class of the reference's cuDNN convolution with TF32 off). Dilation 1 only; `supported` says when the
own path applies (ROCm tensors of a float dtype), else the caller takes torch's convolution. The weight
gradient honours conv2d_gradfix.no_weight_gradients() (reference conv2d_gradfix.py:22-35).
"""
import torch

from .. import custom_ops
from . import conv2d_gradfix, kernel_timer

_lib = custom_ops.get_native()


def supported(x, w, dilation=1):
    d = (dilation, dilation) if isinstance(dilation, int) else tuple(dilation)
    return (x.is_cuda and x.dim() == 4 and w.dim() == 4 and d == (1, 1) and x.numel() > 0
            and x.dtype in (torch.float32, torch.float16, torch.bfloat16))


def _pair(v):
    return (int(v), int(v)) if isinstance(v, int) else (int(v[0]), int(v[1]))


def _im2col(x, kh, kw, s, p, Ho, Wo):
    B, C, H, W = x.shape
    cols = torch.empty([B, C * kh * kw, Ho * Wo], dtype=torch.float32, device=x.device)
    with kernel_timer.region("im2col2d<f32>", 4 * (x.numel() + cols.numel())):
        custom_ops.check(_lib.vfm_im2col2d_f32(x.data_ptr(), cols.data_ptr(), B, C, H, W, kh, kw, s[0], s[1], p[0],
                                               p[1], Ho, Wo, custom_ops.stream_ptr(x.device)), "vfm_im2col2d_f32")
    return cols


def _col2im(cols, B, C, H, W, kh, kw, s, p, Ho, Wo):
    x = torch.empty([B, C, H, W], dtype=torch.float32, device=cols.device)
    with kernel_timer.region("col2im2d<f32>", 4 * (x.numel() + cols.numel())):
        custom_ops.check(_lib.vfm_col2im2d_f32(cols.contiguous().data_ptr(), x.data_ptr(), B, C, H, W, kh, kw, s[0],
                                               s[1], p[0], p[1], Ho, Wo, custom_ops.stream_ptr(cols.device)),
                         "vfm_col2im2d_f32")
    return x


def _gemm(A, B, **kw):
    from . import gemm_hip
    out = gemm_hip.sgemm(A, B, **kw)
    if out is None:
        raise custom_ops.NativeError(f"sgemm does not cover A {tuple(A.shape)} {A.stride()} B {tuple(B.shape)}")
    return out


def _grouped(wm, cols, G, out, bias=None, transpose_w=False):
    """out[b, g] = W_g (or W_g^T) @ cols[b, g] for wm [G, R, Kc] (the weight matrix per group) and cols
    [B, G, K, L]; one batched exact-fp32 product per group (or one over the groups when B == 1)."""
    Bn = cols.shape[0]
    A = wm.transpose(1, 2) if transpose_w else wm                     # [G, M, K]
    if Bn == 1 and G > 1:                        # the per-sample grouped form: one product batched over groups
        _gemm(A, cols[0], out=out[0])
        if bias is not None:
            out[0].add_(bias.view(G, -1, 1))
        return out
    for g in range(G):
        _gemm(A[g], cols[:, g], out=out[:, g], bias=None if bias is None else bias.view(G, -1)[g],
              bias_dim=None if bias is None else 0)
    return out


class _Conv2d(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, x, w, bias, stride, padding, groups):
        B, C, H, W = x.shape
        O, Cg, kh, kw = w.shape
        G = groups
        s, p = _pair(stride), _pair(padding)
        Ho, Wo = (H + 2 * p[0] - kh) // s[0] + 1, (W + 2 * p[1] - kw) // s[1] + 1
        xf = x.detach().float().contiguous()
        cols = _im2col(xf, kh, kw, s, p, Ho, Wo).view(B, G, Cg * kh * kw, Ho * Wo)
        wm = w.detach().float().reshape(G, O // G, Cg * kh * kw).contiguous()
        y = torch.empty([B, G, O // G, Ho * Wo], dtype=torch.float32, device=x.device)
        _grouped(wm, cols, G, y, bias=None if bias is None else bias.detach().float().contiguous())
        ctx.save_for_backward(cols, wm)
        ctx.geo = (B, C, H, W, O, Cg, kh, kw, G, s, p, Ho, Wo)
        ctx.dt = (x.dtype, w.dtype, None if bias is None else bias.dtype)
        return y.view(B, O, Ho, Wo).to(x.dtype)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dy):
        cols, wm = ctx.saved_tensors
        B, C, H, W, O, Cg, kh, kw, G, s, p, Ho, Wo = ctx.geo
        xdt, wdt, bdt = ctx.dt
        dyf = dy.float().contiguous().view(B, G, O // G, Ho * Wo)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dcols = torch.empty([B, G, Cg * kh * kw, Ho * Wo], dtype=torch.float32, device=dy.device)
            _grouped(wm, dyf, G, dcols, transpose_w=True)
            dx = _col2im(dcols.view(B, C * kh * kw, Ho * Wo), B, C, H, W, kh, kw, s, p, Ho, Wo).to(xdt)
        if ctx.needs_input_grad[1] and not conv2d_gradfix.weight_gradients_disabled:
            dwm = torch.stack([_gemm(dyf[:, g], cols[:, g].transpose(1, 2), reduce_batch=True) for g in range(G)])
            dw = dwm.view(O, Cg, kh, kw).to(wdt)
        if bdt is not None and ctx.needs_input_grad[2]:
            db = dyf.sum((0, 3)).reshape(O).to(bdt)
        return dx, dw, db, None, None, None


class _ConvTranspose2d(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, x, w, bias, stride, padding, output_padding, groups):
        B, Cin, H, W = x.shape
        _, Og, kh, kw = w.shape
        G = groups
        Cg = Cin // G
        s, p, op = _pair(stride), _pair(padding), _pair(output_padding)
        Ho = (H - 1) * s[0] - 2 * p[0] + kh + op[0]
        Wo = (W - 1) * s[1] - 2 * p[1] + kw + op[1]
        xf = x.detach().float().contiguous().view(B, G, Cg, H * W)
        wm = w.detach().float().reshape(G, Cg, Og * kh * kw).contiguous()          # W_g [Cg, Og k^2]
        cols = torch.empty([B, G, Og * kh * kw, H * W], dtype=torch.float32, device=x.device)
        _grouped(wm, xf, G, cols, transpose_w=True)
        y = _col2im(cols.view(B, G * Og * kh * kw, H * W), B, G * Og, Ho, Wo, kh, kw, s, p, H, W)
        if bias is not None:
            y.add_(bias.detach().float().view(1, -1, 1, 1))
        ctx.save_for_backward(xf, wm)
        ctx.geo = (B, Cin, H, W, Og, kh, kw, G, s, p, Ho, Wo)
        ctx.dt = (x.dtype, w.dtype, None if bias is None else bias.dtype)
        return y.to(x.dtype)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dy):
        xf, wm = ctx.saved_tensors
        B, Cin, H, W, Og, kh, kw, G, s, p, Ho, Wo = ctx.geo
        xdt, wdt, bdt = ctx.dt
        Cg = Cin // G
        dyf = dy.float().contiguous()
        dx = dw = db = None
        cols = _im2col(dyf, kh, kw, s, p, H, W).view(B, G, Og * kh * kw, H * W)
        if ctx.needs_input_grad[0]:
            dxv = torch.empty([B, G, Cg, H * W], dtype=torch.float32, device=dy.device)
            _grouped(wm, cols, G, dxv)
            dx = dxv.view(B, Cin, H, W).to(xdt)
        if ctx.needs_input_grad[1] and not conv2d_gradfix.weight_gradients_disabled:
            dwm = torch.stack([_gemm(xf[:, g], cols[:, g].transpose(1, 2), reduce_batch=True) for g in range(G)])
            dw = dwm.view(Cin, Og, kh, kw).to(wdt)
        if bdt is not None and ctx.needs_input_grad[2]:
            db = dyf.sum((0, 2, 3)).to(bdt)
        return dx, dw, db, None, None, None, None


def conv2d(x, w, bias=None, stride=1, padding=0, groups=1):
    return _Conv2d.apply(x, w, bias, stride, padding, int(groups))


def conv_transpose2d(x, w, bias=None, stride=1, padding=0, output_padding=0, groups=1):
    return _ConvTranspose2d.apply(x, w, bias, stride, padding, output_padding, int(groups))
