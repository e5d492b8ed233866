"""nn.Linear on the MFMA GEMM (csrc/gemm.hip) with autograd.

Used by the trainable fusion adapter (reference networks/utils/ldm_utils.py:55-166:
PlainAttention.qkv / proj, AttnProjectionBlock.proj, GeGluMlp w0/w1/w2; fp32, outside
autocast) and the frozen DINO ViT-S of the projected discriminator (discriminator.py:145-168,
fp32, gradients w.r.t. its input only). `Linear` is a drop-in nn.Linear subclass (same
parameters and state-dict keys); on ROCm tensors its forward and backward products run on
the HIP GEMM (fp32 operands as the fp32-equivalent f32x6 split, csrc/gemm.hip), elsewhere F.linear.

  forward   y  = x W^T + b            (bias in the GEMM epilogue)
  backward  dx = dy W,  dW = dy^T x (fp32),  db = sum dy
Gradients that the autograd engine will not consume in this pass are not computed (see
decoder_hip._wanted: the adaptive-VF `autograd.grad` runs data-only backward passes).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F
from .. import custom_ops


def _gemm():
    from . import gemm_hip          # loads the kernel library (ROCm tensors only reach here)
    return gemm_hip


def _wanted(ctx, i):
    from .decoder_hip import _wanted as w
    return w(ctx, i)


def _edges(ctx, *args):
    from .decoder_hip import _edges as e
    e(ctx, *args)


class _LinearFn(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, x, w, b):
        _edges(ctx, x, w, b)
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        if x2.stride(-1) != 1:
            x2 = x2.contiguous()
        wc = w if w.dtype == x.dtype else w.to(x.dtype)
        y = _gemm().try_gemm(x2, wc.t(), bias=b, bias_dim=1, cache_b=True, auto=True)
        if y is None:
            y = F.linear(x2, wc, None if b is None else b.to(x.dtype))
        ctx.save_for_backward(x2, wc)
        ctx.meta = (shape, w.dtype, None if b is None else b.dtype)
        return y.reshape(*shape[:-1], w.shape[0])

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dy):
        x2, wc = ctx.saved_tensors
        shape, wdt, bdt = ctx.meta
        dy2 = dy.reshape(-1, dy.shape[-1])
        if dy2.stride(-1) != 1 or dy2.dtype != x2.dtype:
            dy2 = dy2.contiguous().to(x2.dtype)
        dx = dw = db = None
        if ctx.needs_input_grad[0] and _wanted(ctx, 0):
            dx = _gemm().try_gemm(dy2, wc, cache_b=True, auto=True)
            if dx is None:
                dx = dy2 @ wc
            dx = dx.reshape(shape)
        if ctx.needs_input_grad[1] and _wanted(ctx, 1):
            dw = _gemm().try_gemm(dy2.t(), x2, out_dtype=torch.float32, auto=True)
            if dw is None:
                dw = dy2.t().float() @ x2.float()
            dw = dw.to(wdt)
        if bdt is not None and ctx.needs_input_grad[2] and _wanted(ctx, 2):
            db = dy2.sum(0, dtype=torch.float32).to(bdt)
        return dx, dw, db


class _BmmFn(custom_ops.FastFunction):
    """C[z] = A[z] @ B[z] (fp32 / bf16 ROCm views) on our GEMMs, both gradients on them too."""

    @staticmethod
    def forward(ctx, a, b):
        _edges(ctx, a, b)
        out = _gemm().try_gemm(a, b, auto=True)
        if out is None:
            out = torch.bmm(a, b)
        ctx.save_for_backward(a, b)
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dc):
        a, b = ctx.saved_tensors
        da = db = None
        if ctx.needs_input_grad[0] and _wanted(ctx, 0):
            da = _gemm().try_gemm(dc, b.transpose(1, 2), auto=True)
            if da is None:
                da = torch.bmm(dc, b.transpose(1, 2))
        if ctx.needs_input_grad[1] and _wanted(ctx, 1):
            db = _gemm().try_gemm(a.transpose(1, 2), dc, auto=True)
            if db is None:
                db = torch.bmm(a.transpose(1, 2), dc)
        return da, db


def bmm(a, b):
    """torch.bmm with its forward and backward products on the HIP GEMMs for ROCm fp32 / bf16 operands (the
    adapter's VF-loss cosine Gram matrices, reference networks/utils/ldm_utils.py:385-395)."""
    if a.is_cuda and a.dtype == b.dtype and a.dtype in (torch.float32, torch.bfloat16):
        return _BmmFn.apply(a, b)
    return torch.bmm(a, b)


def linear(x, weight, bias=None):
    if x.is_cuda and x.dtype in (torch.float32, torch.bfloat16):
        return _LinearFn.apply(x, weight, bias)
    return F.linear(x, weight, bias)


class Linear(nn.Linear):
    """nn.Linear whose ROCm forward/backward run on the HIP GEMM."""

    def forward(self, x):
        return linear(x, self.weight, self.bias)
