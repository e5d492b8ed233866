"""Fused multiply-add `fma(a, b, c) = a * b + c` with broadcast-aware gradients
(reference `torch_utils/ops/fma.py:15-58`)."""
import torch


def fma(a, b, c):
    return _FusedMultiplyAdd.apply(a, b, c)


def _reduce_to(t, shape):
    """Sum `t` over the dimensions that were broadcast to produce it from `shape`."""
    shape = tuple(shape)
    lead = t.ndim - len(shape)
    assert lead >= 0
    if lead:
        t = t.sum(dim=tuple(range(lead)))
    dims = tuple(i for i, s in enumerate(shape) if s == 1 and t.shape[i] != 1)
    if dims:
        t = t.sum(dim=dims, keepdim=True)
    assert tuple(t.shape) == shape
    return t


class _FusedMultiplyAdd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, c):
        ctx.save_for_backward(a, b)
        ctx.c_shape = c.shape
        return torch.addcmul(c, a, b)

    @staticmethod
    def backward(ctx, dout):
        a, b = ctx.saved_tensors
        da = _reduce_to(dout * b, a.shape) if ctx.needs_input_grad[0] else None
        db = _reduce_to(dout * a, b.shape) if ctx.needs_input_grad[1] else None
        dc = _reduce_to(dout, ctx.c_shape) if ctx.needs_input_grad[2] else None
        return da, db, dc
