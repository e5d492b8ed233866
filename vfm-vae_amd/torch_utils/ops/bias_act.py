"""Fused bias + activation + gain + clamp with 1st/2nd-order gradients.

Drop-in for the reference `torch_utils/ops/bias_act.py` (activation table
:21-31, API :52-86). `impl='cuda'` on a ROCm device runs `csrc/bias_act.hip`
via the C ABI `vfm_bias_act`; `impl='ref'` or CPU tensors run `_bias_act_ref`.
"""
import numpy as np
import torch

import dnnlib
from .. import custom_ops
from .. import misc

# name -> func (ref path), default alpha/gain, kernel code, which forward tensor the
# gradient needs ('x', 'y' or ''), and whether a 2nd-order gradient exists.
activation_funcs = {
    'linear':   dnnlib.EasyDict(func=lambda x, **_: x,                                        def_alpha=0,   def_gain=1,          cuda_idx=1, ref='',  has_2nd_grad=False),
    'relu':     dnnlib.EasyDict(func=lambda x, **_: torch.nn.functional.relu(x),              def_alpha=0,   def_gain=np.sqrt(2), cuda_idx=2, ref='y', has_2nd_grad=False),
    'lrelu':    dnnlib.EasyDict(func=lambda x, alpha, **_: torch.nn.functional.leaky_relu(x, alpha), def_alpha=0.2, def_gain=np.sqrt(2), cuda_idx=3, ref='y', has_2nd_grad=False),
    'tanh':     dnnlib.EasyDict(func=lambda x, **_: torch.tanh(x),                            def_alpha=0,   def_gain=1,          cuda_idx=4, ref='y', has_2nd_grad=True),
    'sigmoid':  dnnlib.EasyDict(func=lambda x, **_: torch.sigmoid(x),                         def_alpha=0,   def_gain=1,          cuda_idx=5, ref='y', has_2nd_grad=True),
    'elu':      dnnlib.EasyDict(func=lambda x, **_: torch.nn.functional.elu(x),               def_alpha=0,   def_gain=1,          cuda_idx=6, ref='y', has_2nd_grad=True),
    'selu':     dnnlib.EasyDict(func=lambda x, **_: torch.nn.functional.selu(x),              def_alpha=0,   def_gain=1,          cuda_idx=7, ref='y', has_2nd_grad=True),
    'softplus': dnnlib.EasyDict(func=lambda x, **_: torch.nn.functional.softplus(x),          def_alpha=0,   def_gain=1,          cuda_idx=8, ref='y', has_2nd_grad=True),
    'swish':    dnnlib.EasyDict(func=lambda x, **_: torch.sigmoid(x) * x,                     def_alpha=0,   def_gain=np.sqrt(2), cuda_idx=9, ref='x', has_2nd_grad=True),
}


def _resolve(act, alpha, gain, clamp):
    assert clamp is None or clamp >= 0
    spec = activation_funcs[act]
    alpha = float(alpha if alpha is not None else spec.def_alpha)
    gain = float(gain if gain is not None else spec.def_gain)
    clamp = float(clamp if clamp is not None else -1)
    return spec, alpha, gain, clamp


def bias_act(x, b=None, dim=1, act='linear', alpha=None, gain=None, clamp=None, impl='cuda'):
    """y = clamp(act(x + b) * gain, -clamp, clamp); b is broadcast along `dim`.

    Any rank; contiguous or channels-last. Matches reference bias_act.py:52-86.
    """
    assert isinstance(x, torch.Tensor)
    assert impl in ('ref', 'cuda')
    if impl == 'cuda' and x.device.type == 'cuda':
        spec, alpha, gain, clamp = _resolve(act, alpha, gain, clamp)
        return _BiasActHip.apply(x, b, dim, act, alpha, gain, clamp)
    return _bias_act_ref(x=x, b=b, dim=dim, act=act, alpha=alpha, gain=gain, clamp=clamp)


@misc.profiled_function
def _bias_act_ref(x, b=None, dim=1, act='linear', alpha=None, gain=None, clamp=None):
    """Pure-torch restatement (reference bias_act.py:90-120)."""
    assert isinstance(x, torch.Tensor)
    spec, alpha, gain, clamp = _resolve(act, alpha, gain, clamp)
    if b is not None:
        assert isinstance(b, torch.Tensor) and b.ndim == 1 and 0 <= dim < x.ndim and b.shape[0] == x.shape[dim]
        shape = [1] * x.ndim
        shape[dim] = -1
        x = x + b.reshape(shape)
    x = spec.func(x, alpha=alpha)
    if gain != 1:
        x = x * gain
    if clamp >= 0:
        x = x.clamp(-clamp, clamp)
    return x


# ---------------------------------------------------------------------------
# HIP path.


def _memfmt(x):
    return torch.channels_last if (x.ndim == 4 and x.stride(1) == 1 and x.shape[1] > 1) else torch.contiguous_format


def _run(x, b, xref, yref, dy, grad, dim, spec, alpha, gain, clamp):
    """One launch through the registered op torch.ops.vfmvae.bias_act (csrc/torch_ops.cpp over
    vfm_bias_act; the reference plugin's schema, empty tensors for absent inputs, bias_act.cpp:32-90)."""
    e = x.new_empty([0])
    return custom_ops.get_torch_ops().bias_act(x, e if b is None else b.contiguous(), e if xref is None else xref,
                                               e if yref is None else yref, e if dy is None else dy, int(grad),
                                               int(dim), int(spec.cuda_idx), float(alpha), float(gain), float(clamp))


class _BiasActHip(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, x, b, dim, act, alpha, gain, clamp):
        spec = activation_funcs[act]
        ctx.memory_format = _memfmt(x)
        x = x.contiguous(memory_format=ctx.memory_format)
        b = b.contiguous() if b is not None else None
        y = x
        if act != 'linear' or gain != 1 or clamp >= 0 or b is not None:
            y = _run(x, b, None, None, None, 0, dim, spec, alpha, gain, clamp)
        need_x = 'x' in spec.ref or spec.has_2nd_grad
        # y is also needed for the clamp mask of the gradient. The reference CUDA path drops
        # it for act='linear' (bias_act.py:151-154 saves y only if 'y' in spec.ref), so its kernel
        # never zeroes the gradient of clamped outputs there; _bias_act_ref (autograd through
        # torch.clamp) does. We follow the mathematically exact _ref behaviour.
        need_y = 'y' in spec.ref or clamp >= 0
        ctx.save_for_backward(x if need_x else None, b if need_x else None, y if need_y else None)
        ctx.cfg = (dim, act, alpha, gain, clamp)
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous(memory_format=ctx.memory_format)
        x, b, y = ctx.saved_tensors
        dim, act, alpha, gain, clamp = ctx.cfg
        dx = db = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            dx = dy
            if act != 'linear' or gain != 1 or clamp >= 0:
                dx = _BiasActGradHip.apply(dy, x, b, y, ctx.cfg, ctx.memory_format)
        if ctx.needs_input_grad[1]:
            db = dx.sum([i for i in range(dx.ndim) if i != dim])
        return dx, db, None, None, None, None, None


class _BiasActGradHip(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, dy, x, b, y, cfg, memory_format):
        dim, act, alpha, gain, clamp = cfg
        spec = activation_funcs[act]
        dx = _run(dy, b, x, y, None, 1, dim, spec, alpha, gain, clamp)
        ctx.save_for_backward(dy if spec.has_2nd_grad else None, x, b, y)
        ctx.cfg = cfg
        ctx.memory_format = memory_format
        return dx

    @staticmethod
    def backward(ctx, d_dx):
        d_dx = d_dx.contiguous(memory_format=ctx.memory_format)
        dy, x, b, y = ctx.saved_tensors
        dim, act, alpha, gain, clamp = ctx.cfg
        spec = activation_funcs[act]
        d_dy = d_x = d_b = None
        if ctx.needs_input_grad[0]:
            d_dy = _BiasActGradHip.apply(d_dx, x, b, y, ctx.cfg, ctx.memory_format)
        if spec.has_2nd_grad and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2]):
            d_x = _run(d_dx, b, x, y, dy, 2, dim, spec, alpha, gain, clamp)
        if spec.has_2nd_grad and ctx.needs_input_grad[2]:
            d_b = d_x.sum([i for i in range(d_x.ndim) if i != dim])
        return d_dy, d_x, d_b, None, None, None
