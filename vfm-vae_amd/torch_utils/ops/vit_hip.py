"""gfx950 row kernels of the frozen ViT towers (csrc/vit.hip, C ABI in include/vfmvae.h).

The residual LayerNorm is forward only: the SigLIP2 encoder is frozen and runs under no_grad
(reference networks/utils/vfms/siglip2_utils.py:114-137). `layer_norm_grad` is the LayerNorm with a
backward to its input for the frozen DINOv2 discriminator backbone in the G phase. Loading the library
raises if it is missing (no silent fallback on ROCm tensors).
"""
import os

import torch

from .. import custom_ops
from . import kernel_timer

_lib = custom_ops.get_native()


def supported(h):
    return h.is_cuda and h.dtype == torch.float32 and h.shape[-1] % 256 == 0 and h.shape[-1] <= 2048


def residual_layer_norm(h, delta, ln, out_dtype, write_h=True):
    """(h + delta, LayerNorm(h + delta) in out_dtype); delta None -> (h, LN(h)).
    h: fp32 [..., D] contiguous; delta: [..., D] any float dtype."""
    if torch.is_grad_enabled() and (h.requires_grad or (delta is not None and delta.requires_grad)):
        raise RuntimeError("vit_hip.residual_layer_norm is forward-only (frozen tower under no_grad)")
    h = h.contiguous()
    D = h.shape[-1]
    rows = h.numel() // D
    y = torch.empty(h.shape, dtype=out_dtype, device=h.device)
    h_out = None
    if delta is not None:
        delta = delta.contiguous()
        if delta.shape != h.shape:
            raise RuntimeError(f"delta shape {tuple(delta.shape)} != h shape {tuple(h.shape)}")
        if write_h:
            h_out = torch.empty_like(h)
    w = ln.weight.detach().float().contiguous() if ln.weight is not None else None
    b = ln.bias.detach().float().contiguous() if ln.bias is not None else None
    # the kernel reads the affine parameters as 16-B vectors
    w = w.clone() if w is not None and w.data_ptr() % 16 else w
    b = b.clone() if b is not None and b.data_ptr() % 16 else b
    es = 0 if delta is None else delta.element_size()
    nbytes = rows * D * (4 + es + y.element_size() + (4 if h_out is not None else 0))
    with kernel_timer.region('residual_layer_norm', nbytes):
        rc = _lib.vfm_residual_layer_norm(h.data_ptr(), custom_ops.ptr(delta), custom_ops.ptr(h_out),
                                          custom_ops.ptr(w), custom_ops.ptr(b), y.data_ptr(),
                                          custom_ops.dtype_code(delta) if delta is not None else 0,
                                          custom_ops.dtype_code(y), rows, D, float(ln.eps),
                                          custom_ops.stream_ptr(h.device))
    custom_ops.check(rc, "vfm_residual_layer_norm")
    return (h_out if h_out is not None else h), y


_DN = {torch.float32: "f32", torch.bfloat16: "bf16", torch.float16: "f16"}
# Routing switch (vit_utils.Block / vit_ops.layer_norm): on by default since round 6. The kernels replace
# torch's LayerNorm kernels in the DINO discriminator (2.1 -> 0.8 ms/step of kernel time); round 5 measured
# them 1-2 % slower in the bench (profiles/r5_bp_ln_grad_ab.txt: per-call host work), since then the frozen
# affine parameters are cached on the module (`_frozen_affine`). VFM_LN_GRAD=0: torch's LayerNorm (A/B).
LN_GRAD = os.environ.get("VFM_LN_GRAD", "1") == "1"


def layer_norm_grad_supported(h, ln):
    """fp32 [.., D] input needing a gradient, frozen (or absent) affine parameters, D % 128 == 0, D <= 1024."""
    D = h.shape[-1]
    return (h.is_cuda and h.dtype == torch.float32 and D % 128 == 0 and D <= 1024 and h.numel() > 0
            and not (ln.weight is not None and ln.weight.requires_grad)
            and not (ln.bias is not None and ln.bias.requires_grad))


class _LayerNorm(custom_ops.FastFunction):
    """LayerNorm(x) * w + b in out_dtype with fp32 statistics; gradient to x only (frozen w / b)."""

    @staticmethod
    def forward(ctx, x, w, b, eps, out_dtype):
        x = x.contiguous()
        D = x.shape[-1]
        rows = x.numel() // D
        y = torch.empty(x.shape, dtype=out_dtype, device=x.device)
        mean = torch.empty([rows], dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        with kernel_timer.region(f'layer_norm_fwd<{_DN[y.dtype]}>', rows * D * (4 + y.element_size())):
            custom_ops.check(_lib.vfm_layer_norm_fwd(x.data_ptr(), custom_ops.ptr(w), custom_ops.ptr(b), y.data_ptr(),
                                                     mean.data_ptr(), rstd.data_ptr(), custom_ops.dtype_code(y), rows,
                                                     D, float(eps), custom_ops.stream_ptr(x.device)),
                             "vfm_layer_norm_fwd")
        ctx.save_for_backward(x, w, mean, rstd)
        return y

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dy):
        x, w, mean, rstd = ctx.saved_tensors
        D = x.shape[-1]
        rows = x.numel() // D
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        with kernel_timer.region(f'layer_norm_bwd<{_DN[dy.dtype]}>', rows * D * (8 + dy.element_size())):
            custom_ops.check(_lib.vfm_layer_norm_bwd(x.data_ptr(), dy.data_ptr(), custom_ops.ptr(w), mean.data_ptr(),
                                                     rstd.data_ptr(), dx.data_ptr(), custom_ops.dtype_code(dy), rows,
                                                     D, custom_ops.stream_ptr(x.device)), "vfm_layer_norm_bwd")
        return dx, None, None, None, None


def _frozen_affine(ln):
    """fp32, contiguous, 8-B aligned (w, b) of a frozen LayerNorm, cached on the module until a parameter's
    version or storage moves (the per-call detach / cast / alignment checks were most of this op's host time)."""
    key = tuple((t.data_ptr(), t._version) if t is not None else None for t in (ln.weight, ln.bias))
    hit = getattr(ln, "_vfm_affine", None)
    if hit is not None and hit[0] == key and not torch.cuda.is_current_stream_capturing():
        return hit[1]
    out = []
    for t in (ln.weight, ln.bias):
        t = t.detach().float().contiguous() if t is not None else None
        out.append(t.clone() if t is not None and t.data_ptr() % 8 else t)
    if not torch.cuda.is_current_stream_capturing():
        ln._vfm_affine = (key, tuple(out))
    return tuple(out)


def layer_norm_grad(h, ln, out_dtype):
    """LayerNorm of an fp32 stream that needs a gradient, through frozen parameters (DINOv2 discriminator)."""
    w, b = _frozen_affine(ln)
    return _LayerNorm.apply(h, w, b, float(ln.eps), out_dtype)
