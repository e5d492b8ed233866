"""gfx950 row kernels of the frozen ViT towers (csrc/vit.hip, C ABI in include/vfmvae.h).

Forward only: the SigLIP2 encoder is frozen and runs under no_grad
(reference networks/utils/vfms/siglip2_utils.py:114-137). Loading the library
raises if it is missing (no silent fallback on ROCm tensors).
"""
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
