"""Fused self-attention forward of the frozen ViT towers (csrc/attention.hip).

Replaces `F.scaled_dot_product_attention(q, k, v)` in HF SiglipAttention under bf16
autocast (reference networks/utils/vfms/siglip2_utils.py:121) and in the DINOv2 / CLIP
towers. Forward only (the towers run frozen under no_grad); bf16, head dim 64. The
library is required on ROCm tensors: a missing kernel library raises (no fallback).
"""
import torch

from .. import custom_ops
from . import kernel_timer

_lib = custom_ops.get_native()
HEAD_DIM = 64


def supported(x, head_dim):
    return x.is_cuda and x.dtype == torch.bfloat16 and head_dim == HEAD_DIM


def _strides(t):
    """(batch, token, head) element strides of a [B, N, H, d] view with unit stride on d."""
    if t.stride(3) != 1:
        raise RuntimeError("attention operand needs unit stride along the head dim")
    return custom_ops.strides_of([t.stride(0), t.stride(1), t.stride(2)])


def attention(q, k, v, out=None):
    """q, k, v: bf16 [B, N, H, 64] views (any batch/token/head strides) -> o [B, N, H, 64]
    (a fresh contiguous tensor unless `out` is given)."""
    if torch.is_grad_enabled() and (q.requires_grad or k.requires_grad or v.requires_grad):
        raise RuntimeError("attn_hip.attention is forward-only (frozen towers under no_grad)")
    B, N, H, d = q.shape
    if k.shape != q.shape or v.shape != q.shape:
        raise RuntimeError(f"q/k/v shapes differ: {tuple(q.shape)} {tuple(k.shape)} {tuple(v.shape)}")
    if out is None:
        out = torch.empty(B, N, H, d, dtype=q.dtype, device=q.device)
    flops = 4 * B * H * N * N * d
    nbytes = 4 * B * N * H * d * q.element_size()
    with kernel_timer.region(f"attention_fwd<bf16,{d}>", nbytes, flops, "mfma"):
        rc = _lib.vfm_attention_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), B, H, N, d,
                                    _strides(q), _strides(k), _strides(v), _strides(out), float(d) ** -0.5,
                                    custom_ops.stream_ptr(q.device))
    custom_ops.check(rc, "vfm_attention_fwd")
    return out


def attention_packed(qkv, heads):
    """qkv: bf16 [B, N, 3*D] (q | k | v, heads contiguous inside each) -> [B, N, D]."""
    B, N, D3 = qkv.shape
    D = D3 // 3
    v5 = qkv.view(B, N, 3, heads, D // heads)
    o = attention(v5[:, :, 0], v5[:, :, 1], v5[:, :, 2])
    return o.view(B, N, D)
