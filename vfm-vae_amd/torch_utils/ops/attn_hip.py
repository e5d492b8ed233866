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


# ------------------------------------------------------------------------------------------------
# fp32 attention with gradients (csrc/attention_f32.hip): the generator's fusion-adapter
# AttnProjection (reference networks/utils/ldm_utils.py:55-93; encode heads of 64, the decode
# post_quant's heads of 32) and decoder SelfAttention with null key/value (reference
# networks/utils/gigagan_utils.py:53-91), both fp32 and trained, and the DINO discriminator
# tower. fp32-equivalent products (f32x6; f32x3 opt-in, custom_ops.F32_PRODUCTS).

def _s4(t):
    """(batch, token, head) strides of a [B, N, H, d] fp32 view the kernel can read in place."""
    st = t.stride()
    if st[3] != 1 or any(x % 4 for x in st[:3]) or t.data_ptr() % 16:
        return None
    return custom_ops.strides_of([st[0], st[1], st[2]])


def _ready(t):
    s = _s4(t)
    if s is None:
        t = t.contiguous()
        s = _s4(t)
    return t, s


class _Attention32(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, q, k, v):
        B, Nq, H, d = q.shape
        Nk = k.shape[1]
        (q, sq), (k, sk), (v, sv) = _ready(q), _ready(k), _ready(v)
        o = torch.empty(B, Nq, H, d, dtype=torch.float32, device=q.device)
        lse = torch.empty(B, H, Nq, dtype=torch.float32, device=q.device)
        flops = 4 * B * H * Nq * Nk * d
        prec, _, tag = custom_ops.f32_precision()
        with kernel_timer.region(f"attention_fwd<{tag},{d}>", 4 * (2 * B * Nq * H * d + 2 * B * Nk * H * d), flops,
                                 "mfma"):
            rc = _lib.vfm_attention_f32_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(),
                                            B, H, Nq, Nk, d, sq, sk, sv, _s4(o), float(d) ** -0.5, prec,
                                            custom_ops.stream_ptr(q.device))
        custom_ops.check(rc, "vfm_attention_f32_fwd")
        ctx.save_for_backward(q, k, v, o, lse)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        B, Nq, H, d = q.shape
        Nk = k.shape[1]
        do, sdo = _ready(do)
        dq = torch.empty(B, Nq, H, d, dtype=torch.float32, device=q.device)
        dk = torch.empty(B, Nk, H, d, dtype=torch.float32, device=q.device)
        dv = torch.empty(B, Nk, H, d, dtype=torch.float32, device=q.device)
        delta = torch.empty(B, H, Nq, dtype=torch.float32, device=q.device)
        flops = 10 * B * H * Nq * Nk * d          # S and dP recomputed in both passes, dV, dK, dQ
        prec, _, tag = custom_ops.f32_precision()
        with kernel_timer.region(f"attention_bwd<{tag},{d}>", 4 * 4 * (B * Nq * H * d + B * Nk * H * d), flops,
                                 "mfma"):
            rc = _lib.vfm_attention_f32_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), do.data_ptr(),
                                            lse.data_ptr(), delta.data_ptr(), dq.data_ptr(), dk.data_ptr(),
                                            dv.data_ptr(), B, H, Nq, Nk, d, _s4(q), _s4(k), _s4(v), _s4(o), sdo,
                                            _s4(dq), _s4(dk), _s4(dv), float(d) ** -0.5, prec,
                                            custom_ops.stream_ptr(q.device))
        custom_ops.check(rc, "vfm_attention_f32_bwd")
        return dq, dk, dv


class _Attention32Packed(custom_ops.FastFunction):
    """The same kernels on a packed projection qkv [B, N, 3, H, d] (a view of a linear's [B, N, 3 H d]
    output): q / k / v are read in place and the backward writes dq / dk / dv into ONE packed gradient
    buffer, so autograd neither copies the strided views nor stacks three gradients back together."""

    @staticmethod
    def forward(ctx, qkv):
        q, k, v = qkv.unbind(2)
        o = _Attention32.forward(ctx, q, k, v)
        ctx.packed_shape = qkv.shape
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        B, Nq, H, d = q.shape
        do, sdo = _ready(do)
        dqkv = torch.empty(ctx.packed_shape, dtype=torch.float32, device=q.device)
        dq, dk, dv = dqkv.unbind(2)
        delta = torch.empty(B, H, Nq, dtype=torch.float32, device=q.device)
        flops = 10 * B * H * Nq * Nq * d
        prec, _, tag = custom_ops.f32_precision()
        with kernel_timer.region(f"attention_bwd<{tag},{d}>", 4 * 4 * 2 * B * Nq * H * d, flops, "mfma"):
            rc = _lib.vfm_attention_f32_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), do.data_ptr(),
                                            lse.data_ptr(), delta.data_ptr(), dq.data_ptr(), dk.data_ptr(),
                                            dv.data_ptr(), B, H, Nq, Nq, d, _s4(q), _s4(k), _s4(v), _s4(o), sdo,
                                            _s4(dq), _s4(dk), _s4(dv), float(d) ** -0.5, prec,
                                            custom_ops.stream_ptr(q.device))
        custom_ops.check(rc, "vfm_attention_f32_bwd")
        return dqkv


def sdpa_f32_packed(qkv, heads):
    """sdpa over a packed fp32 projection qkv [B, N, 3 H d] (d = 64 or 32) -> [B, H, N, d] (a view of a
    token-major tensor), or None when the layout does not fit the kernels (the caller unpacks)."""
    B, N, D3 = qkv.shape
    d = D3 // (3 * heads)
    if not (qkv.is_cuda and qkv.dtype == torch.float32 and d in (32, HEAD_DIM) and 3 * heads * d == D3):
        return None
    q5 = qkv.reshape(B, N, 3, heads, d)
    if _s4(q5[:, :, 0]) is None:
        return None
    return _Attention32Packed.apply(q5).transpose(1, 2)


def supported_f32(q, k, v):
    return (q.is_cuda and q.dtype == torch.float32 and k.dtype == torch.float32 and v.dtype == torch.float32
            and q.shape[-1] in (32, HEAD_DIM) and k.shape == v.shape and q.shape[0] == k.shape[0]
            and q.shape[1] == k.shape[1])


def sdpa_f32(q, k, v):
    """F.scaled_dot_product_attention(q, k, v) for fp32 [B, H, N, 64 or 32] operands (no mask, default
    scale), forward and backward on the HIP kernels. Returns [B, H, Nq, d] (a view of a
    token-major [B, Nq, H, 64] tensor)."""
    o = _Attention32.apply(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2))
    return o.transpose(1, 2)
