"""Decoder attention blocks (GigaGAN-style, channel-first) with learned null key/value.

Same classes and parameter names as the reference `networks/utils/gigagan_utils.py`
(ChannelRMSNorm :31-39, SelfAttention :53-91, CrossAttention :94-146,
FeedForward :149-167, SelfAttentionBlock :170-185, CrossAttentionBlock :188-204).
The 1x1 projections run as GEMMs on [B, C, HW] views; attention is fused
(`scaled_dot_product_attention`, flash kernels on ROCm).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from torch_utils.ops import decoder_ops, vit_ops


def exists(v):
    return v is not None


def default(*vals):
    for v in vals:
        if v is not None:
            return v
    return None


class ChannelRMSNorm(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.scale = dim ** 0.5
        self.gamma = nn.Parameter(torch.ones(dim, 1, 1))

    def forward(self, x):
        if x.is_cuda:
            from torch_utils.ops import decoder_hip
            if decoder_hip.channel_rms_norm_supported(x):
                # one HIP launch (csrc/rmsnorm.hip); torch's channel-norm reduction also replays wrongly
                # from a HIP graph
                return decoder_hip.channel_rms_norm(x, self.gamma, self.scale)
        return F.normalize(x, dim=1) * self.scale * self.gamma


class RMSNorm(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.scale = dim ** 0.5
        self.gamma = nn.Parameter(torch.ones(dim))

    def forward(self, x):
        return F.normalize(x, dim=-1) * self.scale * self.gamma


def _pointwise(conv: nn.Conv2d, x3):
    """1x1 conv on a [B, C, P] view as a GEMM."""
    w = conv.weight.reshape(conv.out_channels, conv.in_channels)
    y = decoder_ops.pointwise(w, x3)
    if conv.bias is not None:
        y = y + conv.bias.to(y.dtype)[None, :, None]
    return y


class SelfAttention(nn.Module):
    def __init__(self, dim, dim_head=64, heads=8):
        super().__init__()
        self.heads = heads
        self.dim_head = dim_head
        inner = dim_head * heads
        self.norm = ChannelRMSNorm(dim)
        self.to_q = nn.Conv2d(dim, inner, 1, bias=False)
        self.to_k = nn.Conv2d(dim, inner, 1, bias=False)
        self.to_v = nn.Conv2d(dim, inner, 1, bias=False)
        self.null_kv = nn.Parameter(torch.randn(2, heads, dim_head) * 0.02)
        self.to_out = nn.Conv2d(inner, dim, 1, bias=False)
        nn.init.zeros_(self.to_out.weight)

    # fp32 ROCm inputs: projections, attention with the null key / value and the output projection as one
    # Function with no activation copies (torch_utils/ops/gigaattn_hip.py); VFM_GIGA_ATTN=0: unfused chain
    fused = __import__("os").environ.get("VFM_GIGA_ATTN", "1") == "1"

    def forward(self, fmap):
        B, C, H, W = fmap.shape
        h, d = self.heads, self.dim_head
        x = self.norm(fmap).reshape(B, C, H * W)
        wqkv = torch.cat([self.to_q.weight, self.to_k.weight, self.to_v.weight], 0).reshape(3 * h * d, C)
        if self.fused and self.to_out.bias is None and not decoder_ops.force_ref():
            from torch_utils.ops import gigaattn_hip
            if gigaattn_hip.supported(x, h, d):
                y = gigaattn_hip.null_kv_self_attention(x, wqkv, self.null_kv,
                                                        self.to_out.weight.reshape(C, h * d), h)
                return y.reshape(B, C, H, W)
        qkv = decoder_ops.pointwise(wqkv, x)                                   # [B, 3hd, P]
        q, k, v = qkv.reshape(B, 3, h, d, H * W).permute(1, 0, 2, 4, 3).unbind(0)  # [B, h, P, d]
        nk, nv = (t.to(q.dtype)[None, :, None, :].expand(B, h, 1, d) for t in self.null_kv.unbind(0))
        k = torch.cat([nk, k], dim=2)
        v = torch.cat([nv, v], dim=2)
        out = vit_ops.sdpa(q, k, v)                                            # [B, h, P, d]
        out = out.permute(0, 1, 3, 2).reshape(B, h * d, H * W)
        return _pointwise(self.to_out, out).reshape(B, C, H, W)


class CrossAttention(nn.Module):
    def __init__(self, dim, dim_context, dim_head=64, heads=8):
        super().__init__()
        self.heads = heads
        self.dim_head = dim_head
        inner = dim_head * heads
        kv_input_dim = default(dim_context, dim)
        self.norm = ChannelRMSNorm(dim)
        self.norm_context = RMSNorm(kv_input_dim)
        self.to_q = nn.Conv2d(dim, inner, 1, bias=False)
        self.to_kv = nn.Linear(kv_input_dim, inner * 2, bias=False)
        self.to_out = nn.Conv2d(inner, dim, 1, bias=False)
        nn.init.zeros_(self.to_out.weight)
        self.null_kv = nn.Parameter(torch.randn(2, heads, dim_head) * 0.02)

    def forward(self, fmap, context, mask=None):
        B, C, H, W = fmap.shape
        h, d = self.heads, self.dim_head
        x = self.norm(fmap).reshape(B, C, H * W)
        ctx = self.norm_context(context)
        q = _pointwise(self.to_q, x).reshape(B, h, d, H * W).transpose(2, 3)
        if q.is_cuda:                                   # fused SDPA needs stride(-1) == 1 (see SelfAttention)
            q = q.contiguous()
        k, v = self.to_kv(ctx).chunk(2, dim=-1)
        k = k.reshape(B, -1, h, d).transpose(1, 2)
        v = v.reshape(B, -1, h, d).transpose(1, 2)
        nk, nv = (t.to(q.dtype)[None, :, None, :].expand(B, h, 1, d) for t in self.null_kv.unbind(0))
        k = torch.cat([nk, k.to(q.dtype)], dim=2)
        v = torch.cat([nv, v.to(q.dtype)], dim=2)
        if exists(mask):
            pad = torch.zeros(mask.shape[0], 1, dtype=torch.bool, device=mask.device)
            mask = torch.cat([pad, mask], dim=1)[:, None, None, :].expand(-1, h, q.shape[2], -1)
        out = F.scaled_dot_product_attention(q, k, v, attn_mask=mask)
        out = out.transpose(2, 3).reshape(B, h * d, H * W)
        return _pointwise(self.to_out, out).reshape(B, C, H, W)


class _ChannelFirstFF(nn.Sequential):
    """norm -> 1x1 (dim -> hidden) -> GELU -> 1x1 (hidden -> dim); keys 0..3 as nn.Sequential."""

    def forward(self, x):
        norm, proj1, act, proj2 = self[0], self[1], self[2], self[3]
        if not isinstance(proj1, nn.Conv2d):
            return super().forward(x)
        B, C, H, W = x.shape
        y = _pointwise(proj1, norm(x).reshape(B, C, H * W))
        y = F.gelu(y)
        return _pointwise(proj2, y).reshape(B, C, H, W)


def FeedForward(dim, mult=4, channel_first=False):
    hidden = int(dim * mult)
    if channel_first:
        proj1, proj2 = nn.Conv2d(dim, hidden, 1), nn.Conv2d(hidden, dim, 1)
        nn.init.zeros_(proj2.weight)
        return _ChannelFirstFF(ChannelRMSNorm(dim), proj1, nn.GELU(), proj2)
    proj1, proj2 = nn.Linear(dim, hidden), nn.Linear(hidden, dim)
    nn.init.zeros_(proj2.weight)
    return nn.Sequential(RMSNorm(dim), proj1, nn.GELU(), proj2)


class SelfAttentionBlock(nn.Module):
    def __init__(self, dim, dim_head=64, heads=8, ff_mult=4):
        super().__init__()
        self.attn = SelfAttention(dim=dim, dim_head=dim_head, heads=heads)
        self.ff = FeedForward(dim=dim, mult=ff_mult, channel_first=True)

    def forward(self, x):
        x = self.attn(x) + x
        return self.ff(x) + x


class CrossAttentionBlock(nn.Module):
    def __init__(self, dim, dim_context, dim_head=64, heads=8, ff_mult=4):
        super().__init__()
        self.attn = CrossAttention(dim=dim, dim_context=dim_context, dim_head=dim_head, heads=heads)
        self.ff = FeedForward(dim=dim, mult=ff_mult, channel_first=True)

    def forward(self, x, context, mask=None):
        x = self.attn(x, context=context, mask=mask) + x
        return self.ff(x) + x
