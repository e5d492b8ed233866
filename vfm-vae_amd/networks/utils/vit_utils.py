"""Frozen ViT backbone for the projected (StyleGAN-T) discriminator.

Replaces the reference's timm `vit_small_patch16_224_dino` + DPT hook
machinery (`networks/utils/vit_utils.py:67-155`, `networks/discriminator.py:145-168`).
The module tree and parameter names follow timm's VisionTransformer
(patch_embed.proj, cls_token, pos_embed, blocks.N.{norm1,attn.qkv,attn.proj,norm2,
mlp.fc1,mlp.fc2}, norm), so `D` checkpoints load; activations are returned
explicitly instead of through global forward hooks (the reference keeps them in
a module-level dict, which is not re-entrant).

Features per hook: tokens after block h (and after pos-drop for the patch hook),
readout-added (x[:, 1:] + x[:, :1]) and transposed to [B, D, N] (AddReadout +
Transpose of the reference, start_index 1).
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from torch_utils.ops import vit_ops


class PatchEmbed(nn.Module):
    def __init__(self, img_size=224, patch_size=16, in_chans=3, embed_dim=384):
        super().__init__()
        self.img_size = (img_size, img_size)
        self.patch_size = (patch_size, patch_size)
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)


class Attention(nn.Module):
    def __init__(self, dim, num_heads):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.qkv = nn.Linear(dim, dim * 3, bias=True)
        self.proj = nn.Linear(dim, dim)

    def forward(self, x):
        B, N, D = x.shape
        qkv = vit_ops.linear(x, self.qkv.weight.to(x.dtype), self.qkv.bias)
        o = vit_ops.sdpa_packed(qkv, self.num_heads).transpose(1, 2).reshape(B, N, D)
        return vit_ops.linear(o, self.proj.weight.to(x.dtype), self.proj.bias)


class Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)

    def forward(self, x):
        h = F.gelu(vit_ops.linear(x, self.fc1.weight.to(x.dtype), self.fc1.bias))
        return vit_ops.linear(h, self.fc2.weight.to(x.dtype), self.fc2.bias)


class Block(nn.Module):
    def __init__(self, dim, num_heads, mlp_ratio=4.0):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = Attention(dim, num_heads)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = Mlp(dim, int(dim * mlp_ratio))

    def forward(self, x):
        x = x + self.attn(_norm(self.norm1, x))
        return x + self.mlp(_norm(self.norm2, x))


def _norm(ln, x):
    """nn.LayerNorm(x); on ROCm fp32 with frozen parameters (the DINO discriminator backbone) the native
    LayerNorm with an input gradient (csrc/vit.hip ln2_fwd / ln2_bwd) instead of torch's two kernels."""
    if x.is_cuda and x.dtype == torch.float32:
        from torch_utils.ops import vit_hip
        if vit_hip.LN_GRAD and vit_hip.layer_norm_grad_supported(x, ln):
            return vit_hip.layer_norm_grad(x, ln, torch.float32)
    return ln(x)


class VisionTransformer(nn.Module):
    """timm-layout ViT with a class token; forward_flex resizes the position grid."""

    def __init__(self, img_size=224, patch_size=16, embed_dim=384, depth=12, num_heads=6, mlp_ratio=4.0):
        super().__init__()
        self.embed_dim = embed_dim
        self.patch_embed = PatchEmbed(img_size, patch_size, 3, embed_dim)
        n = (img_size // patch_size) ** 2
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, n + 1, embed_dim))
        self.pos_drop = nn.Identity()
        self.blocks = nn.ModuleList([Block(embed_dim, num_heads, mlp_ratio) for _ in range(depth)])
        self.norm = nn.LayerNorm(embed_dim, eps=1e-6)
        self.start_index = 1
        self.patch_size = [patch_size, patch_size]

    def reset_parameters(self, seed=4321):
        g = torch.Generator().manual_seed(seed)
        with torch.no_grad():
            for m in self.modules():
                if isinstance(m, nn.Linear):
                    m.weight.copy_(torch.randn(m.weight.shape, generator=g).clamp_(-2, 2) * 0.02)
                    nn.init.zeros_(m.bias)
                elif isinstance(m, nn.LayerNorm):
                    nn.init.ones_(m.weight)
                    nn.init.zeros_(m.bias)
            fan_in = 3 * self.patch_size[0] * self.patch_size[1]
            self.patch_embed.proj.weight.copy_(torch.randn(self.patch_embed.proj.weight.shape, generator=g) / math.sqrt(fan_in))
            self.patch_embed.proj.bias.zero_()
            self.pos_embed.copy_(torch.randn(self.pos_embed.shape, generator=g).clamp_(-2, 2) * 0.02)
            self.cls_token.copy_(torch.randn(self.cls_token.shape, generator=g) * 1e-6)

    def _resize_pos_embed(self, posemb, gs_h, gs_w):
        tok, grid = posemb[:, :self.start_index], posemb[0, self.start_index:]
        old = int(math.sqrt(grid.shape[0]))
        if (gs_h, gs_w) == (old, old):
            return posemb
        grid = grid.reshape(1, old, old, -1).permute(0, 3, 1, 2)
        grid = F.interpolate(grid, size=(gs_h, gs_w), mode="bilinear", align_corners=False)
        grid = grid.permute(0, 2, 3, 1).reshape(1, gs_h * gs_w, -1)
        return torch.cat([tok, grid], dim=1)

    def forward_flex(self, x, hooks, hook_patch=True):
        """Run the ViT; return {str(i): tokens after blocks[hooks[i]]} (+ patch hook)."""
        B, C, H, W = x.shape
        p = self.patch_size[0]
        tokens = vit_ops.patch_embed(x, self.patch_embed.proj.weight, self.patch_embed.proj.bias, p, x.dtype)
        pos = self._resize_pos_embed(self.pos_embed, H // p, W // p)
        h = torch.cat([self.cls_token.expand(B, -1, -1).to(tokens.dtype), tokens], dim=1) + pos.to(tokens.dtype)
        h = self.pos_drop(h)
        acts = {}
        if hook_patch:
            acts[str(len(hooks))] = h
        last = max(hooks)
        for i, blk in enumerate(self.blocks):
            if i > last:
                break        # later blocks (and the final norm) feed no hook
            h = blk(h)
            if i in hooks:
                acts[str(hooks.index(i))] = h
        return acts


def readout_transpose(x, start_index=1):
    """AddReadout(start_index) + Transpose(1, 2)."""
    if start_index == 2:
        readout = (x[:, 0] + x[:, 1]) / 2
    else:
        readout = x[:, 0]
    return (x[:, start_index:] + readout.unsqueeze(1)).transpose(1, 2).contiguous()


class ViTBackbone(nn.Module):
    """Container matching the reference's `pretrained` module (attribute `.model`)."""

    def __init__(self, model: VisionTransformer, hooks=(2, 5, 8, 11), hook_patch=True):
        super().__init__()
        assert len(hooks) == 4 and list(hooks) == sorted(hooks)
        self.model = model
        self.hooks = list(hooks)
        self.hook_patch = hook_patch


def make_vit_backbone(model, patch_size=(16, 16), hooks=(2, 5, 8, 11), hook_patch=True, start_index=1):
    model.start_index = start_index
    model.patch_size = list(patch_size)
    return ViTBackbone(model, hooks, hook_patch)


def forward_vit(pretrained: ViTBackbone, x):
    acts = pretrained.model.forward_flex(x, pretrained.hooks, pretrained.hook_patch)
    return {k: readout_transpose(v, pretrained.model.start_index) for k, v in acts.items()}
