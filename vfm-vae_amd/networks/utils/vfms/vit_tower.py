"""Shared pieces of the frozen ViT encoder towers (DINOv2, CLIP): local HF config /
safetensors loading, bicubic position-grid resampling (HF `interpolate_pos_encoding`),
and a bf16-GEMM multi-head self-attention over the fp32 residual stream.
"""
import json
import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from torch_utils.ops import vit_ops


def local_config(model_name):
    """config.json of a local HF directory (vision_config if nested), else None."""
    p = os.path.join(model_name, "config.json")
    if os.path.isdir(model_name) and os.path.exists(p):
        cfg = json.load(open(p))
        return cfg.get("vision_config", cfg)
    return None


def load_safetensors_dir(module, path, rename=None):
    """Load every *.safetensors of a local HF directory into `module` (strict on the
    module's own keys except the non-persistent ones). Returns False if none exist."""
    files = sorted(f for f in os.listdir(path) if f.endswith(".safetensors")) if os.path.isdir(path) else []
    if not files:
        return False
    from safetensors.torch import load_file
    state = {}
    for f in files:
        for k, v in load_file(os.path.join(path, f)).items():
            k = rename(k) if rename else k
            if k is not None:
                state[k] = v
    missing, _ = module.load_state_dict(state, strict=False)
    missing = [k for k in missing if not k.endswith("position_ids")]
    if missing:
        raise RuntimeError(f"checkpoint {path} is missing {len(missing)} tensors, e.g. {missing[:3]}")
    return True


def resample_positions(pos, gh, gw):
    """pos: [1 + n*n, D] (CLS first) -> [1, 1 + gh*gw, D] fp32, bicubic on the patch grid
    (align_corners=False), HF interpolate_pos_encoding semantics."""
    n = pos.shape[0] - 1
    side = int(math.isqrt(n))
    if gh * gw == n and gh == gw:
        return pos[None].float()
    cls, grid = pos[:1].float(), pos[1:].float()
    grid = grid.reshape(1, side, side, -1).permute(0, 3, 1, 2)
    grid = F.interpolate(grid, size=(gh, gw), mode="bicubic", align_corners=False)
    grid = grid.permute(0, 2, 3, 1).reshape(gh * gw, -1)
    return torch.cat([cls, grid], 0)[None]


def fused_qkv(owner, wq, bq, wk, bk, wv, bv, dtype):
    """The concatenated [3D, D] qkv weight in the compute dtype and the [3D] bias, cached on `owner` (the frozen
    tower's attention module) until a tensor's storage or version moves: built once, not at every forward."""
    ts = (wq, wk, wv, bq, bk, bv)
    key = (dtype,) + tuple((t.data_ptr(), t._version) if t is not None else None for t in ts)
    capturing = wq.is_cuda and torch.cuda.is_current_stream_capturing()
    hit = getattr(owner, "_vfm_qkv", None) if owner is not None else None
    if hit is not None and hit[0] == key and not capturing:
        return hit[1]
    w = torch.cat([wq, wk, wv], 0).to(dtype)
    b = torch.cat([bq, bk, bv], 0) if bq is not None else None
    if owner is not None and not torch.is_grad_enabled() and not capturing:
        owner._vfm_qkv = (key, (w, b))
    return w, b


def mha(x, wq, bq, wk, bk, wv, bv, wo, bo, heads, owner=None):
    """Self-attention of the compute-dtype tokens x [B, N, D] -> [B, N, D] (compute dtype):
    fused qkv GEMM (weights concatenated once per version, `fused_qkv`), SDPA, output projection."""
    B, N, D = x.shape
    w, b = fused_qkv(owner, wq, bq, wk, bk, wv, bv, x.dtype)
    qkv = vit_ops.linear(x, w, b)
    o = vit_ops.attention_packed(qkv, heads)
    return vit_ops.linear(o, vit_ops.frozen_weight(wo, x.dtype), bo)


def ln(h, norm, dtype):
    return vit_ops.layer_norm(h, norm, dtype)


class Linear(nn.Linear):
    """nn.Linear whose forward runs in the input's (compute) dtype."""

    def forward(self, x):
        return vit_ops.linear(x, vit_ops.frozen_weight(self.weight, x.dtype), self.bias)


def seeded_init(module, seed, std=0.02):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for m in module.modules():
            if isinstance(m, nn.Linear):
                m.weight.copy_(torch.randn(m.weight.shape, generator=g).clamp_(-2, 2) * std)
                if m.bias is not None:
                    m.bias.zero_()
            elif isinstance(m, nn.LayerNorm):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Conv2d):
                fan_in = m.in_channels * m.kernel_size[0] * m.kernel_size[1]
                m.weight.copy_(torch.randn(m.weight.shape, generator=g) / math.sqrt(fan_in))
                if m.bias is not None:
                    m.bias.zero_()
    return g
