"""Frozen DINOv2 vision tower (config 3 of BASELINE.json: DINOv2-L encoder).

Replaces the reference wrapper `networks/utils/vfms/dinov2_utils.py:33-128`, which loads
`transformers.AutoModel.from_pretrained(name)` (Dinov2Model) and runs it under bf16
autocast. The module tree and state-dict keys are HF Dinov2Model's
(embeddings.{cls_token,mask_token,position_embeddings,patch_embeddings.projection},
encoder.layer.N.{norm1, attention.attention.{query,key,value}, attention.output.dense,
layer_scale1.lambda1, norm2, mlp.{fc1,fc2}, layer_scale2.lambda1}, layernorm), so a local HF
directory (config.json + *.safetensors) loads unchanged; without one the architecture named
by the model string is random-initialised from a fixed seed (no network here).

Layer math = HF Dinov2Layer under autocast(bf16): pre-LN (eps 1e-6, fp32) -> bf16 q/k/v +
SDPA + dense -> x lambda1 -> fp32 residual; LN -> fc1 -> GELU (erf) -> fc2 -> x lambda2 ->
residual; final layernorm. Preprocessing = the reference wrapper's (:77-94): optional
bicubic eq-downscale (antialias), bicubic resize by scale_factor, ImageNet mean/std.
Features: hidden_states[i][:, 1:] for i >= 0, last_hidden_state[:, 1:] for -1 (CLS dropped,
reference :113-121); pooled = last_hidden_state[:, 0].
"""
import re
from typing import List

import torch
import torch.nn as nn
import torch.nn.functional as F

from torch_utils import distributed as dist
from torch_utils.ops import vit_ops
from .vit_tower import Linear, ln, load_safetensors_dir, local_config, mha, resample_positions, seeded_init

_SIZES = {"small": (384, 12, 6, 1536), "base": (768, 12, 12, 3072), "large": (1024, 24, 16, 4096)}


def dinov2_config_from_name(model_name):
    cfg = local_config(model_name)
    if cfg is not None:
        if cfg.get("use_swiglu_ffn", False):
            raise NotImplementedError("DINOv2 SwiGLU FFN (giant) is not part of the MI355X training path")
        return dict(hidden_size=cfg["hidden_size"], num_hidden_layers=cfg["num_hidden_layers"],
                    num_attention_heads=cfg["num_attention_heads"],
                    intermediate_size=int(cfg["hidden_size"] * cfg.get("mlp_ratio", 4)),
                    image_size=cfg.get("image_size", 518), patch_size=cfg.get("patch_size", 14),
                    layer_norm_eps=cfg.get("layer_norm_eps", 1e-6), layerscale_value=cfg.get("layerscale_value", 1.0))
    name = model_name.lower()
    size = next((k for k in _SIZES if k in name), "large")
    if "giant" in name:
        raise NotImplementedError("DINOv2 giant (SwiGLU FFN) is not part of the MI355X training path")
    d, n, h, i = _SIZES[size]
    return dict(hidden_size=d, num_hidden_layers=n, num_attention_heads=h, intermediate_size=i, image_size=518,
                patch_size=14, layer_norm_eps=1e-6, layerscale_value=1.0)


class _PatchEmbeddings(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        p = cfg["patch_size"]
        self.projection = nn.Conv2d(3, cfg["hidden_size"], kernel_size=p, stride=p)


class Dinov2Embeddings(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        d, p = cfg["hidden_size"], cfg["patch_size"]
        n = (cfg["image_size"] // p) ** 2
        self.patch_size = p
        self.cls_token = nn.Parameter(torch.zeros(1, 1, d))
        self.mask_token = nn.Parameter(torch.zeros(1, d))
        self.position_embeddings = nn.Parameter(torch.zeros(1, n + 1, d))
        self.patch_embeddings = _PatchEmbeddings(cfg)

    def forward(self, pixel_values, compute_dtype):
        B, _, H, W = pixel_values.shape
        p = self.patch_size
        proj = self.patch_embeddings.projection
        tok = vit_ops.patch_embed(pixel_values, proj.weight, proj.bias, p, compute_dtype)   # [B, N, D]
        h = torch.cat([self.cls_token.expand(B, -1, -1).float(), tok.float()], 1)
        return h + resample_positions(self.position_embeddings[0], H // p, W // p)


class _SelfAttention(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.query, self.key, self.value = Linear(d, d), Linear(d, d), Linear(d, d)


class _SelfOutput(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.dense = Linear(d, d)


class Dinov2Attention(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.heads = cfg["num_attention_heads"]
        self.attention = _SelfAttention(cfg["hidden_size"])
        self.output = _SelfOutput(cfg["hidden_size"])

    def forward(self, x):
        a, o = self.attention, self.output.dense
        return mha(x, a.query.weight, a.query.bias, a.key.weight, a.key.bias, a.value.weight, a.value.bias,
                   o.weight, o.bias, self.heads, owner=self)


class Dinov2LayerScale(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.lambda1 = nn.Parameter(cfg["layerscale_value"] * torch.ones(cfg["hidden_size"]))


class Dinov2MLP(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.fc1 = Linear(cfg["hidden_size"], cfg["intermediate_size"])
        self.fc2 = Linear(cfg["intermediate_size"], cfg["hidden_size"])

    def forward(self, x):
        # fc1 + erf-GELU in one GEMM epilogue on ROCm (vit_ops.linear_gelu), fc2
        return self.fc2(vit_ops.linear_gelu(x, vit_ops.frozen_weight(self.fc1.weight, x.dtype), self.fc1.bias))


class Dinov2Layer(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        d, eps = cfg["hidden_size"], cfg["layer_norm_eps"]
        self.norm1 = nn.LayerNorm(d, eps=eps)
        self.attention = Dinov2Attention(cfg)
        self.layer_scale1 = Dinov2LayerScale(cfg)
        self.norm2 = nn.LayerNorm(d, eps=eps)
        self.mlp = Dinov2MLP(cfg)
        self.layer_scale2 = Dinov2LayerScale(cfg)

    def forward(self, h, compute_dtype):
        """h: fp32 residual stream. bf16 branch outputs are scaled by lambda in fp32 (type
        promotion under autocast) and added to the fp32 stream."""
        a = self.attention(ln(h, self.norm1, compute_dtype))
        h = h + a.float() * self.layer_scale1.lambda1.float()
        m = self.mlp(ln(h, self.norm2, compute_dtype))
        return h + m.float() * self.layer_scale2.lambda1.float()


class _Encoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.layer = nn.ModuleList([Dinov2Layer(cfg) for _ in range(cfg["num_hidden_layers"])])


class Dinov2Model(nn.Module):
    """HF Dinov2Model-compatible container."""

    def __init__(self, cfg):
        super().__init__()
        self.config = cfg
        self.embeddings = Dinov2Embeddings(cfg)
        self.encoder = _Encoder(cfg)
        self.layernorm = nn.LayerNorm(cfg["hidden_size"], eps=cfg["layer_norm_eps"])

    def reset_parameters(self, seed=1234):
        g = seeded_init(self, seed)
        with torch.no_grad():
            e = self.embeddings
            e.cls_token.copy_(torch.randn(e.cls_token.shape, generator=g) * 0.02)
            e.position_embeddings.copy_(torch.randn(e.position_embeddings.shape, generator=g).clamp_(-2, 2) * 0.02)
            for lyr in self.encoder.layer:
                lyr.layer_scale1.lambda1.fill_(self.config["layerscale_value"])
                lyr.layer_scale2.lambda1.fill_(self.config["layerscale_value"])

    @torch.no_grad()
    def forward_features(self, pixel_values, want: List[int], want_last: bool, compute_dtype):
        """({i: hidden_states[i] fp32 [B, 1+N, D]}, last_hidden_state fp32 | None)."""
        h = self.embeddings(pixel_values, compute_dtype)
        saved = {0: h} if 0 in want else {}
        n = len(self.encoder.layer)
        last_needed = n if want_last else max([i for i in want if i > 0], default=0)
        for i, lyr in enumerate(self.encoder.layer[:last_needed], start=1):
            h = lyr(h, compute_dtype)
            if i in want:
                saved[i] = h
        last = F.layer_norm(h, (h.shape[-1],), self.layernorm.weight, self.layernorm.bias,
                            self.layernorm.eps) if want_last else None
        return saved, last


class DINOv2Encoder(nn.Module):
    """Reference interface: encode_image(img, eq_scale_factor, is_eq_prior) -> (patch_features, pooled)."""

    def __init__(self, model_name="facebook/dinov2-large", scale_factor=1.0, patch_from_layers=(-1,),
                 amp_dtype=torch.bfloat16, amp_enabled=True):
        super().__init__()
        self.model_name = model_name
        self.scale_factor = scale_factor
        self.patch_from_layers = list(patch_from_layers)
        self.amp_dtype = amp_dtype
        self.amp_enabled = amp_enabled
        cfg = dinov2_config_from_name(model_name)
        self.patch_size = cfg["patch_size"]
        self.register_buffer("_mean", torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1), persistent=False)
        self.register_buffer("_std", torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1), persistent=False)
        self.vision_model = Dinov2Model(cfg)
        self.vision_model.reset_parameters()
        loaded = load_safetensors_dir(self.vision_model, model_name,
                                      rename=lambda k: re.sub(r"^(dinov2\.|model\.)", "", k))
        self.vision_model.eval().requires_grad_(False)
        self.pretrained_loaded = loaded
        dist.print0(f"DINOv2Encoder ready: {model_name} ({'pretrained' if loaded else 'random init'}), "
                    f"{cfg['num_hidden_layers']} layers, hidden {cfg['hidden_size']}, patch {self.patch_size}, "
                    f"layers {self.patch_from_layers}, scale_factor {scale_factor}")

    def _preprocess_image(self, img, eq_scale_factor, is_eq_prior):
        if img.dtype == torch.uint8:
            img = img.float() / 255.0
        if is_eq_prior and eq_scale_factor < 1.0:
            img = F.interpolate(img, scale_factor=eq_scale_factor, mode="bicubic", align_corners=False, antialias=True)
        if self.scale_factor != 1.0:
            img = F.interpolate(img, scale_factor=self.scale_factor, mode="bicubic", align_corners=False,
                                antialias=(self.scale_factor < 1.0))
        return (img - self._mean.to(img.device)) / self._std.to(img.device)

    @torch.no_grad()
    def encode_image(self, img, eq_scale_factor=1.0, is_eq_prior=False):
        x = self._preprocess_image(img, eq_scale_factor, is_eq_prior)
        dtype = self.amp_dtype if (self.amp_enabled and x.is_cuda) else torch.float32
        n = len(self.vision_model.encoder.layer)
        idx = [i if i >= 0 else n + i + 2 for i in self.patch_from_layers if i != -1]   # hidden_states[i + 1]
        saved, last = self.vision_model.forward_features(x, idx, want_last=True, compute_dtype=dtype)
        feats = []
        for i in self.patch_from_layers:
            if i == -1:
                feats.append(last[:, 1:].float())
            else:
                feats.append(saved[i if i >= 0 else n + i + 2][:, 1:].float())
        return feats, last[:, 0].float()

    @torch.no_grad()
    def encode_text(self, text):
        return None, None, None
