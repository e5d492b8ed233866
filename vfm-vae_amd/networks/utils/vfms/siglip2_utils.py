"""Frozen SigLIP2 vision tower used as the VFM-VAE encoder.

Replaces the reference wrapper `networks/utils/vfms/siglip2_utils.py:43-164`,
which loads `transformers.SiglipVisionModel.from_pretrained(name)` and runs it
under bf16 autocast. Here the tower is a native module with the SAME module
tree and state-dict keys as HF `SiglipVisionModel` (vision_model.embeddings.*,
vision_model.encoder.layers.N.{layer_norm1,self_attn.{q,k,v,out}_proj,
layer_norm2,mlp.fc1,mlp.fc2}, vision_model.post_layernorm, vision_model.head.*),
so a local HF checkpoint directory (config.json + *.safetensors) loads
unchanged; without one (no network here) the architecture named by the model
string is random-initialised from a fixed seed.

Layer math follows HF `SiglipEncoderLayer` (transformers, reference pin 4.50.1):
pre-LN (eps 1e-6) -> q/k/v (bias) -> softmax(QK^T/sqrt(d)) V -> out_proj ->
residual; LN -> fc1 -> gelu(tanh) -> fc2 -> residual; post-LN. Mixed precision
mirrors autocast(bf16): GEMMs and attention in bf16, LayerNorm and the residual
stream in fp32. q/k/v are fused into one GEMM.
"""
import json
import math
import os
import re
from typing import List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from torch_utils import distributed as dist
from torch_utils.ops import vit_ops

__all__ = ["SigLIP2Encoder", "SiglipVisionModel", "siglip_config_from_name"]

_SIZES = {  # hidden, layers, heads, intermediate
    "base": (768, 12, 12, 3072),
    "large": (1024, 24, 16, 4096),
    "so400m": (1152, 27, 16, 4304),
    "giant": (1536, 40, 16, 6144),
}


def _infer_patch_size(model_name: str, default: int = 16) -> int:
    m = re.search(r"patch(\d+)", os.path.basename(model_name.rstrip("/")).lower())
    return int(m.group(1)) if m else default


def siglip_config_from_name(model_name: str) -> dict:
    """Architecture from a local config.json, else from the HF naming convention
    ('siglip2-large-patch16-512' -> hidden 1024, 24 layers, 16 heads, 512 px)."""
    cfg_path = os.path.join(model_name, "config.json")
    if os.path.isdir(model_name) and os.path.exists(cfg_path):
        cfg = json.load(open(cfg_path))
        cfg = cfg.get("vision_config", cfg)
        return dict(hidden_size=cfg["hidden_size"], num_hidden_layers=cfg["num_hidden_layers"],
                    num_attention_heads=cfg["num_attention_heads"], intermediate_size=cfg["intermediate_size"],
                    image_size=cfg.get("image_size", 224), patch_size=cfg.get("patch_size", 16),
                    num_channels=cfg.get("num_channels", 3), layer_norm_eps=cfg.get("layer_norm_eps", 1e-6),
                    vision_use_head=cfg.get("vision_use_head", True))
    name = os.path.basename(model_name.rstrip("/")).lower()
    size = next((k for k in _SIZES if k in name), "large")
    hidden, layers, heads, inter = _SIZES[size]
    m = re.search(r"patch\d+-(\d+)", name)
    image_size = int(m.group(1)) if m else 256
    return dict(hidden_size=hidden, num_hidden_layers=layers, num_attention_heads=heads, intermediate_size=inter,
                image_size=image_size, patch_size=_infer_patch_size(model_name), num_channels=3,
                layer_norm_eps=1e-6, vision_use_head=True)


class SiglipVisionEmbeddings(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.embed_dim = cfg["hidden_size"]
        self.image_size = cfg["image_size"]
        self.patch_size = cfg["patch_size"]
        self.patch_embedding = nn.Conv2d(cfg["num_channels"], self.embed_dim, kernel_size=self.patch_size,
                                         stride=self.patch_size, padding="valid")
        self.num_patches = (self.image_size // self.patch_size) ** 2
        self.num_positions = self.num_patches
        self.position_embedding = nn.Embedding(self.num_positions, self.embed_dim)
        self.register_buffer("position_ids", torch.arange(self.num_positions).expand((1, -1)), persistent=False)

    def positions(self, gh: int, gw: int) -> torch.Tensor:
        """[1, gh*gw, D] fp32 position embeddings, bicubic-resampled when the grid
        differs from the trained one (HF interpolate_pos_encoding)."""
        pos = self.position_embedding.weight
        if gh * gw == self.num_positions and gh == gw:
            return pos[None].float()
        side = int(math.sqrt(self.num_positions))
        grid = pos.float().reshape(1, side, side, -1).permute(0, 3, 1, 2)
        grid = F.interpolate(grid, size=(gh, gw), mode="bicubic", align_corners=False)
        return grid.permute(0, 2, 3, 1).reshape(1, gh * gw, -1)

    def forward(self, pixel_values, compute_dtype=torch.bfloat16):
        B, C, H, W = pixel_values.shape
        p = self.patch_size
        gh, gw = H // p, W // p
        tokens = vit_ops.patch_embed(pixel_values, self.patch_embedding.weight, self.patch_embedding.bias, p,
                                     compute_dtype)                       # [B, gh*gw, D]
        return tokens.float() + self.positions(gh, gw)


class SiglipAttention(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.embed_dim = cfg["hidden_size"]
        self.num_heads = cfg["num_attention_heads"]
        self.head_dim = self.embed_dim // self.num_heads
        self.scale = self.head_dim ** -0.5
        self.k_proj = nn.Linear(self.embed_dim, self.embed_dim)
        self.v_proj = nn.Linear(self.embed_dim, self.embed_dim)
        self.q_proj = nn.Linear(self.embed_dim, self.embed_dim)
        self.out_proj = nn.Linear(self.embed_dim, self.embed_dim)
        self._fused = None

    def fused_qkv(self, dtype):
        key = (dtype, self.q_proj.weight.data_ptr(), self.q_proj.weight._version)
        if self._fused is None or self._fused[0] != key:
            w = torch.cat([self.q_proj.weight, self.k_proj.weight, self.v_proj.weight], 0).detach().to(dtype)
            b = torch.cat([self.q_proj.bias, self.k_proj.bias, self.v_proj.bias], 0).detach().float()
            self._fused = (key, w, b)
        return self._fused[1], self._fused[2]

    def forward(self, x):
        """x: [B, N, D] in compute dtype -> [B, N, D] compute dtype."""
        B, N, D = x.shape
        w, b = self.fused_qkv(x.dtype)
        qkv = vit_ops.linear(x, w, b)                                         # [B, N, 3D]
        o = vit_ops.attention_packed(qkv, self.num_heads)                     # [B, N, D]
        return vit_ops.linear(o, vit_ops.frozen_weight(self.out_proj.weight, x.dtype), self.out_proj.bias)


class SiglipMLP(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.fc1 = nn.Linear(cfg["hidden_size"], cfg["intermediate_size"])
        self.fc2 = nn.Linear(cfg["intermediate_size"], cfg["hidden_size"])

    def forward(self, x):
        h = vit_ops.linear_gelu_tanh(x, vit_ops.frozen_weight(self.fc1.weight, x.dtype), self.fc1.bias)
        return vit_ops.linear(h, vit_ops.frozen_weight(self.fc2.weight, x.dtype), self.fc2.bias)


class SiglipEncoderLayer(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        d, eps = cfg["hidden_size"], cfg["layer_norm_eps"]
        self.layer_norm1 = nn.LayerNorm(d, eps=eps)
        self.self_attn = SiglipAttention(cfg)
        self.layer_norm2 = nn.LayerNorm(d, eps=eps)
        self.mlp = SiglipMLP(cfg)

    def forward(self, h, compute_dtype=torch.bfloat16):
        """h: fp32 residual stream [B, N, D]."""
        a = self.self_attn(vit_ops.layer_norm(h, self.layer_norm1, compute_dtype))
        h = vit_ops.residual_add(h, a)
        m = self.mlp(vit_ops.layer_norm(h, self.layer_norm2, compute_dtype))
        return vit_ops.residual_add(h, m)

    def forward_chained(self, h, y1, next_ln, next_dtype, compute_dtype=torch.bfloat16):
        """Same math as forward() with the LayerNorms fused into the residual adds:
        y1 = layer_norm1(h) (computed by the caller), returns (h_out, next_ln(h_out))
        (next_ln None -> (h_out, None))."""
        a = self.self_attn(y1)
        h, y2 = vit_ops.residual_layer_norm(h, a, self.layer_norm2, compute_dtype)
        m = self.mlp(y2)
        if next_ln is None:
            return vit_ops.residual_add(h, m), None
        return vit_ops.residual_layer_norm(h, m, next_ln, next_dtype)


class SiglipEncoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.layers = nn.ModuleList([SiglipEncoderLayer(cfg) for _ in range(cfg["num_hidden_layers"])])


class SiglipMultiheadAttentionPoolingHead(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        d = cfg["hidden_size"]
        self.probe = nn.Parameter(torch.randn(1, 1, d))
        self.attention = nn.MultiheadAttention(d, cfg["num_attention_heads"], batch_first=True)
        self.layernorm = nn.LayerNorm(d, eps=cfg["layer_norm_eps"])
        self.mlp = SiglipMLP(cfg)

    def forward(self, h):
        probe = self.probe.expand(h.shape[0], 1, -1).to(h.dtype)
        x = self.attention(probe, h, h, need_weights=False)[0]
        y = self.layernorm(x)
        y = self.mlp.fc2(F.gelu(self.mlp.fc1(y), approximate="tanh"))
        return (x + y)[:, 0]


class SiglipVisionTransformer(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.config = cfg
        self.embeddings = SiglipVisionEmbeddings(cfg)
        self.encoder = SiglipEncoder(cfg)
        self.post_layernorm = nn.LayerNorm(cfg["hidden_size"], eps=cfg["layer_norm_eps"])
        self.use_head = cfg.get("vision_use_head", True)
        if self.use_head:
            self.head = SiglipMultiheadAttentionPoolingHead(cfg)


def _accept_flat_layout(state_dict, prefix, *args):
    for k in list(state_dict.keys()):
        if k.startswith(prefix) and k[len(prefix):].split('.')[0] in ('embeddings', 'encoder', 'post_layernorm', 'head'):
            state_dict[prefix + 'vision_model.' + k[len(prefix):]] = state_dict.pop(k)


class SiglipVisionModel(nn.Module):
    """HF-compatible container: `.vision_model` holds the transformer."""

    def __init__(self, cfg):
        super().__init__()
        self.config = cfg
        self.vision_model = SiglipVisionTransformer(cfg)
        # transformers >= 5 flattens SiglipVisionModel (keys `embeddings.*` instead of
        # `vision_model.embeddings.*`); accept both layouts when loading.
        self._register_load_state_dict_pre_hook(_accept_flat_layout)

    def reset_parameters(self, seed: int = 1234):
        """Deterministic random init in the spirit of HF SiglipPreTrainedModel._init_weights."""
        g = torch.Generator().manual_seed(seed)
        d = self.config["hidden_size"]
        for name, mod in self.named_modules():
            if isinstance(mod, nn.Linear):
                bound = math.sqrt(6.0 / (mod.in_features + mod.out_features))
                with torch.no_grad():
                    mod.weight.copy_(torch.rand(mod.weight.shape, generator=g) * 2 * bound - bound)
                    if mod.bias is not None:
                        mod.bias.copy_(torch.randn(mod.bias.shape, generator=g) * 1e-6)
            elif isinstance(mod, nn.LayerNorm):
                nn.init.ones_(mod.weight)
                nn.init.zeros_(mod.bias)
        with torch.no_grad():
            emb = self.vision_model.embeddings
            fan_in = emb.patch_embedding.in_channels * emb.patch_size ** 2
            emb.patch_embedding.weight.copy_(torch.randn(emb.patch_embedding.weight.shape, generator=g) / math.sqrt(fan_in))
            emb.patch_embedding.bias.zero_()
            emb.position_embedding.weight.copy_(torch.randn(emb.position_embedding.weight.shape, generator=g) / math.sqrt(d))
            if self.vision_model.use_head:
                head = self.vision_model.head
                head.probe.copy_(torch.randn(head.probe.shape, generator=g) * math.sqrt(2.0 / (1 + d)))
                bound = math.sqrt(6.0 / (d + 3 * d))
                head.attention.in_proj_weight.copy_(torch.rand(head.attention.in_proj_weight.shape, generator=g) * 2 * bound - bound)
                head.attention.in_proj_bias.zero_()

    def load_hf_checkpoint(self, path: str) -> bool:
        """Load *.safetensors from a local HF directory (full SigLIP or vision-only)."""
        files = sorted(f for f in os.listdir(path) if f.endswith(".safetensors")) if os.path.isdir(path) else []
        if not files:
            return False
        from safetensors.torch import load_file
        state = {}
        for f in files:
            for k, v in load_file(os.path.join(path, f)).items():
                if k.startswith("vision_model.") or k.split(".")[0] in ("embeddings", "encoder", "post_layernorm", "head"):
                    state[k] = v
                elif k.startswith("model.vision_model."):
                    state[k[len("model."):]] = v
        missing, unexpected = self.load_state_dict(state, strict=False)
        missing = [k for k in missing if not k.endswith("position_ids")]
        if missing:
            raise RuntimeError(f"SigLIP checkpoint {path} is missing {len(missing)} tensors, e.g. {missing[:3]}")
        return True

    @torch.no_grad()
    def forward_features(self, pixel_values, hidden_state_indices: List[int], want_last: bool, want_pooled: bool,
                         compute_dtype=torch.bfloat16) -> Tuple[dict, Optional[torch.Tensor], Optional[torch.Tensor]]:
        """Returns ({i: hidden_states[i] fp32}, last_hidden_state fp32 | None, pooled | None).
        hidden_states[0] = embeddings, hidden_states[i] = output of layer i."""
        vm = self.vision_model
        h = vm.embeddings(pixel_values, compute_dtype)
        want = set(hidden_state_indices)
        saved = {0: h} if 0 in want else {}
        n_layers = len(vm.encoder.layers)
        last_needed = n_layers if (want_last or want_pooled) else max([i for i in want if i > 0], default=0)
        layers = vm.encoder.layers[:last_needed]
        last = pooled = None
        if layers:
            # each layer's input LayerNorm is fused into the previous residual add; the last
            # one's into post_layernorm (fp32 out, as LayerNorm under autocast)
            y = vit_ops.layer_norm(h, layers[0].layer_norm1, compute_dtype)
            for i, layer in enumerate(layers, start=1):
                if i < len(layers):
                    nxt, ndt = layers[i].layer_norm1, compute_dtype
                elif want_last or want_pooled:
                    nxt, ndt = vm.post_layernorm, torch.float32
                else:
                    nxt, ndt = None, None
                h, y = layer.forward_chained(h, y, nxt, ndt, compute_dtype)
                if i in want:
                    saved[i] = h
            if want_last or want_pooled:
                last = y
        if want_pooled and vm.use_head:
            pooled = vm.head(last).float()
        return saved, last, pooled


class SigLIP2Encoder(nn.Module):
    """Wrapper with the reference interface: `encode_image(img, eq_scale_factor,
    is_eq_prior) -> (patch_features, pooled)` and `encode_text(text)`."""

    def __init__(self, model_name, conditional, label_type, scale_factor, patch_from_layers,
                 amp_dtype=torch.bfloat16, amp_enabled=True, compute_pooled=False):
        super().__init__()
        self.model_name = model_name
        self.conditional = conditional
        self.label_type = label_type
        self.scale_factor = scale_factor
        self.patch_from_layers = patch_from_layers
        self.amp_dtype = amp_dtype
        self.amp_enabled = amp_enabled
        self.compute_pooled = compute_pooled
        self.patch_size = _infer_patch_size(model_name, default=16)
        self.register_buffer("_mean", torch.tensor([0.5, 0.5, 0.5]).view(1, 3, 1, 1), persistent=False)
        self.register_buffer("_std", torch.tensor([0.5, 0.5, 0.5]).view(1, 3, 1, 1), persistent=False)

        cfg = siglip_config_from_name(model_name)
        self.patch_size = cfg["patch_size"]
        self.vision_model = SiglipVisionModel(cfg)
        self.vision_model.reset_parameters()
        loaded = self.vision_model.load_hf_checkpoint(model_name)
        self.vision_model.eval().requires_grad_(False)
        self.pretrained_loaded = loaded

        if conditional and label_type in ["text", "cls2text"]:
            raise NotImplementedError("SigLIP2 text conditioning needs the HF text tower and tokenizer, "
                                      "which are not part of the MI355X training path")
        self.tokenizer = None
        self.text_model = None
        self.use_text = False
        n = cfg["num_hidden_layers"]
        dist.print0(f"SigLIP2Encoder ready: {model_name} ({'pretrained' if loaded else 'random init'}), "
                    f"{n} layers, hidden {cfg['hidden_size']}, patch {self.patch_size}, "
                    f"layers {patch_from_layers}, scale_factor {scale_factor}")

    def _preprocess_image(self, img, eq_scale_factor, is_eq_prior):
        if img.dtype == torch.uint8:
            img = img.float() / 255.0
        if is_eq_prior and eq_scale_factor < 1.0:
            img = F.interpolate(img, scale_factor=eq_scale_factor, mode="bilinear", align_corners=False, antialias=True)
        if self.scale_factor != 1.0:
            img = F.interpolate(img, scale_factor=self.scale_factor, mode="bilinear", align_corners=False,
                                antialias=(self.scale_factor < 1.0))
        return (img - self._mean.to(img.device)) / self._std.to(img.device)

    @torch.no_grad()
    def encode_image(self, img, eq_scale_factor, is_eq_prior):
        x = self._preprocess_image(img, eq_scale_factor, is_eq_prior)
        n = len(self.vision_model.vision_model.encoder.layers)
        idx = []
        for i in self.patch_from_layers:
            if i >= 0:
                idx.append(i)
            elif i < -1:
                idx.append(n + i + 2)   # hidden_states[i+1]: -2 -> last block output (before post-LN)
        dtype = self.amp_dtype if (self.amp_enabled and x.is_cuda) else torch.float32
        saved, last, pooled = self.vision_model.forward_features(
            x, idx, want_last=(-1 in self.patch_from_layers), want_pooled=self.compute_pooled, compute_dtype=dtype)
        feats = []
        for i in self.patch_from_layers:
            if i == -1:
                feats.append(last.float())
            elif i >= 0:
                feats.append(saved[i].float())
            else:
                feats.append(saved[n + i + 2].float())
        return feats, pooled

    @torch.no_grad()
    def encode_text(self, text):
        return None, None, None
