"""Frozen CLIP vision tower (config 0 of BASELINE.json: f16d32 stage 0 with a CLIP ViT-B/16
encoder, bs=1 CPU reconstruction).

The reference lists CLIP only as "not supported yet" as an encoder
(`networks/utils/vfms/clip_utils.py:2`; `vfm_utils.py:64-109` dispatches qwen/siglip2/
dinov2/mae/eva), so this backend is an addition of the build. Module tree
and state-dict keys are HF CLIPVisionModel's (vision_model.embeddings.{class_embedding,
patch_embedding,position_embedding}, vision_model.pre_layrnorm, vision_model.encoder.layers.N.
{layer_norm1, self_attn.{q,k,v,out}_proj, layer_norm2, mlp.{fc1,fc2}},
vision_model.post_layernorm), so a local HF directory loads unchanged; otherwise seeded
random init of the named architecture.

Layer math = HF CLIPEncoderLayer under autocast(bf16): pre-LN (eps 1e-5) -> bf16 attention ->
fp32 residual; LN -> fc1 -> quick_gelu -> fc2 -> residual. Preprocessing as the other
backends (optional eq-downscale, resize by scale_factor, bicubic) with the OpenAI CLIP
mean/std. Feature indices follow vfm_utils: 0 = embeddings (after pre_layrnorm), i = output
of layer i, -1 = final sequence after post_layernorm, -k = hidden_states[-k+1]; CLS dropped.
"""
import re

import torch
import torch.nn as nn
import torch.nn.functional as F

from torch_utils import distributed as dist
from torch_utils.ops import vit_ops
from .vit_tower import Linear, ln, load_safetensors_dir, local_config, mha, resample_positions, seeded_init

_ARCH = {"base": (768, 12, 12, 3072), "large": (1024, 24, 16, 4096)}


def clip_config_from_name(model_name):
    cfg = local_config(model_name)
    if cfg is not None:
        return dict(hidden_size=cfg["hidden_size"], num_hidden_layers=cfg["num_hidden_layers"],
                    num_attention_heads=cfg["num_attention_heads"], intermediate_size=cfg["intermediate_size"],
                    image_size=cfg.get("image_size", 224), patch_size=cfg.get("patch_size", 32),
                    layer_norm_eps=cfg.get("layer_norm_eps", 1e-5), hidden_act=cfg.get("hidden_act", "quick_gelu"))
    name = model_name.lower()
    size = "large" if "large" in name else "base"
    d, n, h, i = _ARCH[size]
    m = re.search(r"patch(\d+)", name)
    p = int(m.group(1)) if m else 16
    m = re.search(r"patch\d+-(\d+)", name)
    return dict(hidden_size=d, num_hidden_layers=n, num_attention_heads=h, intermediate_size=i,
                image_size=int(m.group(1)) if m else 224, patch_size=p, layer_norm_eps=1e-5, hidden_act="quick_gelu")


def _act(x, name):
    if name == "quick_gelu":
        return x * torch.sigmoid(1.702 * x)
    if name == "gelu":
        return F.gelu(x)
    raise NotImplementedError(name)


class CLIPVisionEmbeddings(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        d, p = cfg["hidden_size"], cfg["patch_size"]
        self.patch_size = p
        self.class_embedding = nn.Parameter(torch.zeros(d))
        self.patch_embedding = nn.Conv2d(3, d, kernel_size=p, stride=p, bias=False)
        self.position_embedding = nn.Embedding((cfg["image_size"] // p) ** 2 + 1, d)

    def forward(self, pixel_values, compute_dtype):
        B, _, H, W = pixel_values.shape
        p = self.patch_size
        tok = vit_ops.patch_embed(pixel_values, self.patch_embedding.weight, None, p, compute_dtype)
        h = torch.cat([self.class_embedding.float()[None, None].expand(B, 1, -1), tok.float()], 1)
        return h + resample_positions(self.position_embedding.weight, H // p, W // p)


class CLIPAttention(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        d = cfg["hidden_size"]
        self.heads = cfg["num_attention_heads"]
        self.k_proj, self.v_proj, self.q_proj, self.out_proj = Linear(d, d), Linear(d, d), Linear(d, d), Linear(d, d)

    def forward(self, x):
        return mha(x, self.q_proj.weight, self.q_proj.bias, self.k_proj.weight, self.k_proj.bias,
                   self.v_proj.weight, self.v_proj.bias, self.out_proj.weight, self.out_proj.bias, self.heads, owner=self)


class CLIPMLP(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.act = cfg["hidden_act"]
        self.fc1 = Linear(cfg["hidden_size"], cfg["intermediate_size"])
        self.fc2 = Linear(cfg["intermediate_size"], cfg["hidden_size"])

    def forward(self, x):
        return self.fc2(_act(self.fc1(x), self.act))


class CLIPEncoderLayer(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        d, eps = cfg["hidden_size"], cfg["layer_norm_eps"]
        self.self_attn = CLIPAttention(cfg)
        self.layer_norm1 = nn.LayerNorm(d, eps=eps)
        self.mlp = CLIPMLP(cfg)
        self.layer_norm2 = nn.LayerNorm(d, eps=eps)

    def forward(self, h, compute_dtype):
        h = vit_ops.residual_add(h, self.self_attn(ln(h, self.layer_norm1, compute_dtype)))
        return vit_ops.residual_add(h, self.mlp(ln(h, self.layer_norm2, compute_dtype)))


class _Encoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.layers = nn.ModuleList([CLIPEncoderLayer(cfg) for _ in range(cfg["num_hidden_layers"])])


class CLIPVisionTransformer(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        d, eps = cfg["hidden_size"], cfg["layer_norm_eps"]
        self.embeddings = CLIPVisionEmbeddings(cfg)
        self.pre_layrnorm = nn.LayerNorm(d, eps=eps)
        self.encoder = _Encoder(cfg)
        self.post_layernorm = nn.LayerNorm(d, eps=eps)


class CLIPVisionModel(nn.Module):
    """HF CLIPVisionModel-compatible container (`.vision_model`)."""

    def __init__(self, cfg):
        super().__init__()
        self.config = cfg
        self.vision_model = CLIPVisionTransformer(cfg)

    def reset_parameters(self, seed=1234):
        g = seeded_init(self, seed)
        with torch.no_grad():
            e = self.vision_model.embeddings
            e.class_embedding.copy_(torch.randn(e.class_embedding.shape, generator=g) * 0.02)
            e.position_embedding.weight.copy_(torch.randn(e.position_embedding.weight.shape, generator=g) * 0.02)

    @torch.no_grad()
    def forward_features(self, pixel_values, want, want_last, compute_dtype):
        vm = self.vision_model
        h = vm.embeddings(pixel_values, compute_dtype)
        h = F.layer_norm(h, (h.shape[-1],), vm.pre_layrnorm.weight, vm.pre_layrnorm.bias, vm.pre_layrnorm.eps)
        saved = {0: h} if 0 in want else {}
        n = len(vm.encoder.layers)
        last_needed = n if want_last else max([i for i in want if i > 0], default=0)
        for i, lyr in enumerate(vm.encoder.layers[:last_needed], start=1):
            h = lyr(h, compute_dtype)
            if i in want:
                saved[i] = h
        last = F.layer_norm(h, (h.shape[-1],), vm.post_layernorm.weight, vm.post_layernorm.bias,
                            vm.post_layernorm.eps) if want_last else None
        return saved, last


class CLIPVisionEncoder(nn.Module):
    """Reference-style interface: encode_image(img, eq_scale_factor, is_eq_prior) -> (feats, pooled)."""

    def __init__(self, model_name="openai/clip-vit-base-patch16", scale_factor=1.0, patch_from_layers=(-1,),
                 amp_dtype=torch.bfloat16, amp_enabled=True):
        super().__init__()
        self.model_name = model_name
        self.scale_factor = scale_factor
        self.patch_from_layers = list(patch_from_layers)
        self.amp_dtype = amp_dtype
        self.amp_enabled = amp_enabled
        cfg = clip_config_from_name(model_name)
        self.patch_size = cfg["patch_size"]
        self.register_buffer("_mean", torch.tensor([0.48145466, 0.4578275, 0.40821073]).view(1, 3, 1, 1),
                             persistent=False)
        self.register_buffer("_std", torch.tensor([0.26862954, 0.26130258, 0.27577711]).view(1, 3, 1, 1),
                             persistent=False)
        self.vision_model = CLIPVisionModel(cfg)
        self.vision_model.reset_parameters()

        def rename(k):
            if k.startswith("vision_model."):
                return k
            if k.startswith("model.vision_model."):
                return k[len("model."):]
            if k.split(".")[0] in ("embeddings", "encoder", "pre_layrnorm", "post_layernorm"):
                return "vision_model." + k    # transformers >= 5 saves CLIPVisionModel flattened
            return None                      # text tower / projections of a full CLIP checkpoint
        loaded = load_safetensors_dir(self.vision_model, model_name, rename=rename)
        self.vision_model.eval().requires_grad_(False)
        self.pretrained_loaded = loaded
        dist.print0(f"CLIPVisionEncoder ready: {model_name} ({'pretrained' if loaded else 'random init'}), "
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
        n = len(self.vision_model.vision_model.encoder.layers)
        idx = [i if i >= 0 else n + i + 2 for i in self.patch_from_layers if i != -1]
        saved, last = self.vision_model.forward_features(x, idx, want_last=True, compute_dtype=dtype)
        feats = []
        for i in self.patch_from_layers:
            t = last if i == -1 else saved[i if i >= 0 else n + i + 2]
            feats.append(t[:, 1:].float())
        return feats, last[:, 0].float()

    @torch.no_grad()
    def encode_text(self, text):
        return None, None, None
