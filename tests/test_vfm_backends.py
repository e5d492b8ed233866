"""DINOv2 (config 3) and CLIP (config 0) encoder towers vs the HF transformers models they
replace (the reference loads them with AutoModel / SiglipVisionModel.from_pretrained and runs
them under bf16 autocast; here fp32 on CPU, same weights via a local HF directory).

HF transformers is the third-party arithmetic at this boundary; tolerance
1e-4 relative (fp32, different GEMM / attention kernels)."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F


def _rel(a, b):
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


@pytest.fixture(scope="module")
def dinov2_dir(tmp_path_factory):
    from transformers import Dinov2Config, Dinov2Model
    d = str(tmp_path_factory.mktemp("m") / "tiny-dinov2-local")
    cfg = Dinov2Config(hidden_size=64, num_hidden_layers=3, num_attention_heads=4, mlp_ratio=4, image_size=56,
                       patch_size=14, layerscale_value=0.7)
    torch.manual_seed(0)
    m = Dinov2Model(cfg)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(torch.randn_like(p) * 0.02)
    m.save_pretrained(d)
    return d


@pytest.mark.parametrize("size", [56, 70])
def test_dinov2_matches_hf(dinov2_dir, size):
    from transformers import Dinov2Model
    from networks.utils.vfms.dinov2_utils import DINOv2Encoder
    hf = Dinov2Model.from_pretrained(dinov2_dir).eval()
    enc = DINOv2Encoder(model_name=dinov2_dir, scale_factor=1.0, patch_from_layers=[0, 2, -2, -1])
    assert enc.pretrained_loaded
    g = torch.Generator().manual_seed(1)
    img = torch.rand(2, 3, size, size, generator=g)
    feats, pooled = enc.encode_image(img, 1.0, False)
    # the reference wrapper's preprocessing (dinov2_utils.py:77-94) then HF forward (:101-121)
    x = (img - torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)) / torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    with torch.no_grad():
        out = hf(pixel_values=x, output_hidden_states=True, return_dict=True)
    ref = [out.hidden_states[0][:, 1:], out.hidden_states[2][:, 1:], out.hidden_states[-1][:, 1:],
           out.last_hidden_state[:, 1:]]
    for f, r in zip(feats, ref):
        assert f.shape == r.shape
        assert _rel(f, r) < 1e-4
    assert _rel(pooled, out.pooler_output) < 1e-4


def test_dinov2_eq_prior_downscale(dinov2_dir):
    from networks.utils.vfms.dinov2_utils import DINOv2Encoder
    enc = DINOv2Encoder(model_name=dinov2_dir, scale_factor=1.0, patch_from_layers=[-1])
    feats, _ = enc.encode_image(torch.rand(1, 3, 112, 112), 0.5, True)
    assert feats[0].shape == (1, 16, 64)


@pytest.fixture(scope="module")
def clip_dir(tmp_path_factory):
    from transformers import CLIPVisionConfig, CLIPVisionModel
    d = str(tmp_path_factory.mktemp("m") / "tiny-clip-vit-patch16")
    cfg = CLIPVisionConfig(hidden_size=64, num_hidden_layers=3, num_attention_heads=4, intermediate_size=128,
                           image_size=32, patch_size=16)
    torch.manual_seed(2)
    m = CLIPVisionModel(cfg)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(torch.randn_like(p) * 0.02)
    m.save_pretrained(d)
    return d


@pytest.mark.parametrize("size", [32, 48])
def test_clip_matches_hf(clip_dir, size):
    from transformers import CLIPVisionModel
    from networks.utils.vfms.clip_utils import CLIPVisionEncoder
    hf = CLIPVisionModel.from_pretrained(clip_dir).eval()
    enc = CLIPVisionEncoder(model_name=clip_dir, scale_factor=1.0, patch_from_layers=[0, 2, -1])
    assert enc.pretrained_loaded
    img = torch.rand(2, 3, size, size, generator=torch.Generator().manual_seed(3))
    feats, pooled = enc.encode_image(img, 1.0, False)
    mean = torch.tensor([0.48145466, 0.4578275, 0.40821073]).view(1, 3, 1, 1)
    std = torch.tensor([0.26862954, 0.26130258, 0.27577711]).view(1, 3, 1, 1)
    with torch.no_grad():
        out = hf(pixel_values=(img - mean) / std, output_hidden_states=True, interpolate_pos_encoding=True)
    post = getattr(hf, "vision_model", hf).post_layernorm      # transformers >= 5 flattens the model
    ref = [out.hidden_states[0][:, 1:], out.hidden_states[2][:, 1:], post(out.last_hidden_state)[:, 1:]]
    for f, r in zip(feats, ref):
        assert f.shape == r.shape
        assert _rel(f, r) < 1e-4
    assert _rel(pooled, out.pooler_output) < 1e-4


def test_vfm_dispatch_names(dinov2_dir, clip_dir):
    from networks.utils.vfm_utils import VFMEncoder
    assert VFMEncoder(dinov2_dir, False, 'cls2text', 1.0, [-1]).patch_size == 14
    assert VFMEncoder(clip_dir, False, 'cls2text', 1.0, [-1]).patch_size == 16
