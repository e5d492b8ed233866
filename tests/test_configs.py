"""BASELINE.json config variants build from their YAML (same class_name / kwarg surface as the
reference configs) and run one validation-mode reconstruction on CPU at batch 1:
  config 0 (CLIP ViT-B/16, the CPU plumbing case), config 3 (DINOv2-L, 384^2 of the dynamic
  256/384/512 stream), config 4 (discrete VQ latent; indices from the codebook lookup).
Architectures are random-initialised (no checkpoints offline)."""
import os

import pytest
import torch
import yaml

from conftest import PKG

CFG = os.path.join(PKG, "configs")


def _build(name):
    import dnnlib
    from train import resolve_config
    c = resolve_config(yaml.safe_load(open(os.path.join(CFG, name))))
    torch.manual_seed(0)
    G = dnnlib.util.construct_class_by_name(label_dim=0, **c.G_kwargs).eval()
    return c, G


@torch.no_grad()
def test_config0_clip_cpu_reconstruction():
    c, G = _build("vfm_vae_f16d32_clip_b16_stage_0_cpu.yaml")
    assert c.batch_size == 1
    img = torch.rand(1, 3, 256, 256, generator=torch.Generator().manual_seed(1))
    out = G(img, ['a photo'], validation=True)
    assert out.gen_img.shape == (1, 3, 256, 256) and torch.isfinite(out.gen_img).all()


@torch.no_grad()
def test_config3_dinov2_dynamic_resolution_cpu():
    from training.data_synthetic import SyntheticDataset
    c, G = _build("vfm_vae_f16d32_dinov2_l_stage_0_dynres.yaml")
    ds = SyntheticDataset(**{k: v for k, v in c.training_set_kwargs.items() if k != 'class_name'})
    pool = ds.make_pool(1, 'cpu')
    assert [p.shape[-1] for p in pool[:3]] == [256, 384, 512]
    img = pool[1].float() / 255.
    out = G(img, ['a photo'], validation=True)
    assert out.gen_img.shape == (1, 3, 384, 384) and torch.isfinite(out.gen_img).all()


@torch.no_grad()
def test_config4_vq_cpu_indices():
    c, G = _build("vfm_vae_f16d32_siglip2_stage_0_vq.yaml")
    img = torch.rand(1, 3, 256, 256, generator=torch.Generator().manual_seed(2))
    out = G(img, ['a photo'], validation=True)
    assert out.gen_img.shape == (1, 3, 256, 256) and torch.isfinite(out.gen_img).all()
    feats, *_ = G.vfm_encoder.encode_image(img)
    z = G.ldm_adapter.encode(feats, return_z_before_quantize=True).z            # [1, 32, 16, 16]
    idx = G.ldm_adapter.quantizer.f_to_idx(z.flatten(2).transpose(1, 2))          # [1, 8, 256]
    assert idx.shape == (1, 8, 256) and idx.dtype == torch.int64
    assert idx.min() >= 0 and idx.max() < 4096
