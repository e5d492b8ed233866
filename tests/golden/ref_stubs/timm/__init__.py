"""Stub: timm.create_model for 'vit_small_patch16_224_dino' (random ViT-S/16)."""
from . import layers, data  # noqa: F401
from ._vit import VisionTransformer


def create_model(name, pretrained=False, **kwargs):
    assert name == 'vit_small_patch16_224_dino', name
    return VisionTransformer()
