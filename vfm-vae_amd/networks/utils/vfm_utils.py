"""VFM encoder dispatch (reference `networks/utils/vfm_utils.py:26-123`).

Index convention of `patch_from_layers` (shared by every backbone):
  0 = output of the patch embedding, i = output of block i,
 -1 = final sequence after the post-norm, -2 = last block, -3 = second-last, ...
"""
from typing import List

import torch
import torch.nn as nn

from .vfms.siglip2_utils import SigLIP2Encoder

VFM2INTERPOLATION = {
    'siglip': 'bilinear',
    'qwen': 'bicubic',
    'dino': 'bicubic',
    'mae': 'bilinear',
    'eva': 'bicubic',
    'clip': 'bicubic',
}


class VFMEncoder(nn.Module):
    def __init__(self, model_name: str, conditional: bool, label_type: str, scale_factor: float,
                 patch_from_layers: List[int], amp_dtype: torch.dtype = torch.bfloat16, amp_enabled: bool = True):
        super().__init__()
        name = model_name.lower()
        if "siglip2" in name:
            self.encoder = SigLIP2Encoder(model_name=model_name, conditional=conditional, label_type=label_type,
                                          scale_factor=scale_factor, patch_from_layers=patch_from_layers,
                                          amp_dtype=amp_dtype, amp_enabled=amp_enabled)
        elif "dinov2" in name:
            from .vfms.dinov2_utils import DINOv2Encoder
            self.encoder = DINOv2Encoder(model_name=model_name, patch_from_layers=patch_from_layers,
                                         scale_factor=scale_factor, amp_dtype=amp_dtype, amp_enabled=amp_enabled)
        elif "clip" in name:
            from .vfms.clip_utils import CLIPVisionEncoder
            self.encoder = CLIPVisionEncoder(model_name=model_name, patch_from_layers=patch_from_layers,
                                             scale_factor=scale_factor, amp_dtype=amp_dtype, amp_enabled=amp_enabled)
        else:
            raise NotImplementedError(
                f"VFM backbone '{model_name}' is not part of the MI355X training path "
                "(supported: siglip2, dinov2, clip)")

    @property
    def patch_size(self) -> int:
        return self.encoder.patch_size

    def encode_image(self, img, eq_scale_factor: float = 1.0, is_eq_prior: bool = False):
        return self.encoder.encode_image(img, eq_scale_factor, is_eq_prior)

    def encode_text(self, text):
        return self.encoder.encode_text(text)
