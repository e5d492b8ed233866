"""Output containers of the network modules (same fields and defaults as the
reference `networks/utils/dataclasses.py`)."""
from dataclasses import dataclass
from typing import List, Optional

import torch


@dataclass
class EncodeOutput:
    """LDMAdapter.encode(): latent z [B, C, H, W] plus the quantisation/alignment terms."""
    z: torch.Tensor
    vf_loss: Optional[torch.Tensor] = None
    vf_last_layer: Optional[torch.Tensor] = None
    kl_loss: Optional[torch.Tensor] = None
    vq_loss: Optional[torch.Tensor] = None
    entropy_loss: Optional[torch.Tensor] = None
    codebook_usages: Optional[torch.Tensor] = None


@dataclass
class GeneratorForwardOutput:
    """Generator.forward(): reconstruction, multiscale images (smallest first) and losses."""
    gen_img: torch.Tensor
    gen_multiscale_imgs: List[torch.Tensor]
    vf_loss: Optional[torch.Tensor] = None
    vf_last_layer: Optional[torch.Tensor] = None
    kl_loss: Optional[torch.Tensor] = None
    vq_loss: Optional[torch.Tensor] = None
    entropy_loss: Optional[torch.Tensor] = None
    codebook_usages: Optional[torch.Tensor] = None
    eq_scale_factor: float = 1.0
    eq_angle_factor: int = 0
    global_text_tokens: Optional[torch.Tensor] = None


@dataclass
class DiscriminatorForwardOutput:
    """StyleGAN-T logits [B, n_heads*tokens] and PatchGAN outputs (per scale, per layer)."""
    stylegan_t_logits: torch.Tensor
    patchgan_logits: Optional[list] = None
