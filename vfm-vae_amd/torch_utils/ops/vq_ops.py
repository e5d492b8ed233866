"""Codebook lookup for the discrete latent: argmax_v <f/|f|, w_v/|w_v|>.

Reference: `networks/utils/quant_utils.py:92-94` (VectorQuantizer.forward) and
:126-131 (f_to_idx): F.normalize both sides (eps 1e-12), fp32 matmul, argmax
(first maximal index). The HIP kernel (`vfm_codebook_argmax`) evaluates the
same expression with a fixed summation order so the int64 indices are
reproducible bit-for-bit against the C oracle.
"""
import torch
import torch.nn.functional as F

_HIP = False  # set by vq_hip when the native kernel is available


def codebook_argmax(features, codebook_weight, impl='cuda'):
    """features [N, C] (any float), codebook_weight [V, C] -> int64 indices [N]."""
    if _HIP and impl == 'cuda' and features.is_cuda:
        from . import vq_hip
        return vq_hip.codebook_argmax(features, codebook_weight)
    f = F.normalize(features.float(), dim=-1)
    w = F.normalize(codebook_weight.float(), dim=1)
    return torch.argmax(f @ w.t(), dim=1)
