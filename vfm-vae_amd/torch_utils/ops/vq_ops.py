"""Codebook lookup for the discrete latent: argmax_v <f/|f|, w_v/|w_v|>.

Reference: `networks/utils/quant_utils.py:84-86` (VectorQuantizer.forward) and
:126-131 (f_to_idx): F.normalize both sides (eps 1e-12), fp32 matmul, argmax
(first maximal index). On ROCm tensors the HIP kernel `vfm_codebook_argmax`
(csrc/vq.hip) evaluates the same expression in a fixed fp32 order, so the int64
indices are reproducible bit-for-bit against the C oracle; a missing kernel
library raises. CPU tensors (or impl='ref') run the torch formulation.
"""
import torch
import torch.nn.functional as F

from . import kernel_timer


def codebook_argmax(features, codebook_weight, impl='cuda'):
    """features [N, C] (any float), codebook_weight [V, C] -> int64 indices [N]."""
    if impl == 'cuda' and features.is_cuda:
        return _codebook_argmax_hip(features, codebook_weight)
    f = F.normalize(features.float(), dim=-1)
    w = F.normalize(codebook_weight.float(), dim=1)
    return torch.argmax(f @ w.t(), dim=1)


def _codebook_argmax_hip(features, codebook_weight):
    from .. import custom_ops
    lib = custom_ops.get_native()
    f = features.detach().float()
    if f.ndim != 2 or f.stride(1) != 1:
        f = f.reshape(-1, f.shape[-1]).contiguous()
    w = codebook_weight.detach().float().contiguous()
    N, C = f.shape
    V = w.shape[0]
    if w.shape[1] != C:
        raise RuntimeError(f"codebook width {w.shape[1]} != feature width {C}")
    if w.device != f.device:
        raise RuntimeError("features and codebook must be on the same device")
    idx = torch.empty(N, dtype=torch.int64, device=f.device)
    ld = f.stride(0) if N > 1 else C
    with kernel_timer.region('codebook_argmax', (N * C + V * C) * 4 + N * 8, flops=2 * N * V * C):
        rc = lib.vfm_codebook_argmax(f.data_ptr(), ld, w.data_ptr(), N, C, V, idx.data_ptr(),
                                     custom_ops.stream_ptr(f.device))
    if rc == custom_ops.VFM_NO_KERNEL:
        raise custom_ops.NativeError(f"vfm_codebook_argmax: no kernel for codebook width {C} "
                                     "(supported: 1, 2, 3, 4, 8, 16, 32, 64)")
    custom_ops.check(rc, "vfm_codebook_argmax")
    return idx
