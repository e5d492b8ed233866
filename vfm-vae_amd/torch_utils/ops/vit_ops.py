"""Dense transformer pieces of the frozen VFM towers (SigLIP2 / DINO ViTs).

Reference math: HF `SiglipEncoderLayer` / timm `Block` as used by
`networks/utils/vfms/siglip2_utils.py:114-137` and `networks/discriminator.py:145-168`
under bf16 autocast: GEMMs in the compute dtype with fp32 accumulation,
LayerNorm and residual stream in fp32.

GEMMs are plain library GEMMs (hipBLASLt through torch.matmul, MFMA); the
epilogues (bias + tanh-GELU) and LayerNorm->bf16 have HIP kernels registered
by `vit_hip` when the native library is present.
"""
import torch
import torch.nn.functional as F

_HIP_OPS = set()


def _hip(name, x):
    return x.is_cuda and name in _HIP_OPS


def patch_embed(pixels, weight, bias, patch, compute_dtype):
    """Non-overlapping patch projection as one GEMM: [B, 3, H, W] -> [B, (H/p)(W/p), D]."""
    B, C, H, W = pixels.shape
    gh, gw = H // patch, W // patch
    x = pixels[:, :, :gh * patch, :gw * patch].to(compute_dtype)
    x = x.reshape(B, C, gh, patch, gw, patch).permute(0, 2, 4, 1, 3, 5).reshape(B, gh * gw, C * patch * patch)
    w = weight.reshape(weight.shape[0], -1).to(compute_dtype)
    y = torch.matmul(x, w.t())
    if bias is not None:
        y = y + bias.to(compute_dtype)
    return y


def linear(x, w, b=None):
    """x @ w^T + b in x's dtype (bias added in fp32 then rounded)."""
    if b is not None:
        return torch.addmm(b.to(x.dtype), x.reshape(-1, x.shape[-1]), w.t()).reshape(*x.shape[:-1], w.shape[0])
    return torch.matmul(x, w.t())


def linear_gelu_tanh(x, w, b=None):
    if _hip("bias_gelu_tanh", x):
        from . import vit_hip
        return vit_hip.linear_gelu_tanh(x, w, b)
    return F.gelu(linear(x, w, b), approximate="tanh")


def layer_norm(h, ln, out_dtype):
    """LayerNorm of the fp32 residual stream, emitted in the GEMM compute dtype."""
    if _hip("layer_norm", h):
        from . import vit_hip
        return vit_hip.layer_norm(h, ln.weight, ln.bias, ln.eps, out_dtype)
    return F.layer_norm(h.float(), (h.shape[-1],), ln.weight.float(), ln.bias.float(), ln.eps).to(out_dtype)


def residual_add(h, delta):
    return h + delta.float()
