"""Dense transformer pieces of the frozen VFM towers (SigLIP2 / DINO ViTs).

Reference math: HF `SiglipEncoderLayer` / timm `Block` as used by
`networks/utils/vfms/siglip2_utils.py:114-137` and `networks/discriminator.py:145-168`
under bf16 autocast: GEMMs in the compute dtype with fp32 accumulation,
LayerNorm and residual stream in fp32.

bf16 GEMMs (the SigLIP2 tower under autocast) run on our 256-tile MFMA GEMM on ROCm tensors outside
autograd (csrc/gemm9.hip), with the bias and fc1's tanh-GELU (the form SigLIP uses) in the epilogue;
with VFM_VIT_GEMM=torch they are hipBLASLt GEMMs through torch.matmul / addmm (A/B).
fp32 linears (the DINO ViT-S tower of the projected discriminator, whose input gradient
the G phase takes) run on our GEMM with fp32-equivalent f32x6 products and autograd
(torch_utils/ops/linear.py). LayerNorm -> compute dtype (optionally fused with the
residual add) is one HIP row kernel (`vit_hip`, csrc/vit.hip).
"""
import os

import torch
import torch.nn.functional as F

from . import kernel_timer

# bf16 linears of the frozen towers on our 256-tile GEMM (csrc/gemm9.hip, bias / bias + tanh-GELU in the
# epilogue); VFM_VIT_GEMM=torch: hipBLASLt (A/B)
OWN_GEMM = os.environ.get("VFM_VIT_GEMM", "hip") == "hip"


def frozen_weight(w, dtype):
    """w cast to dtype; for a tensor that needs no gradient (the frozen towers' weights and biases)
    cached on it until its version moves, so the cast runs once instead of at every forward (not
    cached while a HIP graph is being captured: decoder_hip._cast_cached)."""
    if w is None or w.dtype == dtype:
        return w
    if not w.is_cuda or (w.requires_grad and torch.is_grad_enabled()):
        return w.to(dtype)
    from .decoder_hip import _cast_cached
    return _cast_cached(w, dtype)


def _own_linear(x, w, b, act=None):
    """x @ w^T (+ b, + act) on gemm8 for ROCm bf16 tensors outside autograd, else None. The bias is
    rounded to x's dtype first and added to the fp32 accumulator (hipBLASLt's bias epilogue)."""
    if not (OWN_GEMM and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and _frozen(x, w, b)):
        return None
    from . import gemm_hip
    from .decoder_hip import _cast_cached
    bias = None if b is None else _cast_cached(_cast_cached(b, x.dtype), torch.float32)
    x2 = x.reshape(-1, x.shape[-1])
    y = gemm_hip.try_gemm(x2, w.t(), bias=bias, bias_dim=1, act=act, route=("g9", 0))
    return None if y is None else y.reshape(*x.shape[:-1], w.shape[0])


def _vg(x, w, tag):
    """Timer region of a library GEMM x [.., K] @ w^T [K, N] (kernel_timer.vendor_gemm)."""
    if not kernel_timer.is_enabled() or not x.is_cuda:
        return kernel_timer._NULL
    M = x.numel() // x.shape[-1]
    return kernel_timer.vendor_gemm(f"{'bf16' if x.dtype == torch.bfloat16 else 'f32'},{tag}", M, w.shape[0],
                                    x.shape[-1], 1, x.element_size())


def _frozen(*ts):
    """ROCm tensors that need no autograd graph."""
    return ts[0].is_cuda and not (torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in ts))


def patch_embed(pixels, weight, bias, patch, compute_dtype):
    """Non-overlapping patch projection as one GEMM: [B, 3, H, W] -> [B, (H/p)(W/p), D]."""
    B, C, H, W = pixels.shape
    gh, gw = H // patch, W // patch
    x = pixels[:, :, :gh * patch, :gw * patch].to(compute_dtype)
    x = x.reshape(B, C, gh, patch, gw, patch).permute(0, 2, 4, 1, 3, 5).reshape(B, gh * gw, C * patch * patch)
    w = frozen_weight(weight, compute_dtype).reshape(weight.shape[0], -1)
    y = None
    if x.is_cuda and OWN_GEMM and _frozen(x, w):
        # the patch projection on our GEMMs (bf16: gemm9, fp32: f32x6)
        from . import gemm_hip
        y = gemm_hip.try_gemm(x.reshape(-1, x.shape[-1]), w.t(), auto=True)
        y = None if y is None else y.reshape(B, gh * gw, w.shape[0])
    if y is None and x.is_cuda and OWN_GEMM and x.dtype in (torch.float32, torch.bfloat16):
        # input gradient wanted (the D's patch projection in the G phase): forward and data gradient on our GEMMs
        from .linear import linear as _lin
        y = _lin(x, w)
    if y is None:
        with _vg(x, w, "vit_patch"):
            y = torch.matmul(x, w.t())
    if bias is not None:
        y = y + frozen_weight(bias, compute_dtype)
    return y


def linear(x, w, b=None):
    """x @ w^T + b in x's dtype (bias added in fp32 then rounded)."""
    if x.is_cuda and x.dtype == torch.float32:
        from . import linear as linear_op
        return linear_op.linear(x, w, b)
    if x.is_cuda:
        y = _own_linear(x, w, b)
        if y is not None:
            return y
    with _vg(x, w, "vit_linear"):
        if b is not None:
            return torch.addmm(frozen_weight(b, x.dtype), x.reshape(-1, x.shape[-1]), w.t()).reshape(
                *x.shape[:-1], w.shape[0])
        return torch.matmul(x, w.t())


def linear_gelu(x, w, b=None):
    """gelu(x @ w^T + b), erf form (DINOv2 / HF "gelu"): the bf16 GEMM with the erf-GELU epilogue on ROCm frozen
    towers (one rounding of GELU(acc + b) instead of a bf16 product, a bf16 GELU pass and its HBM round trip)."""
    if b is not None and x.dtype != torch.float32 and _frozen(x, w, b):
        y = _own_linear(x, w, b, act="gelu")
        if y is not None:
            return y
    return F.gelu(linear(x, w, b))


def linear_gelu_tanh(x, w, b=None):
    """gelu_tanh(x @ w^T + b): GEMM with the GELU_BIAS epilogue on ROCm (frozen towers)."""
    if b is not None and x.dtype != torch.float32 and _frozen(x, w, b):
        y = _own_linear(x, w, b, act="gelu_tanh")
        if y is not None:
            return y
        with _vg(x, w, "vit_fc1_gelu"):
            y = torch._addmm_activation(frozen_weight(b, x.dtype), x.reshape(-1, x.shape[-1]), w.t(), use_gelu=True)
        return y.reshape(*x.shape[:-1], w.shape[0])
    return F.gelu(linear(x, w, b), approximate="tanh")


def layer_norm(h, ln, out_dtype):
    """LayerNorm of the fp32 residual stream, emitted in the GEMM compute dtype."""
    if _frozen(h, ln.weight, ln.bias):            # no autograd graph at all (a trainable norm takes the torch path)
        from . import vit_hip
        if vit_hip.supported(h):
            return vit_hip.residual_layer_norm(h, None, ln, out_dtype)[1]
        if h.dtype == torch.float32 and h.shape[-1] % 128 == 0 and h.shape[-1] <= 1024 and vit_hip.LN_GRAD:
            return vit_hip.layer_norm_grad(h, ln, out_dtype)    # D = 384 (DINOv2 ViT-S) without a graph
    elif torch.is_grad_enabled() and h.is_cuda:
        from . import vit_hip
        if vit_hip.LN_GRAD and vit_hip.layer_norm_grad_supported(h, ln):   # frozen backbone, input gradient
            return vit_hip.layer_norm_grad(h, ln, out_dtype)
    return F.layer_norm(h.float(), (h.shape[-1],), ln.weight.float(), ln.bias.float(), ln.eps).to(out_dtype)


def residual_layer_norm(h, delta, ln, out_dtype):
    """(h + delta, LayerNorm(h + delta) in out_dtype) -- one pass on ROCm (frozen towers)."""
    if _frozen(h, delta):
        from . import vit_hip
        if vit_hip.supported(h):
            return vit_hip.residual_layer_norm(h, delta, ln, out_dtype)
    h = residual_add(h, delta)
    return h, F.layer_norm(h, (h.shape[-1],), ln.weight.float(), ln.bias.float(), ln.eps).to(out_dtype)


def residual_add(h, delta):
    return h + delta.float()


def attention_packed(qkv, heads):
    """Multi-head self-attention of a packed [B, N, 3*D] (q | k | v) projection -> [B, N, D].
    ROCm bf16 tensors outside autograd with head dim 64 (the frozen towers) run the fused
    HIP kernel (attn_hip, csrc/attention.hip) straight on the packed layout; everything
    else (CPU, fp32 parity runs, other head dims) is torch SDPA."""
    B, N, D3 = qkv.shape
    D = D3 // 3
    d = D // heads
    if _frozen(qkv):
        from . import attn_hip
        if attn_hip.supported(qkv, d):
            return attn_hip.attention_packed(qkv, heads)
    q, k, v = qkv.reshape(B, N, 3, heads, d).permute(2, 0, 3, 1, 4).unbind(0)
    return sdpa(q, k, v).transpose(1, 2).reshape(B, N, D)


def sdpa_packed(qkv, heads):
    """sdpa of the q / k / v packed in one projection output qkv [B, N, 3 heads d] -> [B, heads, N, d]:
    fp32 ROCm operands on the packed HIP kernels (reads in place, one packed gradient), else unpacked."""
    if qkv.is_cuda and qkv.dtype == torch.float32:
        from . import attn_hip
        out = attn_hip.sdpa_f32_packed(qkv, heads)
        if out is not None:
            return out
    B, N, D3 = qkv.shape
    q, k, v = qkv.reshape(B, N, 3, heads, D3 // (3 * heads)).permute(2, 0, 3, 1, 4).unbind(0)
    return sdpa(q, k, v)


def sdpa(q, k, v):
    """F.scaled_dot_product_attention(q, k, v) (no mask, default scale) on [B, H, N, d] operands.
    fp32 ROCm operands with head dim 64 run the HIP kernels (attn_hip.sdpa_f32, forward and
    backward: the generator's adapter / decoder attention and the D's DINO tower); the rest is
    torch SDPA."""
    if q.is_cuda:
        if q.dtype == torch.float32:
            from . import attn_hip
            if attn_hip.supported_f32(q, k, v):
                return attn_hip.sdpa_f32(q, k, v)
        if q.stride(-1) != 1:
            # AOTriton's fused kernels need stride(-1) == 1 on q (else the math path: an explicit
            # [B, h, N, N] score tensor)
            q = q.contiguous()
    return F.scaled_dot_product_attention(q, k, v)
