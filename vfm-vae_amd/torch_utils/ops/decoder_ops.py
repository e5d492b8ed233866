"""Decoder ops that actually run in the shipped configs (ConvNeXt synthesis layers,
separable upsampling, z-conv stems), with a HIP path on ROCm devices and a
pure-torch path elsewhere.

Reference call sites: `networks/utils/convnext_utils.py:36-257`
(modulated_pointwise_conv2d, ConvNeXtSynthesisLayer, SeparableUpsampleWithFixedBlur),
`networks/utils/shared.py:165-167` (GroupNorm32), `networks/generator.py:839-868`.

Each public function takes `impl` ('cuda' | 'ref'); 'cuda' on a ROCm tensor
dispatches to the gfx950 kernels when they are built for that op (see
`_HIP_OPS`), otherwise (CPU tensors or impl='ref') the torch formulation runs.
"""
import math

import torch
import torch.nn.functional as F

_HIP_OPS = {'group_norm', 'dwconv2d', 'scale_bias_gelu', 'layer_scale_residual', 'shuffle_blur',
            'blur_replicate'}
_FORCE_REF = False        # global switch for A/B experiments and CPU restatement timing


def _use_hip(name, x, impl, **kw):
    """True when the gfx950 kernel runs: ROCm tensor, impl='cuda', op built and shape
    covered (decoder_hip.supported). Importing decoder_hip loads the kernel library
    and raises if it is missing."""
    if not (impl == 'cuda' and x.is_cuda and not _FORCE_REF and name in _HIP_OPS):
        return False
    from . import decoder_hip
    return decoder_hip.supported(name if name != 'blur_replicate' else 'shuffle_blur', x, **kw)


def set_force_ref(flag: bool):
    global _FORCE_REF
    _FORCE_REF = bool(flag)


def force_ref() -> bool:
    """True while set_force_ref(True) holds: every decoder op (and the fused ones built on them, e.g.
    the GigaGAN null-KV attention Function) takes its torch formulation."""
    return _FORCE_REF


# ---------------------------------------------------------------------------
# GroupNorm (fp32 statistics), optionally fused with a per-sample channel scale.


def group_norm(x, num_groups, weight=None, bias=None, eps=1e-5, out_dtype=None, style=None, impl='cuda'):
    """out = (GN(x.float()) * weight + bias) [* style[b, c]] cast to out_dtype.

    `style` ([B, C]) folds the input modulation of a modulated 1x1 conv into the
    normalisation pass (w_b = W * s_b  <=>  W @ (s_b * x))."""
    out_dtype = out_dtype or x.dtype
    if _use_hip('group_norm', x, impl, groups=num_groups):
        from . import decoder_hip
        return decoder_hip.group_norm(x, num_groups, weight, bias, eps, out_dtype, style)
    y = F.group_norm(x.float(), num_groups, weight.float() if weight is not None else None,
                     bias.float() if bias is not None else None, eps)
    if style is not None:
        y = y * style.float()[:, :, None, None]
    return y.to(out_dtype)


# ---------------------------------------------------------------------------
# 1x1 convolution on a flattened plane: y[b] = W @ x[b].


def pointwise(weight, x, impl='cuda'):
    """weight [O, I] (any float dtype; cast to x.dtype for the product), x [B, I, P] -> [B, O, P].

    `torch.matmul(W, x)` folds the batch into the GEMM's M dimension, which for a
    [B, I, P] operand means a transposing copy in forward and transposed (non-
    contiguous) results in both passes. On ROCm tensors the product runs as a
    stride-0-batch bmm (hipBLASLt) whose forward, data-gradient and weight-gradient
    GEMMs all read and write their operands in place, and the weight gradient is
    reduced in fp32 and returned in the parameter's dtype (decoder_hip._Pointwise)."""
    if impl == 'cuda' and x.is_cuda and not _FORCE_REF and x.dim() == 3 and weight.dim() == 2:
        from . import decoder_hip
        return decoder_hip.pointwise(weight, x)
    return torch.matmul(weight.to(x.dtype), x)


# ---------------------------------------------------------------------------
# Depthwise k x k convolution (+bias, + optional additive [H, W] plane).


def dwconv2d(x, weight, bias=None, padding=0, noise=None, impl='cuda', slot=None, noise_strength=None):
    """Depthwise conv: weight [C, 1, k, k], zero padding `padding`, stride 1.
    `noise` ([H_out, W_out], fp32) is added to every channel (legacy noise path); with
    `noise_strength` (0-d) the added plane is noise * noise_strength. `slot`
    (decoder_hip.ResidualSlot, HIP path only) receives the layer's residual gradient."""
    if _use_hip('dwconv2d', x, impl, k=weight.shape[-1]):
        from . import decoder_hip
        return decoder_hip.dwconv2d(x, weight, bias, padding, noise, slot, noise_strength)
    y = F.conv2d(x, weight.to(x.dtype), bias.to(x.dtype) if bias is not None else None, padding=padding,
                 groups=x.shape[1])
    if noise is not None:
        if noise_strength is not None:
            noise = noise * noise_strength
        y = y + noise.to(y.dtype)
    return y


# ---------------------------------------------------------------------------
# Modulated 1x1 epilogue: gelu(h * dcoef[b, o] + bias[o]).


def scale_bias_gelu(h, scale=None, bias=None, impl='cuda'):
    """h: [B, O, P]; scale: [B, O] fp32 (demodulation); bias: [O]. Exact (erf) GELU."""
    if _use_hip('scale_bias_gelu', h, impl):
        from . import decoder_hip
        return decoder_hip.scale_bias_gelu(h, scale, bias)
    z = h.float()
    if scale is not None:
        z = z * scale.float()[:, :, None]
    if bias is not None:
        z = z + bias.float()[None, :, None]
    return F.gelu(z).to(h.dtype)


# ---------------------------------------------------------------------------
# Residual with layer scale: x_in + gamma[c] * (y + b[c]).


def layer_scale_residual(y, bias, gamma, x_in, impl='cuda', slot=None):
    """y: [B, C, P] (or [B, C, H, W]); bias, gamma: [C]; x_in like y. Output dtype = x_in.dtype."""
    if _use_hip('layer_scale_residual', y, impl):
        from . import decoder_hip
        return decoder_hip.layer_scale_residual(y, bias, gamma, x_in, slot)
    shape = [1, -1] + [1] * (y.ndim - 2)
    z = y.float()
    if bias is not None:
        z = z + bias.float().reshape(shape)
    if gamma is not None:
        z = z * gamma.float().reshape(shape)
    return (z + x_in.float()).to(x_in.dtype)


# ---------------------------------------------------------------------------
# Fixed separable blur with replicate padding, fused with the pixel shuffle.


def shuffle_blur(x, blur1d, upscale=2, impl='cuda'):
    """PixelShuffle(upscale) followed by replicate-pad + depthwise blur with the
    normalised outer product of `blur1d` (a python list of taps)."""
    if _use_hip('shuffle_blur', x, impl, k=len(blur1d), r=upscale):
        from . import decoder_hip
        return decoder_hip.shuffle_blur(x, blur1d, upscale)
    y = F.pixel_shuffle(x, upscale)
    return blur_replicate(y, blur1d, impl='ref')


def blur_replicate(x, blur1d, impl='cuda'):
    if _use_hip('blur_replicate', x, impl, k=len(blur1d)):
        from . import decoder_hip
        return decoder_hip.blur_replicate(x, blur1d)
    k = torch.tensor(blur1d, dtype=torch.float32)
    k2 = torch.outer(k, k)
    k2 = k2 / k2.sum()
    kh, kw = k2.shape
    ph, pw = (kh - 1) // 2, (kw - 1) // 2
    pad = (pw, pw + int(kw % 2 == 0), ph, ph + int(kh % 2 == 0))
    c = x.shape[1]
    w = k2[None, None].repeat(c, 1, 1, 1).to(device=x.device, dtype=x.dtype)
    return F.conv2d(F.pad(x, pad, mode='replicate'), w, groups=c)


def torgb(x, weight2d, style, bias, impl='cuda'):
    """Modulated (no demodulation) 1x1 conv to the image channels + bias, fp32 result:
    (W @ (style * x)) + bias (reference convnext_utils.py:145-187). ROCm tensors run the fused
    HIP kernels (csrc/torgb.hip); elsewhere the torch formulation."""
    if impl == 'cuda' and x.is_cuda and not _FORCE_REF:
        from . import decoder_hip
        if decoder_hip.torgb_supported(x, weight2d.shape[0]):
            return decoder_hip.torgb(x, weight2d, style, bias)
    B, C, H, W = x.shape
    xm = x * style.to(x.dtype)[:, :, None, None]
    y = pointwise(weight2d, xm.reshape(B, C, H * W), impl=impl).reshape(B, -1, H, W)
    return y + bias


def convnext_mlp_fusable(m, C, P, x_in):
    """True when the layer's pointwise -> GELU -> pointwise -> residual chain can run as
    one forward kernel (with or without autograd): ROCm bf16 activations, a supported
    width (decoder_hip.MLP_CHANNELS)."""
    if _FORCE_REF or not m.is_cuda or x_in.dtype != torch.bfloat16:
        return False
    from . import decoder_hip
    return decoder_hip.convnext_mlp_supported(m, C, P)


def convnext_mlp_nograd(m, w1, dcoef, b1, w2, b2, gamma, x_in, slot=None):
    from . import decoder_hip
    if torch.is_grad_enabled():
        return decoder_hip.convnext_mlp(m, w1, dcoef, b1, w2, b2, gamma, x_in, slot)
    return decoder_hip.convnext_mlp_nograd(m, w1, dcoef, b1, w2, b2, gamma, x_in)


STYLE_HIP = __import__("os").environ.get("VFM_STYLE_HIP", "1") == "1"     # A/B switch


def style_and_demod(affine, w, w1=None, eps=1e-8):
    """(style [B, C] fp32, dcoef [B, O] or None) of a ConvNeXt synthesis layer: style =
    affine(w) (a StyleSplit over a linear FullyConnectedLayer, reference networks/utils/shared.py),
    dcoef = demod_coefficients(w1, style) when w1 is given. ROCm fp32: csrc/style.hip (two launches
    each way); elsewhere the torch formulation."""
    from . import style_group
    r = style_group.lookup(affine, w, w1, eps)            # the network's grouped launch (style_group.StyleGroup)
    if r is not None:
        return r
    fc = affine.proj
    if (STYLE_HIP and w.is_cuda and not _FORCE_REF and w.dtype == torch.float32 and w.dim() == 2 and fc.activation == 'linear'
            and fc.bias is not None and fc.weight.dtype == torch.float32
            and (w1 is None or w1.dtype == torch.float32)):
        from . import decoder_hip
        return decoder_hip.style_demod(w, fc.weight, fc.bias, w1, fc.weight_gain, fc.bias_gain, eps)
    style = affine(w).float()
    return style, (demod_coefficients(w1, style, eps) if w1 is not None else None)


def demod_coefficients(weight2d, style, eps=1e-8):
    """dcoef[b, o] = rsqrt(sum_i (W[o, i] * s[b, i])^2 + eps), computed as a tiny GEMM."""
    return torch.rsqrt(style.float().square() @ weight2d.float().square().t() + eps)


def gelu_tanh(x):
    return F.gelu(x, approximate='tanh')


SQRT1_2 = 1.0 / math.sqrt(2.0)
