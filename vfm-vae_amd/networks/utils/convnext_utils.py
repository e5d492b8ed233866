"""ConvNeXt decoder layers of the VFM-VAE synthesis network.

Same classes, arguments and parameter/buffer names as the reference
`networks/utils/convnext_utils.py` (:36-257), so checkpoints load unchanged.

The per-sample modulated 1x1 conv is NOT run as a grouped conv with per-sample
weights (reference :36-57). Its algebraic equivalent is used instead:
    W_b = W * s_b[i] * d_b[o]   =>   W_b @ x_b = d_b ⊙ (W @ (s_b ⊙ x_b)),
    d_b[o] = rsqrt(sum_i (W[o,i] s_b[i])^2 + 1e-8),
so the input modulation is folded into the GroupNorm pass, the 1x1 is one
batched GEMM with a shared weight (MFMA via hipBLASLt), and the demodulation,
bias and GELU are one fused epilogue kernel. (The reference's fp16
pre-normalisation of W and s cancels under demodulation up to the 1e-8 epsilon.)
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from networks.utils.shared import GroupNorm32, StyleSplit
from torch_utils.ops import decoder_ops


def trunc_normal_(tensor, std=0.02):
    return nn.init.trunc_normal_(tensor, mean=0.0, std=std, a=-2.0, b=2.0)


def modulated_pointwise_conv2d(x, weight, style, bias=None, demodulate=True):
    """Per-sample modulated (+demodulated) 1x1 conv. x [B, I, H, W], weight [O, I, 1, 1],
    style [B, I], bias broadcastable to [B, O, H, W]."""
    B, I, H, W = x.shape
    w2 = weight.reshape(weight.shape[0], I)
    xm = x * style.to(x.dtype)[:, :, None, None]
    y = decoder_ops.pointwise(w2, xm.reshape(B, I, H * W))
    if demodulate:
        y = y * decoder_ops.demod_coefficients(w2, style).to(y.dtype)[:, :, None]
    y = y.reshape(B, -1, H, W)
    if bias is not None:
        y = y + bias
    return y


class ModulatedPointwiseConv2DLayer(nn.Module):
    def __init__(self, in_channels, out_channels, demodulate=True):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.demodulate = demodulate
        self.weight = nn.Parameter(torch.empty([out_channels, in_channels, 1, 1]))
        self.bias = nn.Parameter(torch.zeros(1, out_channels, 1, 1))
        trunc_normal_(self.weight, std=0.02)

    def forward(self, x, style):
        return modulated_pointwise_conv2d(x, self.weight, style, self.bias, self.demodulate)


class ConvNeXtSynthesisLayer(nn.Module):
    """dwconv k x k (+bias) [+ legacy noise] -> GroupNorm32 -> modulated 1x1 C->4C ->
    GELU -> 1x1 4C->C -> gamma * y + x_in   (reference convnext_utils.py:78-142)."""

    def __init__(self, channels, w_dim, kernel_size, channels_last=False, layer_scale_init=1e-5,
                 demodulate=True, block_index=0, legacy=False):
        super().__init__()
        self.legacy = legacy
        self.channels = channels
        self.kernel_size = kernel_size
        self.affine_pw1 = StyleSplit(w_dim, channels, bias_init=1)
        self.dwconv = nn.Conv2d(channels, channels, kernel_size=kernel_size, padding=kernel_size // 2, groups=channels)
        trunc_normal_(self.dwconv.weight, std=0.02)
        nn.init.constant_(self.dwconv.bias, 0)
        if self.legacy:
            resolution = 8 * 2 ** block_index
            self.register_buffer("noise_const", torch.randn([resolution, resolution]))
            self.noise_strength = nn.Parameter(torch.zeros([]))
        self.pwconv1 = ModulatedPointwiseConv2DLayer(channels, 4 * channels, demodulate)
        self.pwconv2 = nn.Conv2d(4 * channels, channels, kernel_size=1)
        trunc_normal_(self.pwconv2.weight, std=0.02)
        nn.init.zeros_(self.pwconv2.bias)
        self.norm = GroupNorm32(min(32, channels // 4), channels)
        self.act = nn.GELU()
        self.gamma = nn.Parameter(layer_scale_init * torch.ones([1, channels, 1, 1])) if layer_scale_init > 0 else None

    def _noise(self, H, W, split=False):
        """The legacy noise added after the dwconv: noise_const * noise_strength, bilinearly resized to
        H x W (reference convnext_utils.py:131-133). Returns (plane, None) with the product, or with
        split (the GPU path) (resized noise_const, noise_strength) -- resizing is linear, so the same
        math -- so that the dwconv's data-gradient pass over dY also yields the strength's gradient
        sum dY * plane."""
        if not self.legacy:
            return None, None
        if split:
            plane = self.noise_const
            if plane.shape[-2:] != (H, W):
                plane = F.interpolate(plane[None, None], size=(H, W), mode='bilinear', align_corners=False)[0, 0]
            return plane.float(), self.noise_strength
        noise = self.noise_const * self.noise_strength
        if noise.shape[-2:] == (H, W):
            return noise.float(), None        # no [None, None] / [0, 0] round trip: its backward is a zeros + copy
        noise = F.interpolate(noise[None, None], size=(H, W), mode='bilinear', align_corners=False)
        return noise[0, 0].float(), None

    def forward(self, x, w, compute_dtype=None):
        cdt = compute_dtype or x.dtype
        x_in = x
        B, C, H, W = x.shape
        w1 = self.pwconv1.weight.reshape(4 * C, C)
        # style [B, C] = affine_pw1(w), dcoef [B, 4C] = demodulation of pwconv1 (csrc/style.hip on ROCm)
        style, dcoef = decoder_ops.style_and_demod(self.affine_pw1, w, w1 if self.pwconv1.demodulate else None)
        # x feeds the dwconv and the residual: on the HIP path the residual's gradient is added in the
        # dwconv data-gradient kernel instead of by autograd (decoder_hip.ResidualSlot)
        slot = None
        if x.is_cuda and x.dtype == cdt and x.requires_grad and torch.is_grad_enabled():
            from torch_utils.ops import decoder_hip
            slot = decoder_hip.ResidualSlot() if decoder_hip.RESIDUAL_FUSION else None
        plane, strength = self._noise(H, W, split=x.is_cuda)
        d = decoder_ops.dwconv2d(x.to(cdt), self.dwconv.weight, self.dwconv.bias, self.kernel_size // 2,
                                 noise=plane, slot=slot, noise_strength=strength)
        m = decoder_ops.group_norm(d, self.norm.num_groups, self.norm.weight, self.norm.bias, self.norm.eps,
                                   out_dtype=cdt, style=style)                 # GN(d) * s_b
        gamma = self.gamma.reshape(-1) if self.gamma is not None else None
        if decoder_ops.convnext_mlp_fusable(m, C, H * W, x_in):
            # the whole MLP forward in one kernel (hidden 4C tensor on chip without autograd)
            out = decoder_ops.convnext_mlp_nograd(m.reshape(B, C, H * W), w1, dcoef, self.pwconv1.bias.reshape(-1),
                                                  self.pwconv2.weight.reshape(C, 4 * C), self.pwconv2.bias, gamma,
                                                  x_in.reshape(B, C, H * W), slot=slot)
            return out.reshape(B, C, H, W)
        h = decoder_ops.pointwise(w1, m.reshape(B, C, H * W))                    # [B, 4C, HW]
        g = decoder_ops.scale_bias_gelu(h, dcoef, self.pwconv1.bias.reshape(-1))
        y = decoder_ops.pointwise(self.pwconv2.weight.reshape(C, 4 * C), g)     # [B, C, HW]
        out = decoder_ops.layer_scale_residual(y, self.pwconv2.bias, gamma, x_in.reshape(B, C, H * W), slot=slot)
        return out.reshape(B, C, H, W)


class ConvNeXtToRGBLayer(nn.Module):
    """Modulated (no demodulation) 1x1 C -> img_channels + bias (reference :145-187)."""

    def __init__(self, in_channels, out_channels, w_dim, kernel_size=1, channels_last=False):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.kernel_size = kernel_size
        self.channels_last = channels_last
        self.weight = nn.Parameter(torch.randn(out_channels, in_channels, kernel_size, kernel_size) * 0.1)
        self.bias = nn.Parameter(torch.zeros(1, out_channels, 1, 1))
        assert w_dim > 0, "w_dim must be set when use_style=True"
        self.affine = StyleSplit(w_dim, in_channels, bias_init=1)
        self.weight_gain = 1 / np.sqrt(in_channels * kernel_size ** 2)

    def forward(self, x, w):
        B, C, H, W = x.shape
        # the network's grouped launch, else the same style kernel for this layer alone (csrc/style.hip), so
        # the grouped and per-layer results are bit-identical (a captured HIP graph replays the per-layer form)
        style = decoder_ops.style_and_demod(self.affine, w, None)[0] * self.weight_gain    # [B, C]
        if self.kernel_size == 1:
            return decoder_ops.torgb(x, self.weight.reshape(self.out_channels, C), style, self.bias)
        else:
            w_mod = (self.weight[None] * style.reshape(B, 1, -1, 1, 1)).reshape(B * self.out_channels, C,
                                                                               self.kernel_size, self.kernel_size)
            y = F.conv2d(x.reshape(1, B * C, H, W), w_mod.to(x.dtype), groups=B)
            y = y.reshape(B, self.out_channels, y.shape[-2], y.shape[-1])
        return y + self.bias


GAUSSIAN_KERNELS = {
    "3x3": [1, 2, 1],
    "4x4": [1, 3, 3, 1],
    "5x5": [1, 4, 6, 4, 1],
}


class SeparableUpsampleWithFixedBlur(nn.Module):
    """[GN] -> dw3x3 -> 1x1 (C_in -> 4*C_out) -> PixelShuffle(2) -> [GN] -> replicate-pad
    fixed Gaussian blur (reference convnext_utils.py:197-257)."""

    def __init__(self, in_channels, out_channels, upscale_factor=2, blur_kernel="3x3", blur_normalize=True,
                 pad_mode="replicate", pre_normalize=True, use_gaussian_blur=True):
        super().__init__()
        self.out_channels = out_channels
        self.pre_normalize = pre_normalize
        self.use_gaussian_blur = use_gaussian_blur
        self.upscale_factor = upscale_factor
        self.pad_mode = pad_mode
        self.norm = nn.GroupNorm(min(32, in_channels // 4), in_channels) if pre_normalize else \
            nn.GroupNorm(min(32, out_channels // 4), out_channels)
        self.depthwise = nn.Conv2d(in_channels, in_channels, kernel_size=3, padding=1, groups=in_channels, bias=False)
        self.pointwise = nn.Conv2d(in_channels, out_channels * upscale_factor ** 2, kernel_size=1, bias=False)
        self.shuffle = nn.PixelShuffle(upscale_factor)
        self.blur_taps = None
        if self.use_gaussian_blur:
            taps = GAUSSIAN_KERNELS[blur_kernel] if isinstance(blur_kernel, str) else list(blur_kernel)
            assert blur_normalize and pad_mode == "replicate"
            self.blur_taps = [float(t) for t in taps]
            k = torch.tensor(self.blur_taps, dtype=torch.float32)
            k2 = k[:, None] * k[None, :]
            k2 = k2 / k2.sum()
            kh, kw = k2.shape
            ph, pw = (kh - 1) // 2, (kw - 1) // 2
            self.pad = (pw, pw + int(kw % 2 == 0), ph, ph + int(kh % 2 == 0))
            self.register_buffer("blur_weight", k2[None, None].repeat(out_channels, 1, 1, 1))

    def _gn(self, x, out_dtype):
        return decoder_ops.group_norm(x, self.norm.num_groups, self.norm.weight, self.norm.bias, self.norm.eps,
                                      out_dtype=out_dtype)

    def forward(self, x, compute_dtype=None):
        cdt = compute_dtype or x.dtype
        if self.pre_normalize:
            x = self._gn(x, cdt)
        else:
            x = x.to(cdt)
        x = decoder_ops.dwconv2d(x, self.depthwise.weight, None, 1)
        B, C, H, W = x.shape
        x = decoder_ops.pointwise(self.pointwise.weight.reshape(-1, C), x.reshape(B, C, H * W))
        x = x.reshape(B, -1, H, W)
        if self.pre_normalize:
            if self.use_gaussian_blur:
                return decoder_ops.shuffle_blur(x, self.blur_taps, self.upscale_factor)
            return F.pixel_shuffle(x, self.upscale_factor)
        x = F.pixel_shuffle(x, self.upscale_factor)
        x = self._gn(x, cdt)
        if self.use_gaussian_blur:
            x = decoder_ops.blur_replicate(x, self.blur_taps)
        return x
