"""VFM-VAE "Generator" (frozen VFM encoder -> multi-scale fusion -> latent ->
progressive ConvNeXt decoder).

Module API, constructor kwargs (the YAML `G_kwargs` surface), attribute names
and state-dict keys follow the reference `networks/generator.py`
(Generator :915-1206, SynthesisNetwork :655-912, SynthesisBlock :322-579,
MappingNetwork :582-652, legacy StyleGAN layers :46-313), so `train.py`,
`tools/reconstruct` and `tools/decode` drop in unchanged and released
checkpoints load.

MI355X-specific choices (documented deviations):
  * Mixed precision is explicit per block: blocks with index >= num_blocks -
    num_fp16_res run in `amp_dtype` (bf16 by default on MI355X: same MFMA rate
    as fp16, fp32 range; pass amp_dtype='float16' for the reference's fp16),
    the others in fp32 (reference :499-517, :703).
  * `set_train_mode('train_the_second_half_decoder')` trains the blocks whose
    resolution is > 32 (and their z-convs). The reference builds module names
    `synthesis.b64` etc. that match nothing (:1109-1116), which leaves G with no
    trainable parameter; this build implements the evident intent.
    `freeze32` (called by the PatchGAN warm-up, reference loss.py:486-488, but
    undefined there) is the same mode.
"""
from typing import Any, List, Optional, Union

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn.parameter import Parameter

from torch_utils import misc
from torch_utils import distributed as dist
from torch_utils.ops import upfirdn2d, conv2d_resample, bias_act, fma, style_group
from networks.utils.shared import FullyConnectedLayer, MLP, GroupNorm32, StyleSplit, ScaleAdaptiveAvgPool2d
from networks.utils.shared import DepthwiseConv2d, Conv1x1, LeakyReLU
from networks.utils.ldm_utils import LDMAdapter, EquivarianceTransform
from networks.utils.gigagan_utils import SelfAttentionBlock, CrossAttentionBlock
from networks.utils.convnext_utils import ConvNeXtSynthesisLayer, ConvNeXtToRGBLayer, SeparableUpsampleWithFixedBlur
from networks.utils.dataclasses import EncodeOutput, GeneratorForwardOutput
from networks.utils.vfm_utils import VFMEncoder

_DTYPES = {'float16': torch.float16, 'fp16': torch.float16, 'bfloat16': torch.bfloat16, 'bf16': torch.bfloat16,
           'float32': torch.float32}


def _as_dtype(d):
    return _DTYPES[d] if isinstance(d, str) else d


def normalize_2nd_moment(x, dim=1, eps=1e-8):
    return x * (x.square().mean(dim=dim, keepdim=True) + eps).rsqrt()


# ---------------------------------------------------------------------------
# Legacy StyleGAN-T layers (built only when use_convnext=False). They are the
# callers of the StyleGAN-lineage ops (conv2d_resample / bias_act / fma /
# upfirdn2d), which run on the HIP kernels.


def modulated_conv2d(x, weight, styles, noise=None, up=1, down=1, padding=0, resample_filter=None, demodulate=True,
                     flip_weight=True, fused_modconv=True):
    """StyleGAN2 modulated conv (reference generator.py:46-103)."""
    batch_size = x.shape[0]
    out_channels, in_channels, kh, kw = weight.shape
    misc.assert_shape(weight, [out_channels, in_channels, kh, kw])
    misc.assert_shape(x, [batch_size, in_channels, None, None])
    misc.assert_shape(styles, [batch_size, in_channels])
    if x.dtype == torch.float16 and demodulate:   # keep fp16 in range
        weight = weight * (1 / np.sqrt(in_channels * kh * kw) / weight.norm(float('inf'), dim=[1, 2, 3], keepdim=True))
        styles = styles / styles.norm(float('inf'), dim=1, keepdim=True)
    w = dcoefs = None
    if demodulate or fused_modconv:
        w = weight.unsqueeze(0) * styles.reshape(batch_size, 1, -1, 1, 1)
    if demodulate:
        dcoefs = (w.square().sum(dim=[2, 3, 4]) + 1e-8).rsqrt()
    if demodulate and fused_modconv:
        w = w * dcoefs.reshape(batch_size, -1, 1, 1, 1)
    if not fused_modconv:
        x = x * styles.to(x.dtype).reshape(batch_size, -1, 1, 1)
        x = conv2d_resample.conv2d_resample(x=x, w=weight.to(x.dtype), f=resample_filter, up=up, down=down,
                                            padding=padding, flip_weight=flip_weight)
        if demodulate and noise is not None:
            return fma.fma(x, dcoefs.to(x.dtype).reshape(batch_size, -1, 1, 1), noise.to(x.dtype))
        if demodulate:
            return x * dcoefs.to(x.dtype).reshape(batch_size, -1, 1, 1)
        if noise is not None:
            return x.add_(noise.to(x.dtype))
        return x
    x = x.reshape(1, -1, *x.shape[2:])
    w = w.reshape(-1, in_channels, kh, kw)
    x = conv2d_resample.conv2d_resample(x=x, w=w.to(x.dtype), f=resample_filter, up=up, down=down, padding=padding,
                                        groups=batch_size, flip_weight=flip_weight)
    x = x.reshape(batch_size, -1, *x.shape[2:])
    if noise is not None:
        x = x.add_(noise)
    return x


class SynthesisInput(nn.Module):
    """Fourier-feature input layer (reference generator.py:106-172)."""

    def __init__(self, w_dim, channels, size, sampling_rate, bandwidth):
        super().__init__()
        self.w_dim = w_dim
        self.channels = channels
        self.size = np.broadcast_to(np.asarray(size), [2])
        self.sampling_rate = sampling_rate
        self.bandwidth = bandwidth
        freqs = torch.randn([channels, 2])
        radii = freqs.square().sum(dim=1, keepdim=True).sqrt()
        freqs /= radii * radii.square().exp().pow(0.25)
        freqs *= bandwidth
        phases = torch.rand([channels]) - 0.5
        self.weight = Parameter(torch.randn([channels, channels]))
        self.affine = FullyConnectedLayer(w_dim, 4, weight_init=0, bias_init=[1, 0, 0, 0])
        self.register_buffer('transform', torch.eye(3, 3))
        self.register_buffer('freqs', freqs)
        self.register_buffer('phases', phases)

    def forward(self, w):
        B = w.shape[0]
        t = self.affine(w)
        t = t / t[:, :2].norm(dim=1, keepdim=True)
        m_r = torch.eye(3, device=w.device).unsqueeze(0).repeat([B, 1, 1])
        m_r[:, 0, 0], m_r[:, 0, 1], m_r[:, 1, 0], m_r[:, 1, 1] = t[:, 0], -t[:, 1], t[:, 1], t[:, 0]
        m_t = torch.eye(3, device=w.device).unsqueeze(0).repeat([B, 1, 1])
        m_t[:, 0, 2], m_t[:, 1, 2] = -t[:, 2], -t[:, 3]
        transforms = m_r @ m_t @ self.transform.unsqueeze(0)
        freqs = self.freqs.unsqueeze(0)
        phases = self.phases.unsqueeze(0) + (freqs @ transforms[:, :2, 2:]).squeeze(2)
        freqs = freqs @ transforms[:, :2, :2]
        amplitudes = (1 - (freqs.norm(dim=2) - self.bandwidth) / (self.sampling_rate / 2 - self.bandwidth)).clamp(0, 1)
        theta = torch.eye(2, 3, device=w.device)
        theta[0, 0] = 0.5 * self.size[0] / self.sampling_rate
        theta[1, 1] = 0.5 * self.size[1] / self.sampling_rate
        grids = F.affine_grid(theta.unsqueeze(0), [1, 1, int(self.size[1]), int(self.size[0])], align_corners=False)
        x = (grids.unsqueeze(3) @ freqs.permute(0, 2, 1).unsqueeze(1).unsqueeze(2)).squeeze(3)
        x = torch.sin((x + phases.unsqueeze(1).unsqueeze(2)) * (np.pi * 2)) * amplitudes.unsqueeze(1).unsqueeze(2)
        x = x @ (self.weight / np.sqrt(self.channels)).t()
        return x.permute(0, 3, 1, 2).contiguous()


class SynthesisLayer(nn.Module):
    """Legacy modulated 3x3 conv layer (reference generator.py:175-284)."""

    def __init__(self, in_channels, out_channels, w_dim, resolution, kernel_size=3, up=1, use_noise=True,
                 activation='lrelu', resample_filter=[1, 3, 3, 1], conv_clamp=None, channels_last=False,
                 layer_scale_init=1e-5, residual=False, gn_groups=32):
        super().__init__()
        if residual:
            assert in_channels == out_channels
        self.in_channels, self.out_channels, self.w_dim = in_channels, out_channels, w_dim
        self.resolution, self.up, self.use_noise = resolution, up, use_noise
        self.activation, self.conv_clamp = activation, conv_clamp
        self.register_buffer('resample_filter', upfirdn2d.setup_filter(resample_filter))
        self.padding = kernel_size // 2
        self.act_gain = bias_act.activation_funcs[activation].def_gain
        self.residual = residual
        if use_noise:
            self.register_buffer('noise_const', torch.randn([resolution, resolution]))
            self.noise_strength = Parameter(torch.zeros([]))
        self.affine = StyleSplit(w_dim, in_channels, bias_init=1)
        mf = torch.channels_last if channels_last else torch.contiguous_format
        self.weight = Parameter(torch.randn([out_channels, in_channels, kernel_size, kernel_size]).to(memory_format=mf))
        self.bias = Parameter(torch.zeros([out_channels]))
        if residual:
            assert up == 1
            self.norm = GroupNorm32(gn_groups, out_channels)
            self.gamma = Parameter(layer_scale_init * torch.ones([1, out_channels, 1, 1])).to(memory_format=mf)

    def forward(self, x, w, noise_mode='const', fused_modconv=True, gain=1):
        dtype = x.dtype
        misc.assert_shape(x, [None, self.in_channels, self.resolution // self.up, self.resolution // self.up])
        noise = None
        if self.use_noise and noise_mode == 'random':
            noise = torch.randn([x.shape[0], 1, self.resolution, self.resolution], device=x.device) * self.noise_strength
        if self.use_noise and noise_mode == 'const':
            noise = self.noise_const * self.noise_strength
        styles = self.affine(w)
        if self.residual:
            x = self.norm(x)
        y = modulated_conv2d(x=x, weight=self.weight, styles=styles, noise=noise, up=self.up, fused_modconv=fused_modconv,
                             padding=self.padding, resample_filter=self.resample_filter, flip_weight=(self.up == 1))
        y = y.to(dtype)
        act_clamp = self.conv_clamp * gain if self.conv_clamp is not None else None
        y = bias_act.bias_act(y, self.bias.to(x.dtype), act=self.activation, gain=self.act_gain * gain, clamp=act_clamp)
        if self.residual:
            y = (self.gamma * y).to(dtype).add_(x).mul(np.sqrt(2))
        return y


class ToRGBLayer(nn.Module):
    """Legacy modulated (no demod) ToRGB (reference generator.py:287-313)."""

    def __init__(self, in_channels, out_channels, w_dim, kernel_size=1, conv_clamp=None, channels_last=False):
        super().__init__()
        self.in_channels, self.out_channels, self.w_dim = in_channels, out_channels, w_dim
        self.conv_clamp = conv_clamp
        self.affine = StyleSplit(w_dim, in_channels, bias_init=1)
        mf = torch.channels_last if channels_last else torch.contiguous_format
        self.weight = Parameter(0.1 * torch.randn([out_channels, in_channels, kernel_size, kernel_size]).to(memory_format=mf))
        self.bias = Parameter(torch.zeros([out_channels]))
        self.weight_gain = 1 / np.sqrt(in_channels * (kernel_size ** 2))

    def forward(self, x, w):
        styles = self.affine(w) * self.weight_gain
        x = modulated_conv2d(x=x, weight=self.weight, styles=styles, demodulate=False)
        return bias_act.bias_act(x, self.bias.to(x.dtype), clamp=self.conv_clamp)


# ---------------------------------------------------------------------------
# VFM-VAE decoder.


class SynthesisBlock(nn.Module):
    def __init__(self, block_index, in_channels, out_channels, last_out_channels, c_dim, w_dim, resolution,
                 img_channels, is_first, is_last, num_res_blocks=1, use_multiscale_output=False, architecture='skip',
                 resample_filter=[1, 3, 3, 1], conv_clamp=None, use_fp16=False, fp16_channels_last=False,
                 fused_modconv_default='inference_only', attn_block_indices=[], attn_depths=[], use_self_attn=False,
                 use_cross_attn=False, attn_heads=8, attn_ff_mult=4, use_convnext=False, use_gaussian_blur=True,
                 add_additional_convnext=False, legacy=False, amp_dtype=torch.bfloat16, **layer_kwargs):
        assert architecture in ['orig', 'skip']
        super().__init__()
        self.block_index = block_index
        self.in_channels, self.out_channels, self.last_out_channels = in_channels, out_channels, last_out_channels
        self.c_dim, self.w_dim, self.resolution, self.img_channels = c_dim, w_dim, resolution, img_channels
        self.is_last, self.architecture = is_last, architecture
        self.use_fp16 = use_fp16
        self.amp_dtype = amp_dtype
        self.channels_last = use_fp16 and fp16_channels_last
        self.num_conv = 0
        self.num_torgb = 0
        assert architecture == 'skip' if use_multiscale_output else True
        self.use_multiscale_output = use_multiscale_output
        self.use_convnext = use_convnext
        self.add_additional_convnext = add_additional_convnext
        if not use_convnext:
            self.fused_modconv_default = fused_modconv_default
            self.register_buffer('resample_filter', upfirdn2d.setup_filter(resample_filter))
        kernel_size = 5 if block_index <= 1 else 7
        self.kernel_size = kernel_size
        blur_kernel = "3x3" if block_index <= 2 else "5x5"

        if in_channels == 0:
            self.input = SynthesisInput(w_dim=w_dim, channels=out_channels, size=resolution, sampling_rate=resolution,
                                        bandwidth=2)
            self.num_conv += 1
        else:
            if use_convnext:
                self.seperate_upsample_conv = SeparableUpsampleWithFixedBlur(
                    in_channels, out_channels, upscale_factor=2, pre_normalize=not is_first,
                    use_gaussian_blur=use_gaussian_blur, blur_kernel=blur_kernel)
                self.conv0 = ConvNeXtSynthesisLayer(out_channels, w_dim=w_dim, kernel_size=kernel_size,
                                                    channels_last=self.channels_last, block_index=block_index,
                                                    legacy=legacy)
            else:
                self.conv0 = SynthesisLayer(in_channels, out_channels, w_dim=w_dim, resolution=resolution, up=2,
                                            resample_filter=resample_filter, conv_clamp=conv_clamp,
                                            channels_last=self.channels_last, **layer_kwargs)
            self.num_conv += 1

        convs = []
        for _ in range(num_res_blocks):
            if use_convnext:
                n_layers = 3 if block_index <= 3 and add_additional_convnext else 2
                for _ in range(n_layers):
                    convs.append(ConvNeXtSynthesisLayer(out_channels, w_dim=w_dim, kernel_size=kernel_size,
                                                        channels_last=self.channels_last, block_index=block_index,
                                                        legacy=legacy))
            else:
                convs.append(SynthesisLayer(out_channels, out_channels, w_dim=w_dim, resolution=resolution,
                                            conv_clamp=conv_clamp, channels_last=self.channels_last, **layer_kwargs))
                convs.append(SynthesisLayer(out_channels, out_channels, w_dim=w_dim, resolution=resolution,
                                            conv_clamp=conv_clamp, channels_last=self.channels_last, residual=True,
                                            **layer_kwargs))
        self.convs1 = nn.ModuleList(convs)
        self.num_conv += len(convs)

        if is_last or architecture == 'skip':
            if use_convnext:
                self.torgb = ConvNeXtToRGBLayer(out_channels, img_channels, w_dim=w_dim, channels_last=self.channels_last)
            else:
                self.torgb = ToRGBLayer(out_channels, img_channels, w_dim=w_dim, conv_clamp=conv_clamp,
                                        channels_last=self.channels_last)
            self.num_torgb += 1

        if use_multiscale_output and last_out_channels is not None:
            self.last_upsample_conv = SeparableUpsampleWithFixedBlur(last_out_channels, out_channels, upscale_factor=2,
                                                                     use_gaussian_blur=use_gaussian_blur,
                                                                     blur_kernel=blur_kernel)

        self.attn_block_indices, self.attn_depths = attn_block_indices, attn_depths
        self.use_self_attn, self.use_cross_attn = use_self_attn, use_cross_attn
        self.attn_heads, self.attn_ff_mult = attn_heads, attn_ff_mult
        depth = attn_depths[attn_block_indices.index(block_index)] if block_index in attn_block_indices else 0
        self.has_self_attn = use_self_attn and depth > 0
        self.has_cross_attn = use_cross_attn and depth > 0
        self.self_attns = nn.ModuleList([
            SelfAttentionBlock(out_channels, dim_head=out_channels // attn_heads, heads=attn_heads, ff_mult=attn_ff_mult)
            for _ in range(depth)]) if self.has_self_attn else None
        self.cross_attns = nn.ModuleList([
            CrossAttentionBlock(out_channels, dim_context=c_dim, dim_head=out_channels // attn_heads, heads=attn_heads,
                                ff_mult=attn_ff_mult)
            for _ in range(depth)]) if self.has_cross_attn else None

    def compute_dtype(self, device, force_fp32=False):
        if device.type != 'cuda' or force_fp32 or not self.use_fp16:
            return torch.float32
        return self.amp_dtype

    def forward(self, x, x_sum, img, ws, text, text_mask, force_fp32=False, fused_modconv=True, **layer_kwargs):
        w_iter = iter(ws.unbind(dim=1))
        dtype = self.compute_dtype(ws.device, force_fp32)
        if self.in_channels == 0:
            x = self.input(next(w_iter))
        x = x.to(dtype=dtype)

        if self.use_convnext:
            x = self.seperate_upsample_conv(x, compute_dtype=dtype)
            x = self.conv0(x, next(w_iter), compute_dtype=dtype)
            for conv in self.convs1:
                x = conv(x, next(w_iter), compute_dtype=dtype)
        else:
            if fused_modconv is None or fused_modconv == 'inference_only':
                fused_modconv = not self.training
            amp = torch.autocast(device_type='cuda', dtype=dtype, enabled=(dtype != torch.float32))
            with amp:
                if self.in_channels == 0:
                    for conv in self.convs1:
                        x = conv(x, next(w_iter), fused_modconv=fused_modconv, gain=np.sqrt(0.5), **layer_kwargs)
                else:
                    x = self.conv0(x, next(w_iter), fused_modconv=fused_modconv, **layer_kwargs)
                    for conv in self.convs1:
                        x = conv(x, next(w_iter), fused_modconv=fused_modconv, gain=np.sqrt(0.5), **layer_kwargs)

        if self.has_self_attn or self.has_cross_attn:
            with torch.autocast(device_type='cuda', dtype=dtype, enabled=(dtype != torch.float32 and x.is_cuda)):
                if self.has_self_attn:
                    for attn in self.self_attns:
                        x = attn(x)
                if self.has_cross_attn:
                    assert text is not None, "Text input must be provided for cross-attention."
                    for attn in self.cross_attns:
                        x = attn(x, text, mask=text_mask)
        x = x.to(dtype=dtype)

        if self.use_multiscale_output:
            if self.last_out_channels is not None:
                x_sum = self.last_upsample_conv(x_sum, compute_dtype=dtype) + x
            else:
                x_sum = x
            img = self.torgb(x_sum, next(w_iter)).to(dtype=torch.float32, memory_format=torch.contiguous_format)
        else:
            if img is not None:
                misc.assert_shape(img, [None, self.img_channels, self.resolution // 2, self.resolution // 2])
                img = upfirdn2d.upsample2d(img, self.resample_filter)
            if self.is_last or self.architecture == 'skip':
                y = self.torgb(x, next(w_iter)).to(dtype=torch.float32, memory_format=torch.contiguous_format)
                img = img.add_(y) if img is not None else y
        assert x.dtype == dtype
        assert img is None or img.dtype == torch.float32
        return x, x_sum, img

    def extra_repr(self):
        return f'resolution={self.resolution:d}, architecture={self.architecture:s}'


class MappingNetwork(nn.Module):
    def __init__(self, z_dim_input, z_dim_output, c_dim, w_dim, label_type, num_layers=2, activation='lrelu',
                 lr_multiplier=0.01, x_avg_beta=0.995):
        super().__init__()
        self.z_dim_input, self.z_dim_output = z_dim_input, z_dim_output
        self.c_dim, self.w_dim = c_dim, w_dim
        self.x_avg_beta = x_avg_beta
        self.num_ws = None
        self.label_type = label_type
        if label_type in ['text', 'cls2text']:
            self.mlp = MLP([z_dim_input] * num_layers + [z_dim_output], activation=activation,
                           lr_multiplier=lr_multiplier, linear_out=True)
            self.register_buffer('x_avg', torch.zeros([z_dim_output], dtype=torch.float32))
        elif label_type == 'cls2id':
            assert z_dim_input < w_dim, 'z_dim must be less than w_dim for cls2id.'
            c_embed_dim = 1024
            self.embed = FullyConnectedLayer(c_dim, c_embed_dim) if c_dim > 0 else None
            feats = [z_dim_input + c_embed_dim] * num_layers + [w_dim] if c_dim > 0 else [z_dim_input] * num_layers + [w_dim]
            self.mlp = MLP(feats, activation=activation, lr_multiplier=lr_multiplier, linear_out=True)
            self.register_buffer('x_avg', torch.zeros([w_dim], dtype=torch.float32))

    def forward(self, z, c, truncation_psi=1.0):
        if self.label_type in ['text', 'cls2text']:
            x = self.mlp(normalize_2nd_moment(z))
        else:
            x = self.mlp(torch.cat([normalize_2nd_moment(z), normalize_2nd_moment(self.embed(c))], dim=1)) \
                if self.c_dim > 0 else self.mlp(normalize_2nd_moment(z))
        if self.x_avg_beta is not None and self.training:
            self.x_avg.copy_(x.detach().mean(0).lerp(self.x_avg, self.x_avg_beta))
        if truncation_psi != 1:
            assert self.x_avg_beta is not None
            x = self.x_avg.lerp(x, truncation_psi)
        if self.label_type in ['text', 'cls2text'] and self.c_dim > 0:
            w = torch.cat([x, F.normalize(c, dim=1)], dim=1)
        else:
            w = x
        if self.num_ws is not None:
            w = w.unsqueeze(1).repeat([1, self.num_ws, 1])
        return w


class SynthesisNetwork(nn.Module):
    def __init__(self, c_dim, w_dim, img_resolution, img_channels=3, channel_base=32768, channel_max=512,
                 num_fp16_res=3, conv_clamp=None, num_blocks=6, num_res_blocks=3, z_resolution=16, z_dim=8,
                 concat_z_block_indices=[], concat_z_mapped_dims=[], how_to_process_concat_z='unshuffle',
                 activation_for_concat_z='gelu', use_multiscale_output=False, attn_block_indices=[], attn_depths=[],
                 use_self_attn=False, use_cross_attn=False, use_convnext=False, use_gaussian_blur=True,
                 add_additional_convnext=False, legacy=False, amp_dtype='bfloat16', **block_kwargs):
        assert img_resolution >= 4
        super().__init__()
        self.c_dim, self.w_dim = c_dim, w_dim
        self.img_resolution = img_resolution
        self.img_resolution_log2 = int(np.log2(img_resolution))
        self.img_channels = img_channels
        self.num_blocks = num_blocks
        res_start = img_resolution // (2 ** (num_blocks - 1))
        self.block_resolutions = [res_start * (2 ** i) for i in range(num_blocks)]
        scale = img_resolution / 256
        channels = {i: min(channel_base // int(r / scale), channel_max) for i, r in enumerate(self.block_resolutions)}
        self.amp_dtype = _as_dtype(amp_dtype)
        self.num_fp16_res = num_fp16_res
        fp16_idx = num_blocks - num_fp16_res
        self.z_resolution, self.z_dim = z_resolution, z_dim
        self.concat_z_block_indices = concat_z_block_indices
        self.concat_z_mapped_dims = concat_z_mapped_dims
        self.how_to_process_concat_z = how_to_process_concat_z
        self.activation_for_concat_z = activation_for_concat_z
        self.use_multiscale_output = use_multiscale_output
        self.attn_block_indices = attn_block_indices
        self.use_self_attn, self.use_cross_attn = use_self_attn, use_cross_attn

        self.z_convs = nn.ModuleDict()
        self.adjust_concat_z_dims = dict()
        for idx in concat_z_block_indices:
            res = self.block_resolutions[idx]
            mapped = concat_z_mapped_dims[idx] if len(concat_z_mapped_dims) > 0 else None
            act = activation_for_concat_z
            if res < z_resolution * 2:
                factor = int(z_resolution / res * 2)
                if how_to_process_concat_z == 'unshuffle':
                    cin = int(z_dim * factor ** 2)
                    out = mapped if mapped is not None else cin
                    layers = [nn.PixelUnshuffle(factor), self._make_3x3_conv(cin, out, activation=act),
                              self._make_1x1_conv(out, out, use_activation=False)]
                else:
                    out = mapped if mapped is not None else z_dim
                    layers = [ScaleAdaptiveAvgPool2d(factor), self._make_3x3_conv(z_dim, out, activation=act),
                              self._make_1x1_conv(out, out, use_activation=False)]
            elif res == z_resolution * 2:
                out = mapped if mapped is not None else z_dim
                layers = [self._make_3x3_conv(z_dim, out, activation=act), self._make_1x1_conv(out, out, use_activation=False)]
            else:
                factor = int(res / z_resolution / 2)
                out = mapped if mapped is not None else z_dim
                layers = [self._make_3x3_conv(z_dim, int(out * factor ** 2), activation=act), nn.PixelShuffle(factor),
                          self._make_1x1_conv(out, out, use_activation=False)]
            self.z_convs[f"{idx:01d}"] = nn.Sequential(*layers)
            self.adjust_concat_z_dims[idx] = out

        self.blocks = nn.ModuleDict()
        self.num_ws = 0
        for idx in range(num_blocks):
            in_channels = channels[idx - 1] if idx > 0 else 0
            last_out = channels[idx - 1] if idx > 0 else None
            if idx in concat_z_block_indices:
                in_channels += self.adjust_concat_z_dims[idx]
            block = SynthesisBlock(
                block_index=idx, in_channels=in_channels, out_channels=channels[idx], last_out_channels=last_out,
                c_dim=c_dim, w_dim=w_dim, resolution=self.block_resolutions[idx], img_channels=img_channels,
                is_first=(idx == 0), is_last=(idx == num_blocks - 1), use_fp16=(idx >= fp16_idx),
                conv_clamp=conv_clamp, num_res_blocks=num_res_blocks, use_multiscale_output=use_multiscale_output,
                use_convnext=use_convnext, use_gaussian_blur=use_gaussian_blur,
                add_additional_convnext=add_additional_convnext, legacy=legacy, attn_block_indices=attn_block_indices,
                attn_depths=attn_depths, use_self_attn=use_self_attn, use_cross_attn=use_cross_attn,
                amp_dtype=self.amp_dtype, **block_kwargs)
            self.num_ws += block.num_conv + block.num_torgb
            self.blocks[f"{idx:01d}"] = block

    def _make_3x3_conv(self, cin, cout, activation='gelu', use_activation=True):
        # HIP depthwise / 1x1 GEMM / GroupNorm / LReLU (same modules and state-dict keys as nn.*)
        layers = [DepthwiseConv2d(cin, cin, 3, padding=1, groups=cin, bias=False), Conv1x1(cin, cout, 1, bias=False),
                  GroupNorm32(min(32, cout), cout)]
        if use_activation:
            layers += [{'lrelu': lambda: LeakyReLU(negative_slope=0.2), 'silu': nn.SiLU, 'gelu': nn.GELU}[activation]()]
        return nn.Sequential(*layers)

    def _make_1x1_conv(self, cin, cout, activation='gelu', use_activation=True):
        layers = [Conv1x1(cin, cout, 1, bias=False), GroupNorm32(min(32, cout), cout)]
        if use_activation:
            layers += [{'lrelu': lambda: LeakyReLU(negative_slope=0.2), 'silu': nn.SiLU, 'gelu': nn.GELU}[activation]()]
        return nn.Sequential(*layers)

    def forward(self, z, ws, text, text_mask, **block_kwargs):
        with torch.autograd.profiler.record_function('split_ws'):
            ws = ws.to(torch.float32)
            block_ws, w_idx = [], 0
            for idx in range(self.num_blocks):
                b = self.blocks[f"{idx:01d}"]
                block_ws.append(ws.narrow(1, w_idx, b.num_conv + b.num_torgb))
                w_idx += b.num_conv + b.num_torgb
        x = x_sum = img = None
        multiscale = []
        # every layer's style (+ demodulation) in one grouped launch per phase on ROCm (torch_utils/ops/style_group.py)
        with style_group.StyleGroup(self, ws):
            img, multiscale = self._blocks(z, block_ws, text, text_mask, **block_kwargs)
        return img, multiscale[::-1]

    def _blocks(self, z, block_ws, text, text_mask, **block_kwargs):
        x = x_sum = img = None
        multiscale = []
        for idx, cur_ws in enumerate(block_ws):
            block = self.blocks[f"{idx:01d}"]
            if idx in self.concat_z_block_indices:
                dt = block.compute_dtype(z.device)
                with torch.autocast(device_type='cuda', dtype=dt, enabled=(dt != torch.float32 and z.is_cuda)):
                    zc = self.z_convs[f"{idx:01d}"](z)
                x = torch.cat([x, zc.to(x.dtype) if x.dtype == torch.float32 else zc], dim=1) if x is not None else zc
            x, x_sum, img = block(x, x_sum, img, cur_ws, text, text_mask, **block_kwargs)
            if not block.is_last:
                multiscale.append(img)
        return img, multiscale

    def extra_repr(self):
        return (f'w_dim={self.w_dim:d}, num_ws={self.num_ws:d}, img_resolution={self.img_resolution:d}, '
                f'img_channels={self.img_channels:d}, num_fp16_res={self.num_fp16_res:d}')


class Generator(nn.Module):
    def __init__(self, conditional: bool, label_type: str, label_dim: Optional[int], vfm_name: str, scale_factor: float,
                 patch_from_layers: List[int], patch_in_dimensions: List[int], patch_out_dimensions: List[int],
                 compression_mode: str, how_to_compress: str, how_to_decompress: str, decompress_factor: int,
                 attnproj_quant_layers: int = 1, attnproj_post_quant_layers: int = 1,
                 resolution_compression_factor: int = 16, z_dimension: int = 32, vocab_width: int = 64,
                 z_pooled_resolution: int = 1, z_dim_for_mapping_mlp_output: int = 128, vocab_size: int = 32768,
                 vocab_beta: float = 0.25, use_entropy_loss: bool = False, entropy_temp: float = 0.01,
                 num_codebooks: int = 8, use_kl_loss: bool = False, use_vf_loss: bool = False,
                 use_adaptive_vf_loss: bool = False, distmat_margin: float = 0.0, cos_margin: float = 0.0,
                 distmat_weight: float = 1.0, cos_weight: float = 1.0, concat_z_block_indices: list = [],
                 concat_z_mapped_dims: list = [], how_to_process_concat_z: str = 'unshuffle',
                 activation_for_concat_z: str = 'gelu', use_multiscale_output: bool = True,
                 attn_block_indices: list = [], attn_depths: list = [], use_self_attn: bool = True,
                 use_cross_attn: bool = False, use_convnext: bool = True, use_gaussian_blur: bool = True,
                 add_additional_convnext: bool = True, use_equivariance_regularization: bool = False,
                 equivariance_regularization_p_prior: float = 0.5,
                 equivariance_regularization_p_prior_scale: float = 0.25, img_resolution: int = 256,
                 img_channels: int = 3, train_mode: str = 'train_all', num_blocks: int = 6, num_fp16_res: int = 3,
                 conv_clamp: Optional[int] = 256, legacy: bool = False, synthesis_kwargs: dict = {},
                 amp_dtype: str = 'bfloat16'):
        super().__init__()
        self.conditional = conditional
        self.label_type = label_type
        self.num_blocks = num_blocks
        self.img_resolution = img_resolution
        self.img_channels = img_channels
        self.vfm_encoder = VFMEncoder(model_name=vfm_name, conditional=conditional, label_type=label_type,
                                      scale_factor=scale_factor, patch_from_layers=patch_from_layers)
        ps = self.vfm_encoder.patch_size
        self.patch_resolutions = [int(img_resolution * scale_factor // ps) for _ in patch_from_layers]
        assert img_resolution * scale_factor % ps == 0, \
            f'Image resolution {img_resolution * scale_factor} must be divisible by the VFM patch size {ps}.'
        self.z_resolution = int(img_resolution // resolution_compression_factor)
        self.z_dim = z_dimension if compression_mode == 'continuous' else vocab_width
        self.z_pooled_resolution = z_pooled_resolution
        self.z_dim_for_mapping = self.z_dim * decompress_factor * z_pooled_resolution ** 2
        self.z_dim_for_concatenated = self.z_dim * decompress_factor
        self.z_dim_for_mapping_mlp_output = z_dim_for_mapping_mlp_output
        if conditional:
            if label_type in ['text', 'cls2text']:
                self.c_dim = self.vfm_encoder.encoder.text_model.config.hidden_size
                self.z_dim_for_mapping_mlp_input = self.z_dim_for_mapping
                self.w_dim = z_dim_for_mapping_mlp_output + self.c_dim
            elif label_type == 'cls2id':
                self.label_dim = label_dim
                self.c_dim = label_dim
                self.c_embed_dim = 1024
                self.z_dim_for_mapping_mlp_input = self.z_dim_for_mapping + self.c_embed_dim
                self.w_dim = z_dim_for_mapping_mlp_output
        else:
            self.c_dim = 0
            self.z_dim_for_mapping_mlp_input = self.z_dim_for_mapping
            self.w_dim = z_dim_for_mapping_mlp_output

        self.ldm_adapter = LDMAdapter(
            patch_from_layers=patch_from_layers, patch_resolutions=self.patch_resolutions,
            patch_in_dimensions=patch_in_dimensions, patch_out_dimensions=patch_out_dimensions,
            compression_mode=compression_mode, how_to_compress=how_to_compress, how_to_decompress=how_to_decompress,
            decompress_factor=decompress_factor, attnproj_quant_layers=attnproj_quant_layers,
            attnproj_post_quant_layers=attnproj_post_quant_layers, z_resolution=self.z_resolution,
            z_dimension=z_dimension, vocab_width=vocab_width, vocab_size=vocab_size, vocab_beta=vocab_beta,
            use_entropy_loss=use_entropy_loss, entropy_temp=entropy_temp, num_codebooks=num_codebooks,
            use_kl_loss=use_kl_loss, use_vf_loss=use_vf_loss, use_adaptive_vf_loss=use_adaptive_vf_loss,
            distmat_margin=distmat_margin, cos_margin=cos_margin, distmat_weight=distmat_weight, cos_weight=cos_weight)
        self.concat_z_block_indices = concat_z_block_indices
        self.concat_z_mapped_dims = concat_z_mapped_dims
        self.use_multiscale_output = use_multiscale_output
        self.equivariance_transform = EquivarianceTransform(apply=use_equivariance_regularization,
                                                            p_eq_prior=equivariance_regularization_p_prior,
                                                            p_eq_prior_scale=equivariance_regularization_p_prior_scale)
        self.mapping = MappingNetwork(z_dim_input=self.z_dim_for_mapping_mlp_input,
                                      z_dim_output=self.z_dim_for_mapping_mlp_output, c_dim=self.c_dim, w_dim=self.w_dim,
                                      label_type=self.label_type)
        self.synthesis = SynthesisNetwork(
            z_resolution=self.z_resolution, z_dim=self.z_dim_for_concatenated, c_dim=self.c_dim, w_dim=self.w_dim,
            img_resolution=img_resolution, img_channels=img_channels, concat_z_block_indices=concat_z_block_indices,
            concat_z_mapped_dims=concat_z_mapped_dims, how_to_process_concat_z=how_to_process_concat_z,
            activation_for_concat_z=activation_for_concat_z, attn_block_indices=attn_block_indices,
            attn_depths=attn_depths, use_self_attn=use_self_attn, use_cross_attn=use_cross_attn,
            use_convnext=use_convnext, use_gaussian_blur=use_gaussian_blur,
            add_additional_convnext=add_additional_convnext, use_multiscale_output=use_multiscale_output,
            num_blocks=num_blocks, num_fp16_res=num_fp16_res, conv_clamp=conv_clamp, legacy=legacy,
            amp_dtype=amp_dtype, **synthesis_kwargs)
        self.num_ws = self.synthesis.num_ws
        self.mapping.num_ws = self.num_ws
        self.set_train_mode(train_mode)

    def set_train_mode(self, mode: str):
        if mode == 'train_all':
            layers = ['synthesis', 'mapping.mlp', 'ldm_adapter']
            if self.conditional and self.label_type == 'cls2id':
                layers.append('mapping.embed')
        elif mode == 'train_text_encoder':
            layers = ['clip']
        elif mode in ('train_the_second_half_decoder', 'freeze32'):
            layers = [f'synthesis.blocks.{i}' for i, r in enumerate(self.synthesis.block_resolutions) if r > 32]
            layers += [f'synthesis.z_convs.{i}' for i in self.concat_z_block_indices
                       if self.synthesis.block_resolutions[i] > 32]
        elif mode == 'train_decoder':
            layers = ['synthesis', 'mapping.mlp', 'ldm_adapter.post_quant']
            if self.conditional and self.label_type == 'cls2id':
                layers.append('mapping.embed')
        else:
            raise ValueError(f"Unknown train_mode {mode}")
        self.train_mode = mode
        self.trainable_layers = layers
        dist.print0(f"[Generator] train_mode set to {mode}.")

    @torch.no_grad()
    def encode(self, img, return_z_before_quantize=False, eq_scale_factor: float = 1.0, is_eq_prior: bool = False):
        feats, *_ = self.vfm_encoder.encode_image(img, eq_scale_factor=eq_scale_factor, is_eq_prior=is_eq_prior)
        return self.ldm_adapter.encode(feats, return_z_before_quantize).z

    @torch.no_grad()
    def decode(self, z, c=None, truncation_psi=1.0, **synthesis_kwargs):
        z = self.ldm_adapter.decode(z)
        z_pooled = F.adaptive_avg_pool2d(z, (self.z_pooled_resolution, self.z_pooled_resolution)).flatten(1)
        if self.label_type in ['text', 'cls2text']:
            fine, glob, mask = self.vfm_encoder.encode_text(c)
            ws = self.mapping(z_pooled, glob, truncation_psi=truncation_psi)
            img, *_ = self.synthesis(z, ws, fine, mask, **synthesis_kwargs)
        else:
            ws = self.mapping(z_pooled, c, truncation_psi=truncation_psi)
            img, *_ = self.synthesis(z, ws, None, None, **synthesis_kwargs)
        return img

    def forward(self, img, c, truncation_psi=1.0, validation=False, **synthesis_kwargs):
        eq_scale, eq_angle, is_prior = self.equivariance_transform(validation=validation)
        feats, *_ = self.vfm_encoder.encode_image(img, eq_scale_factor=eq_scale if is_prior else 1.0,
                                                  is_eq_prior=is_prior)
        enc: EncodeOutput = self.ldm_adapter.encode(feats)
        z = enc.z
        if not validation and not is_prior:
            if eq_scale != 1.0:
                z = F.interpolate(z, scale_factor=eq_scale, mode='bilinear', align_corners=False)
            if eq_angle != 0:
                z = torch.rot90(z, k=eq_angle, dims=[-1, -2])
        z = self.ldm_adapter.decode(z)
        z_pooled = F.adaptive_avg_pool2d(z, (self.z_pooled_resolution, self.z_pooled_resolution)).flatten(1)
        if self.label_type in ['text', 'cls2text']:
            fine, glob, mask = self.vfm_encoder.encode_text(c)
            ws = self.mapping(z_pooled, glob, truncation_psi=truncation_psi)
            gen_img, gen_ms = self.synthesis(z, ws, fine, mask, **synthesis_kwargs)
        else:
            glob = None
            ws = self.mapping(z_pooled, c, truncation_psi=truncation_psi)
            gen_img, gen_ms = self.synthesis(z, ws, None, None, **synthesis_kwargs)
        return GeneratorForwardOutput(gen_img=gen_img, gen_multiscale_imgs=gen_ms, vf_loss=enc.vf_loss,
                                      vf_last_layer=enc.vf_last_layer, kl_loss=enc.kl_loss, vq_loss=enc.vq_loss,
                                      entropy_loss=enc.entropy_loss, codebook_usages=enc.codebook_usages,
                                      eq_scale_factor=eq_scale, eq_angle_factor=eq_angle, global_text_tokens=glob)
