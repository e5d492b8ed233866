"""Multi-scale feature fusion and latent bottleneck (LDMAdapter).

Same classes, constructor arguments and parameter/buffer names as the reference
`networks/utils/ldm_utils.py` (init_weights :25-50, PlainAttention :55-93,
GeGluMlp :96-114, AttnProjectionBlock :117-138, AttnProjection :140-166,
GeneralPixelUnshuffle :169-196, LDMAdapter :199-488, EquivarianceTransform
:491-517), so released checkpoints load unchanged.
"""
import random
from typing import List

import torch
import torch.nn as nn
import torch.nn.functional as F

from torch_utils import distributed as dist
from torch_utils.ops import vit_ops
from torch_utils.ops.linear import Linear, linear, bmm
from networks.utils import kl_utils
from networks.utils.kl_utils import DiagonalGaussianDistribution
from networks.utils.shared import Conv1x1
from networks.utils.quant_utils import VectorQuantizerM
from networks.utils.dataclasses import EncodeOutput


def init_weights(model, conv_std_or_gain):
    """Linear/Embedding: trunc-normal(0.02); conv: trunc-normal(std) if std > 0 else
    xavier-normal(gain=-std); norms: weight 1, bias 0."""
    dist.print0(f'[init_weights] {type(model).__name__} with {"std" if conv_std_or_gain > 0 else "gain"}={abs(conv_std_or_gain):g}')
    convs = (nn.Conv1d, nn.Conv2d, nn.Conv3d, nn.ConvTranspose1d, nn.ConvTranspose2d, nn.ConvTranspose3d)
    norms = (nn.LayerNorm, nn.BatchNorm1d, nn.BatchNorm2d, nn.BatchNorm3d, nn.SyncBatchNorm, nn.GroupNorm,
             nn.InstanceNorm1d, nn.InstanceNorm2d, nn.InstanceNorm3d)
    for m in model.modules():
        if isinstance(m, nn.Linear):
            nn.init.trunc_normal_(m.weight.data, std=0.02)
            if m.bias is not None:
                nn.init.constant_(m.bias.data, 0.)
        elif isinstance(m, nn.Embedding):
            nn.init.trunc_normal_(m.weight.data, std=0.02)
            if m.padding_idx is not None:
                m.weight.data[m.padding_idx].zero_()
        elif isinstance(m, convs):
            if conv_std_or_gain > 0:
                nn.init.trunc_normal_(m.weight.data, std=conv_std_or_gain)
            else:
                nn.init.xavier_normal_(m.weight.data, gain=-conv_std_or_gain)
            if getattr(m, 'bias', None) is not None:
                nn.init.constant_(m.bias.data, 0.)
        elif isinstance(m, norms):
            if m.bias is not None:
                nn.init.constant_(m.bias.data, 0.)
            if m.weight is not None:
                nn.init.constant_(m.weight.data, 1.)


class PlainAttention(nn.Module):
    """Self-attention used as a projection: in_dim > out_dim averages the heads
    (out = mean_h attn_h), otherwise heads are concatenated."""

    def __init__(self, in_dim, out_dim, num_heads):
        super().__init__()
        width = in_dim if in_dim > out_dim else out_dim
        self.head_dim = width // num_heads
        self.qkv = Linear(in_dim, width * 3, bias=False)
        self.q_bias = nn.Parameter(torch.zeros(width))
        self.v_bias = nn.Parameter(torch.zeros(width))
        self.register_buffer('zero_k_bias', torch.zeros(width))
        self.in_dim = in_dim
        self.out_dim = out_dim
        self.num_heads = num_heads
        self.scale = self.head_dim ** -0.5
        self.proj = Linear(out_dim, out_dim)

    def forward(self, x):
        B, N, C = x.shape
        bias = torch.cat((self.q_bias, self.zero_k_bias, self.v_bias))
        qkv = linear(x, self.qkv.weight, bias)
        x = vit_ops.sdpa_packed(qkv, self.num_heads)                         # [B, h, N, d]
        if self.in_dim > self.out_dim:
            x = x.mean(dim=1)
            if self.in_dim // self.num_heads != self.out_dim:
                x = F.adaptive_avg_pool1d(x, self.out_dim)
        else:
            x = x.transpose(1, 2).reshape(B, N, -1)
        return self.proj(x)


class GeGluMlp(nn.Module):
    def __init__(self, in_features, hidden_features):
        super().__init__()
        self.norm = nn.LayerNorm(in_features, eps=1e-6)
        self.act = nn.GELU(approximate='tanh')
        self.w0 = Linear(in_features, hidden_features)
        self.w1 = Linear(in_features, hidden_features)
        self.w2 = Linear(hidden_features, in_features)

    def forward(self, x):
        x = self.norm(x)
        return self.w2(self.act(self.w0(x)) * self.w1(x))


class AttnProjectionBlock(nn.Module):
    def __init__(self, in_dim, out_dim, num_heads, norm_layer=nn.LayerNorm, mlp_ratio=2):
        super().__init__()
        assert out_dim % in_dim == 0 or in_dim % out_dim == 0
        self.in_dim = in_dim
        self.out_dim = out_dim
        self.norm1 = norm_layer(in_dim)
        self.attn = PlainAttention(in_dim, out_dim, num_heads)
        self.proj = Linear(in_dim, out_dim)
        self.norm3 = norm_layer(in_dim)
        self.norm2 = norm_layer(out_dim)
        self.mlp = GeGluMlp(in_features=out_dim, hidden_features=int(out_dim * mlp_ratio))

    def forward(self, x):
        x = self.proj(self.norm3(x)) + self.attn(self.norm1(x))
        return x + self.mlp(self.norm2(x))


class AttnProjection(nn.Module):
    def __init__(self, in_dim, out_dim, num_heads, num_layers, is_quant, norm_layer=nn.LayerNorm, mlp_ratio=2):
        super().__init__()
        assert out_dim % in_dim == 0 or in_dim % out_dim == 0
        self.in_dim = in_dim
        self.out_dim = out_dim
        self.num_layers = num_layers
        blocks = []
        for i in range(num_layers):
            if is_quant:   # keep the width until the last block, which projects
                dims = (in_dim, in_dim) if i < num_layers - 1 else (in_dim, out_dim)
            else:          # project in the first block, keep the width afterwards
                dims = (in_dim, out_dim) if i == 0 else (out_dim, out_dim)
            blocks.append(AttnProjectionBlock(dims[0], dims[1], num_heads, norm_layer, mlp_ratio))
        self.blocks = nn.ModuleList(blocks)

    def forward(self, x):
        for blk in self.blocks:
            x = blk(x)
        return x


class GeneralPixelUnshuffle(nn.Module):
    """PixelUnshuffle for [B, C, H, W] or square token maps [B, H*W, C]; optional
    flattening back to tokens."""

    def __init__(self, downscale_factor, flatten_output=False):
        super().__init__()
        self.downscale_factor = downscale_factor
        self.flatten_output = flatten_output
        self.pixel_unshuffle = nn.PixelUnshuffle(downscale_factor)

    def forward(self, x):
        if x.dim() == 3:
            B, HW, D = x.shape
            side = int(HW ** 0.5)
            assert side * side == HW
            x = x.permute(0, 2, 1).reshape(B, D, side, side)
        elif x.dim() != 4:
            raise ValueError(f"Unsupported input shape: {x.shape}")
        x = self.pixel_unshuffle(x)
        if self.flatten_output:
            B, C, H, W = x.shape
            return x.permute(0, 2, 3, 1).reshape(B, H * W, C)
        return x


def _tokens_to_map(x):
    B, L, D = x.shape
    s = int(L ** 0.5)
    return x.transpose(1, 2).reshape(B, D, s, s)


def _map_to_tokens(x):
    B, D, H, W = x.shape
    return x.reshape(B, D, H * W).transpose(1, 2)


class LDMAdapter(nn.Module):
    def __init__(self, patch_from_layers: List[int], patch_resolutions: List[int], patch_in_dimensions: List[int],
                 patch_out_dimensions: List[int], compression_mode: str, how_to_compress: str, how_to_decompress: str,
                 decompress_factor: int, attnproj_quant_layers: int, attnproj_post_quant_layers: int,
                 z_resolution: int, z_dimension: int, vocab_width: int = 64, vocab_size: int = 32768,
                 vocab_beta: float = 0.25, use_entropy_loss: bool = False, entropy_temp: float = 0.01,
                 num_codebooks: int = 8, use_kl_loss: bool = False, use_vf_loss: bool = False,
                 use_adaptive_vf_loss: bool = False, distmat_margin: float = 0.0, cos_margin: float = 0.0,
                 distmat_weight: float = 1.0, cos_weight: float = 1.0):
        super().__init__()
        n = len(patch_from_layers)
        assert n == len(patch_resolutions) == len(patch_in_dimensions) == len(patch_out_dimensions)
        assert all(r >= z_resolution and r % z_resolution == 0 for r in patch_resolutions)
        assert all(i >= o for i, o in zip(patch_in_dimensions, patch_out_dimensions))
        assert (-1 in patch_from_layers) if use_vf_loss else True
        self.patch_from_layers = patch_from_layers
        self.patch_resolutions = patch_resolutions
        self.patch_in_dimensions = patch_in_dimensions
        self.patch_out_dimensions = patch_out_dimensions
        self.compression_mode = compression_mode
        self.z_resolution = z_resolution
        self.z_dimension = z_dimension
        self.how_to_compress = how_to_compress
        self.how_to_decompress = how_to_decompress
        self.decompress_factor = decompress_factor
        self.use_kl_loss = use_kl_loss
        self.use_vf_loss = use_vf_loss
        self.use_adaptive_vf_loss = use_adaptive_vf_loss

        quants = []
        for i in range(n):
            ratio = patch_resolutions[i] // z_resolution
            if how_to_compress == 'conv':
                head = nn.Conv2d(patch_in_dimensions[i], patch_out_dimensions[i], kernel_size=1, bias=True)
                tail = GeneralPixelUnshuffle(ratio, flatten_output=False) if ratio > 1 else nn.Identity()
            elif how_to_compress == 'attnproj':
                head = AttnProjection(in_dim=patch_in_dimensions[i], out_dim=patch_out_dimensions[i],
                                      num_heads=max(1, patch_in_dimensions[i] // patch_out_dimensions[i]),
                                      num_layers=attnproj_quant_layers, is_quant=True)
                tail = GeneralPixelUnshuffle(ratio, flatten_output=True) if ratio > 1 else nn.Identity()
            else:
                raise ValueError(how_to_compress)
            quants.append(nn.Sequential(head, tail))
        self.patch_quants = nn.ModuleList(quants)
        for m in self.patch_quants:
            init_weights(m[0], conv_std_or_gain=-0.5)

        final_in = sum(o * (r // z_resolution) ** 2 if r > z_resolution else o
                       for o, r in zip(patch_out_dimensions, patch_resolutions))
        final_out = z_dimension * 2 if compression_mode == 'continuous' else vocab_width
        if how_to_compress == 'conv':
            self.final_quant = nn.Conv2d(final_in, final_out, kernel_size=1, bias=True)
        else:
            self.final_quant = AttnProjection(in_dim=final_in, out_dim=final_out,
                                              num_heads=max(1, final_in // final_out),
                                              num_layers=attnproj_quant_layers, is_quant=True)
        init_weights(self.final_quant, conv_std_or_gain=-0.5)

        in_ch = z_dimension if compression_mode == 'continuous' else vocab_width
        out_ch = in_ch * decompress_factor
        if how_to_decompress == 'conv':
            self.post_quant = nn.Conv2d(in_ch, out_ch, kernel_size=1, bias=True)
        else:
            self.post_quant = AttnProjection(in_dim=in_ch, out_dim=out_ch, num_heads=max(1, out_ch // in_ch),
                                             num_layers=attnproj_post_quant_layers, is_quant=False)
        init_weights(self.post_quant, conv_std_or_gain=-0.5)

        if compression_mode == 'discrete':
            self.quantizer = VectorQuantizerM(vocab_size=vocab_size, vocab_width=vocab_width, beta=vocab_beta,
                                              use_entropy_loss=use_entropy_loss, entropy_temp=entropy_temp,
                                              num_codebooks=num_codebooks)
            self.quantizer.init_vocab(eini=-1)
        else:
            self.quantizer = None

        if use_vf_loss:
            vf_dim = patch_in_dimensions[patch_from_layers.index(-1)]
            self.linear_proj = Conv1x1(in_ch, vf_dim, 1, bias=False)   # nn.Conv2d keys; 1x1 on our GEMMs
            init_weights(self.linear_proj, conv_std_or_gain=-0.5)
            self.distmat_margin = distmat_margin
            self.cos_margin = cos_margin
            self.distmat_weight = distmat_weight
            self.cos_weight = cos_weight
        else:
            self.linear_proj = None

    def _compute_vf_loss(self, z, aux):
        """Alignment loss: mean relu(|cos-Gram(z) - cos-Gram(aux)| - m1) + mean relu(1 - m2 - cos(z, aux))."""
        B, C = z.shape[:2]
        zn = F.normalize(z.reshape(B, C, -1), dim=1)
        an = F.normalize(aux.reshape(B, aux.shape[1], -1), dim=1)
        z_cos = bmm(zn.transpose(1, 2), zn)
        a_cos = bmm(an.transpose(1, 2), an)
        l1 = F.relu((z_cos - a_cos).abs() - self.distmat_margin).mean()
        l2 = F.relu(1 - self.cos_margin - F.cosine_similarity(aux, z)).mean()
        return l1 * self.distmat_weight + l2 * self.cos_weight

    def encode(self, patch_features: List[torch.Tensor], return_z_before_quantize: bool = False) -> EncodeOutput:
        assert len(patch_features) == len(self.patch_quants)
        mids = []
        for x, proj in zip(patch_features, self.patch_quants):
            if self.how_to_compress == 'conv':
                x = _map_to_tokens(proj(_tokens_to_map(x)))
            else:
                x = proj(x)
            mids.append(x)
        x = torch.cat(mids, dim=-1)
        if self.how_to_compress == 'conv':
            x = self.final_quant(_tokens_to_map(x))
        else:
            x = _tokens_to_map(self.final_quant(x))

        vq_loss = entropy_loss = usages = kl_loss = 0.0
        z_before_quantize = x
        if self.compression_mode == 'continuous':
            z, kl = kl_utils.sample_and_kl(x, need_kl=self.use_kl_loss)     # posterior sample (+ KL)
            if self.use_kl_loss:
                kl_loss = kl.mean()
        else:
            z_tokens, vq_loss, entropy_loss, usages = self.quantizer(_map_to_tokens(x))
            z = _tokens_to_map(z_tokens)

        vf_loss = 0.0
        vf_last_layer = None
        if self.use_vf_loss:
            aux = _tokens_to_map(patch_features[self.patch_from_layers.index(-1)].detach().clone())
            if aux.shape[-1] != z.shape[2]:
                aux = F.adaptive_avg_pool2d(aux, (z.shape[2], z.shape[2]))
            vf_loss = self._compute_vf_loss(self.linear_proj(z), aux)
            if self.use_adaptive_vf_loss:
                vf_last_layer = self.final_quant.weight if self.how_to_compress == 'conv' else \
                    self.final_quant.blocks[-1].mlp.w2.weight

        return EncodeOutput(z=z if not return_z_before_quantize else z_before_quantize, vf_loss=vf_loss,
                            vf_last_layer=vf_last_layer, kl_loss=kl_loss, vq_loss=vq_loss,
                            entropy_loss=entropy_loss, codebook_usages=usages)

    def decode(self, z):
        if self.how_to_decompress == 'conv':
            return self.post_quant(z)
        H, W = z.shape[-2:]
        t = self.post_quant(_map_to_tokens(z))
        return t.transpose(1, 2).reshape(t.shape[0], -1, H, W)


class EquivarianceTransform(nn.Module):
    """Draws (scale, quarter-turns, is_prior) for equivariance regularisation from
    python's `random` (same draws and order as reference ldm_utils.py:503-517)."""

    SCALES = (0.25, 0.5, 0.75, 1.0)

    def __init__(self, apply=False, p_eq_prior=0.5, p_eq_prior_scale=0.25):
        super().__init__()
        self.apply = apply
        self.p_eq_prior = p_eq_prior
        self.p_eq_prior_scale = p_eq_prior_scale
        self.forced = None          # (scale, quarter_turns, is_prior): shape warm-up only, consumes no draws

    def variants(self):
        """Every (scale, quarter_turns, is_prior) shape class forward() can produce."""
        if not self.apply:
            return [(1.0, 0, False)]
        return [(s, 0, p) for p in (False, True) for s in self.SCALES]

    def outcomes(self):
        """Every distinct value forward(validation=False) can return."""
        if not self.apply:
            return [(1.0, 0, False)]
        return [(s, a, False) for s in self.SCALES for a in range(4)] + [(s, 0, True) for s in self.SCALES]

    def forward(self, validation: bool):
        if not self.apply or validation:
            return 1.0, 0, False
        if self.forced is not None:
            return self.forced
        if random.random() < self.p_eq_prior:
            return random.choice([0.25, 0.5, 0.75, 1.0]), random.choice([0, 1, 2, 3]), False
        scale = random.choice([0.25, 0.5, 0.75]) if random.random() < self.p_eq_prior_scale else 1.0
        return scale, 0, True
