"""Projected discriminator: frozen DINO ViT-S/16 + spectral-norm Conv1d heads
(StyleGAN-T) and/or a multi-scale PatchGAN.

Module API, constructor arguments and state-dict keys follow the reference
`networks/discriminator.py` (SpectralConv1d :39-42, BatchNormLocal :45-71,
BatchNormLocal2d :75-99, DiscHead :116-142, DINO :145-168, NLayerDiscriminator
:180-228, MultiscaleDiscriminator :231-268, ProjectedDiscriminator :271-366).

The DINO weights are a `timm.create_model(..., pretrained=True)` download in the
reference; offline they are loaded from `VFM_DINO_CHECKPOINT` (a timm-layout
state dict, safetensors or .pth read with weights_only=True) when that is set,
otherwise the ViT-S/16 architecture is random-initialised from a fixed seed.
"""
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from torch_utils.ops import decoder_ops
from torch.nn.utils.spectral_norm import SpectralNorm

from torch_utils import distributed as dist
from networks.utils.dataclasses import DiscriminatorForwardOutput
from networks.utils.shared import ResidualBlock, FullyConnectedLayer
from networks.utils.vit_utils import VisionTransformer, make_vit_backbone, forward_vit
from networks.utils.vfm_utils import VFM2INTERPOLATION
from training.diffaug import DiffAugment

# VFM_DHEAD_FOLDED=0: the per-sample batched GEMMs (stride-0 weight) instead of the batch-folded GEMMs
_FOLDED = os.environ.get("VFM_DHEAD_FOLDED", "1") == "1"

IMAGENET_DEFAULT_MEAN = (0.485, 0.456, 0.406)
IMAGENET_DEFAULT_STD = (0.229, 0.224, 0.225)


class SpectralConv1d(nn.Conv1d):
    """Spectral-normalised Conv1d (reference discriminator.py:39-42).

    On ROCm fp32 tensors the convolution of the whole batch is one exact-fp32 GEMM each way, the
    batch folded into the im2col columns ([C k, B L], patchgan_hip.conv1d_folded), instead of
    MIOpen's per-sample im2col + small-GEMM loop; same math."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        SpectralNorm.apply(self, name='weight', n_power_iterations=1, dim=0, eps=1e-12)
        # training-mode power iteration + W / sigma on csrc/specnorm.hip for ROCm weights (same buffers,
        # same state-dict keys; torch's hook runs otherwise)
        from torch_utils.ops import specnorm
        specnorm.install_fused_spectral_norm(self)

    def _conv_forward(self, x, weight, bias):
        if not x.is_cuda or self.groups != 1 or self.stride != (1,) or self.dilation != (1,) or x.dim() != 3:
            return super()._conv_forward(x, weight, bias)
        k = self.kernel_size[0]
        p = self.padding[0]
        circ = self.padding_mode == 'circular'
        from torch_utils.ops import patchgan_hip
        if (_FOLDED and self.padding_mode in ('zeros', 'circular')
                and patchgan_hip.conv1d_folded_supported(x, k, p, circ)):
            # the whole batch as one GEMM each way, batch folded into the columns (csrc/im2col1d.hip CBL)
            return patchgan_hip.conv1d_folded(x, weight.reshape(weight.shape[0], -1), bias, k, p, circ)
        if k > 1 or p > 0:
            if self.padding_mode in ('zeros', 'circular') and patchgan_hip.im2col1d_supported(x, k, p, circ):
                x = patchgan_hip.im2col1d(x, k, p, circ)             # one launch each way (csrc/im2col1d.hip)
                return self._gemm_out(x, weight, bias)
            mode = 'constant' if self.padding_mode == 'zeros' else self.padding_mode
            xp = F.pad(x, (p, p), mode=mode) if p > 0 else x
            B, C, _ = xp.shape
            cols = xp.unfold(2, k, 1)                                  # [B, C, L, k]
            L = cols.shape[2]
            x = cols.permute(0, 1, 3, 2).reshape(B, C * k, L)
        return self._gemm_out(x, weight, bias)

    @staticmethod
    def _gemm_out(x, weight, bias):
        # exact fp32 GEMM (hipBLASLt): the heads' BatchNormLocal over virtual batches of <= 8
        # samples amplifies GEMM rounding into the input gradient, so these stay on the vendor's
        # fp32 products. As a batched product with the weight broadcast (stride-0 batch): torch.matmul's
        # 2-D x 3-D form folds the batch through x's transpose, which copies the [B, C k, L] columns
        # forward and the gradient backward (~2.7 ms/step of copies, profiles/r4_h_opsites_timed.txt)
        w2 = weight.reshape(weight.shape[0], -1)
        y = torch.bmm(w2.expand(x.shape[0], *w2.shape), x) if x.dim() == 3 else torch.matmul(w2, x)
        if bias is not None:
            y = y + bias.to(y.dtype)[None, :, None]
        return y


class BatchNormLocal(nn.Module):
    """BatchNorm over virtual batches of `virtual_bs` samples ([B, C, L] inputs)."""

    def __init__(self, num_features, affine=True, virtual_bs=8, eps=1e-5):
        super().__init__()
        self.virtual_bs = virtual_bs
        self.eps = eps
        self.affine = affine
        if affine:
            self.weight = nn.Parameter(torch.ones(num_features))
            self.bias = nn.Parameter(torch.zeros(num_features))

    def forward(self, x):
        shape = x.shape
        G = int(np.ceil(x.size(0) / self.virtual_bs))
        x = x.view(G, -1, x.size(-2), x.size(-1))
        var, mean = torch.var_mean(x, dim=[1, 3], keepdim=True, unbiased=False)
        x = (x - mean) * torch.rsqrt(var + self.eps)
        if self.affine:
            x = x * self.weight[None, :, None] + self.bias[None, :, None]
        return x.view(shape)


class BatchNormLocal2d(nn.Module):
    """BatchNorm over virtual batches of `virtual_bs` samples ([B, C, H, W] inputs)."""

    def __init__(self, num_features, affine=True, virtual_bs=8, eps=1e-5):
        super().__init__()
        self.virtual_bs = virtual_bs
        self.eps = eps
        self.affine = affine
        if affine:
            self.weight = nn.Parameter(torch.ones(num_features))
            self.bias = nn.Parameter(torch.zeros(num_features))

    def forward(self, x):
        shape = x.shape
        B, C, H, W = shape
        G = int(np.ceil(B / self.virtual_bs))
        x = x.view(G, -1, C, H, W)
        var, mean = torch.var_mean(x, dim=[1, 3, 4], keepdim=True, unbiased=False)
        x = (x - mean) * torch.rsqrt(var + self.eps)
        if self.affine:
            x = x * self.weight[None, None, :, None, None] + self.bias[None, None, :, None, None]
        return x.view(shape)


class HeadBlock(nn.Sequential):
    """SpectralConv1d -> BatchNormLocal -> LeakyReLU(0.2) (same modules / state-dict keys as the
    reference's nn.Sequential). On ROCm fp32 inputs the BatchNormLocal + LeakyReLU pair runs as one
    fused HIP kernel per direction (patchgan_hip.bn_local1d_lrelu); the conv is the batch-folded
    im2col + exact-fp32 product of patchgan_hip._Conv1dFolded."""

    def forward(self, x):
        conv, bn, act = self[0], self[1], self[2]
        if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 3):
            return super().forward(x)
        h = conv(x)
        G = int(np.ceil(h.shape[0] / bn.virtual_bs))
        if h.shape[0] % G:
            return act(bn(h))
        from torch_utils.ops import patchgan_hip
        return patchgan_hip.bn_local1d_lrelu(h, bn.weight if bn.affine else None, bn.bias if bn.affine else None, G,
                                            bn.eps, act.negative_slope)


def make_block(channels, kernel_size):
    return HeadBlock(
        SpectralConv1d(channels, channels, kernel_size=kernel_size, padding=kernel_size // 2, padding_mode='circular'),
        BatchNormLocal(channels),
        nn.LeakyReLU(0.2, True),
    )


class DiscHead(nn.Module):
    def __init__(self, channels, c_dim, cmap_dim=64):
        super().__init__()
        self.channels, self.c_dim, self.cmap_dim = channels, c_dim, cmap_dim
        self.main = nn.Sequential(make_block(channels, kernel_size=1), ResidualBlock(make_block(channels, kernel_size=9)))
        if c_dim > 0:
            self.cmapper = FullyConnectedLayer(c_dim, cmap_dim)
            self.cls = SpectralConv1d(channels, cmap_dim, kernel_size=1, padding=0)
        else:
            self.cls = SpectralConv1d(channels, 1, kernel_size=1, padding=0)

    def forward(self, x, c):
        out = self.cls(self.main(x))
        if self.c_dim > 0:
            cmap = self.cmapper(c).unsqueeze(-1)
            out = (out * cmap).sum(1, keepdim=True) * (1 / np.sqrt(self.cmap_dim))
        return out


class DINO(nn.Module):
    def __init__(self, hooks=[2, 5, 8, 11], hook_patch=True):
        super().__init__()
        self.n_hooks = len(hooks) + int(hook_patch)
        self.patch_size = 16
        vit = VisionTransformer(img_size=224, patch_size=16, embed_dim=384, depth=12, num_heads=6)
        vit.reset_parameters()
        ckpt = os.environ.get("VFM_DINO_CHECKPOINT")
        if ckpt:
            if ckpt.endswith(".safetensors"):
                from safetensors.torch import load_file
                state = load_file(ckpt)
            else:
                state = torch.load(ckpt, map_location="cpu", weights_only=True)
            vit.load_state_dict({k: v for k, v in state.items() if not k.startswith("head")}, strict=False)
            dist.print0(f"[DINO] loaded {ckpt}")
        self.model = make_vit_backbone(vit, patch_size=[16, 16], hooks=hooks, hook_patch=hook_patch)
        self.model.eval().requires_grad_(False)
        self.img_resolution = vit.patch_embed.img_size[0]
        self.embed_dim = vit.embed_dim

    def forward(self, x):
        return forward_vit(self.model, x)


def weights_init(m):
    name = m.__class__.__name__
    if name.find('Conv') != -1:
        m.weight.data.normal_(0.0, 0.02)
    elif name.find('BatchNorm2d') != -1:
        m.weight.data.normal_(1.0, 0.02)
        m.bias.data.fill_(0)


class PatchBlock(nn.Sequential):
    """nn.Sequential of the PatchGAN's Conv2d / BatchNormLocal2d / LeakyReLU (same state-dict keys).
    ROCm fp32 inputs run the HIP path (torch_utils/ops/patchgan_hip.py): NHWC activations, k4 convs
    as im2col + MFMA GEMM, BatchNormLocal2d + LeakyReLU fused; outputs are NCHW views of the NHWC
    results (channels_last memory)."""

    def forward(self, x):
        from torch_utils.ops import patchgan_hip
        mods = list(self)
        if not patchgan_hip.supported(x) or not self._hip_ok(mods, x.shape[0]):
            return super().forward(x)
        h = x.permute(0, 2, 3, 1)
        i = 0
        while i < len(mods):
            m = mods[i]
            nxt = mods[i + 1] if i + 1 < len(mods) else None
            if isinstance(m, nn.Conv2d):
                fuse = isinstance(nxt, nn.LeakyReLU) and m.bias is not None
                h = patchgan_hip.conv_nhwc(h, m.weight, None if fuse else m.bias, m.stride[0], m.padding[0])
                if fuse:
                    h = patchgan_hip.bias_lrelu(h, m.bias, nxt.negative_slope)
                    i += 1
            elif isinstance(m, BatchNormLocal2d):
                G = int(np.ceil(h.shape[0] / m.virtual_bs))
                if isinstance(nxt, nn.LeakyReLU):
                    slope, i = nxt.negative_slope, i + 1
                else:
                    slope = 1.0
                h = patchgan_hip.bn_local_lrelu(h, m.weight if m.affine else None, m.bias if m.affine else None, G,
                                                m.eps, slope)
            elif isinstance(m, nn.LeakyReLU):
                h = patchgan_hip.bias_lrelu(h, None, m.negative_slope)
            else:
                h = m(h.permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
            i += 1
        return h.permute(0, 3, 1, 2)

    @staticmethod
    def _hip_ok(mods, B):
        for m in mods:
            if isinstance(m, nn.Conv2d):
                if m.groups != 1 or m.dilation != (1, 1) or m.padding_mode != 'zeros' or m.stride[0] != m.stride[1] \
                        or m.padding[0] != m.padding[1] or m.kernel_size[0] != m.kernel_size[1]:
                    return False
            elif isinstance(m, BatchNormLocal2d):
                G = int(np.ceil(B / m.virtual_bs))
                C = m.weight.shape[0] if m.affine else 0
                if B % G or (m.affine and (C % 4 or 256 % (C // 4))):
                    return False
        return True


class NLayerDiscriminator(nn.Module):
    def __init__(self, input_nc, ndf=64, n_layers=3, norm_layer=BatchNormLocal2d, use_sigmoid=False,
                 get_interm_feat=False):
        super().__init__()
        self.get_interm_feat = get_interm_feat
        self.n_layers = n_layers
        kw, padw = 4, int(np.ceil((4 - 1.0) / 2))
        seq = [[nn.Conv2d(input_nc, ndf, kernel_size=kw, stride=2, padding=padw), nn.LeakyReLU(0.2, True)]]
        nf = ndf
        for _ in range(1, n_layers):
            nf_prev, nf = nf, min(nf * 2, 512)
            seq += [[nn.Conv2d(nf_prev, nf, kernel_size=kw, stride=2, padding=padw), norm_layer(nf), nn.LeakyReLU(0.2, True)]]
        nf_prev, nf = nf, min(nf * 2, 512)
        seq += [[nn.Conv2d(nf_prev, nf, kernel_size=kw, stride=1, padding=padw), norm_layer(nf), nn.LeakyReLU(0.2, True)]]
        seq += [[nn.Conv2d(nf, 1, kernel_size=kw, stride=1, padding=padw)]]
        if use_sigmoid:
            seq += [[nn.Sigmoid()]]
        if get_interm_feat:
            for n, layers in enumerate(seq):
                setattr(self, f'model{n}', PatchBlock(*layers))
        else:
            self.model = PatchBlock(*[m for layers in seq for m in layers])

    def forward(self, x):
        if self.get_interm_feat:
            res = [x]
            for n in range(self.n_layers + 2):
                res.append(getattr(self, f'model{n}')(res[-1]))
            return res[1:]
        return self.model(x)


class MultiscaleDiscriminator(nn.Module):
    def __init__(self, input_nc, ndf=64, n_layers=3, norm_layer=BatchNormLocal2d, use_sigmoid=False, num_D=3,
                 get_interm_feat=True):
        super().__init__()
        self.num_D, self.n_layers, self.get_interm_feat = num_D, n_layers, get_interm_feat
        for i in range(num_D):
            net = NLayerDiscriminator(input_nc, ndf, n_layers, norm_layer, use_sigmoid, get_interm_feat)
            if get_interm_feat:
                for j in range(n_layers + 2):
                    setattr(self, f'scale{i}_layer{j}', getattr(net, f'model{j}'))
            else:
                setattr(self, f'layer{i}', net.model)
        self.downsample = nn.AvgPool2d(3, stride=2, padding=[1, 1], count_include_pad=False)

    def singleD_forward(self, model, x):
        if self.get_interm_feat:
            res = [x]
            for m in model:
                res.append(m(res[-1]))
            return res[1:]
        return [model(x)]

    def forward(self, x):
        out = []
        for i in range(self.num_D):
            k = self.num_D - 1 - i
            model = [getattr(self, f'scale{k}_layer{j}') for j in range(self.n_layers + 2)] if self.get_interm_feat \
                else getattr(self, f'layer{k}')
            out.append(self.singleD_forward(model, x))
            if i != self.num_D - 1:
                x = self.downsample(x)
        return out


def _random_crop(x, size):
    """torchvision RandomCrop semantics: one offset for the whole batch, torch RNG."""
    h, w = x.shape[-2:]
    i = int(torch.randint(0, h - size + 1, size=(1,)).item())
    j = int(torch.randint(0, w - size + 1, size=(1,)).item())
    return x[..., i:i + size, j:j + size]


class ProjectedDiscriminator(nn.Module):
    def __init__(self, c_dim, vfm_name, use_stylegan_t_discriminator=True, diffaug=True, p_crop=0.5,
                 use_patchgan_discriminator=False, get_interm_feat=False):
        super().__init__()
        self.use_stylegan_t_discriminator = use_stylegan_t_discriminator
        self.use_patchgan_discriminator = use_patchgan_discriminator
        if use_stylegan_t_discriminator:
            self.diffaug = diffaug
            self.p_crop = p_crop
            self.vfm_name = (vfm_name or '').lower()
            self.interpolation = 'bilinear'
            for name in VFM2INTERPOLATION:
                if name in self.vfm_name:
                    self.interpolation = VFM2INTERPOLATION[name]
                    break
            self.register_buffer('_norm_mean', torch.tensor(IMAGENET_DEFAULT_MEAN).view(1, 3, 1, 1), persistent=False)
            self.register_buffer('_norm_std', torch.tensor(IMAGENET_DEFAULT_STD).view(1, 3, 1, 1), persistent=False)
            self.dino = DINO()
            self.c_dim = c_dim
            self.heads = nn.ModuleDict([(str(i), DiscHead(self.dino.embed_dim, c_dim)) for i in range(self.dino.n_hooks)])
        if use_patchgan_discriminator:
            self.get_interm_feat = get_interm_feat
            self.patchgan_discriminator = MultiscaleDiscriminator(input_nc=3, num_D=3, get_interm_feat=get_interm_feat)
            self.patchgan_discriminator.apply(weights_init)

    def train(self, mode=True):
        if self.use_stylegan_t_discriminator:
            self.dino = self.dino.train(False)
            self.heads = self.heads.train(mode)
        if self.use_patchgan_discriminator:
            self.patchgan_discriminator = self.patchgan_discriminator.train(mode)
        return self

    def eval(self):
        return self.train(False)

    def stylegan_t_forward(self, x, c_enc):
        if self.diffaug:
            x = DiffAugment(x, policy='color,translation,cutout')
        x = (x + 1.0) / 2.0
        res = self.dino.img_resolution
        if x.size(-1) > res and np.random.random() < self.p_crop:
            x = _random_crop(x, res)
        if x.size(-1) < res:
            x = F.interpolate(x, res, mode=self.interpolation, align_corners=False)
        elif x.size(-1) > res:
            x = F.interpolate(x, res, mode=self.interpolation, align_corners=False, antialias=True)
        x = (x - self._norm_mean) / self._norm_std
        feats = self.dino(x)
        from torch_utils.ops import specnorm_group
        with specnorm_group.SpecNormGroup(self.heads):   # every head weight's spectral norm in one launch per phase
            logits = [head(feats[k], c_enc).view(x.size(0), -1) for k, head in self.heads.items()]
        return torch.cat(logits, dim=1)

    def patchgan_forward(self, x):
        return self.patchgan_discriminator(x)

    def forward(self, x, c_enc):
        return DiscriminatorForwardOutput(
            stylegan_t_logits=self.stylegan_t_forward(x, c_enc) if self.use_stylegan_t_discriminator else None,
            patchgan_logits=self.patchgan_forward(x) if self.use_patchgan_discriminator else None)
