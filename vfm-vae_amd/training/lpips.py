"""LPIPS-VGG16 perceptual distance.

Same module tree and state-dict keys as the reference `training/lpips.py`
(LPIPS :61-104, ScalingLayer :107-114, NetLinLayer :117-123, vgg16 :126-163;
keys net.sliceK.<torchvision index>.*, linK.model.1.weight) so the published
`vgg.pth` / torchvision VGG16 weights load unchanged.

The reference downloads torchvision VGG16 and the LPIPS linear heads at
construction time (lpips.py:19-58, :129). Offline, weights are read from
`VFM_LPIPS_CHECKPOINT` (LPIPS vgg.pth, weights_only) and
`VFM_VGG16_CHECKPOINT` (torchvision vgg16 state dict) when set; otherwise
the architecture is random-initialised from a fixed seed.
"""
import os
from collections import namedtuple

import torch
import torch.nn as nn

from torch_utils import distributed as dist
from torch_utils.ops import lpips_ops

# torchvision vgg16 `features` (cfg D): channels per conv; 'M' = max-pool.
_VGG16_CFG = [64, 64, 'M', 128, 128, 'M', 256, 256, 256, 'M', 512, 512, 512, 'M', 512, 512, 512]
_SLICES = [(0, 4), (4, 9), (9, 16), (16, 23), (23, 30)]


def _vgg16_features():
    layers, cin = [], 3
    for v in _VGG16_CFG:
        if v == 'M':
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers += [nn.Conv2d(cin, v, kernel_size=3, padding=1), nn.ReLU(inplace=True)]
            cin = v
    return layers


def _load(path):
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path)
    return torch.load(path, map_location="cpu", weights_only=True)


class vgg16(nn.Module):
    def __init__(self, requires_grad=False, pretrained=True):
        super().__init__()
        feats = _vgg16_features()
        g = torch.Generator().manual_seed(2024)
        for m in feats:
            if isinstance(m, nn.Conv2d):
                with torch.no_grad():
                    fan_out = m.out_channels * 9
                    m.weight.copy_(torch.randn(m.weight.shape, generator=g) * (2.0 / fan_out) ** 0.5)
                    m.bias.zero_()
        ckpt = os.environ.get("VFM_VGG16_CHECKPOINT") if pretrained else None
        if ckpt:
            state = _load(ckpt)
            for i, m in enumerate(feats):
                if isinstance(m, nn.Conv2d):
                    m.weight.data.copy_(state[f"features.{i}.weight"])
                    m.bias.data.copy_(state[f"features.{i}.bias"])
        self.N_slices = 5
        for k, (a, b) in enumerate(_SLICES, start=1):
            s = nn.Sequential()
            for i in range(a, b):
                s.add_module(str(i), feats[i])
            setattr(self, f"slice{k}", s)
        if not requires_grad:
            for p in self.parameters():
                p.requires_grad = False

    # 'hip': fp32 ROCm inputs run the fused NHWC stack (torch_utils/ops/vgg_hip.py); 'torch': MIOpen (A/B)
    impl = os.environ.get('VFM_LPIPS_VGG', 'hip')

    def forward(self, X):
        if X.is_cuda and X.dtype == torch.float32 and self.impl == 'hip':
            from torch_utils.ops import vgg_hip
            convs = [m for k in range(1, 6) for m in getattr(self, f"slice{k}") if isinstance(m, nn.Conv2d)]
            outs = vgg_hip.vgg16_taps(X, convs)
        else:
            outs = []
            h = X
            for k in range(1, 6):
                h = getattr(self, f"slice{k}")(h)
                outs.append(h)
        return namedtuple("VggOutputs", ['relu1_2', 'relu2_2', 'relu3_3', 'relu4_3', 'relu5_3'])(*outs)


class ScalingLayer(nn.Module):
    def __init__(self):
        super().__init__()
        self.register_buffer('shift', torch.tensor([-.030, -.088, -.188])[None, :, None, None])
        self.register_buffer('scale', torch.tensor([.458, .448, .450])[None, :, None, None])

    def forward(self, inp):
        return (inp - self.shift) / self.scale


class NetLinLayer(nn.Module):
    """(Dropout) + 1x1 conv to one channel, no bias."""

    def __init__(self, chn_in, chn_out=1, use_dropout=False):
        super().__init__()
        layers = [nn.Dropout()] if use_dropout else []
        layers += [nn.Conv2d(chn_in, chn_out, 1, stride=1, padding=0, bias=False)]
        self.model = nn.Sequential(*layers)


def normalize_tensor(x, eps=1e-10):
    return x / (torch.sqrt(torch.sum(x ** 2, dim=1, keepdim=True)) + eps)


def spatial_average(x, keepdim=True):
    return x.mean([2, 3], keepdim=keepdim)


class LPIPS(nn.Module):
    # 'ref': the torch expression for the distance head (A/B, tests)
    head_impl = os.environ.get('VFM_LPIPS_HEAD', 'cuda')

    def __init__(self, use_dropout=True):
        super().__init__()
        self.scaling_layer = ScalingLayer()
        self.chns = [64, 128, 256, 512, 512]
        self.net = vgg16(pretrained=True, requires_grad=False)
        for i, c in enumerate(self.chns):
            setattr(self, f"lin{i}", NetLinLayer(c, use_dropout=use_dropout))
            with torch.no_grad():   # default head: uniform positive weights (the trained heads are >= 0)
                getattr(self, f"lin{i}").model[-1].weight.fill_(1.0 / c)
        self.load_from_pretrained()
        for p in self.parameters():
            p.requires_grad = False

    def load_from_pretrained(self, name="vgg_lpips"):
        ckpt = os.environ.get("VFM_LPIPS_CHECKPOINT")
        if ckpt:
            self.load_state_dict(_load(ckpt), strict=False)
            dist.print0(f"loaded pretrained LPIPS loss from {ckpt}")

    def forward(self, input, target):
        net = self.net
        if (input.is_cuda and input.dtype == torch.float32 and target.dtype == torch.float32
                and input.shape == target.shape and net.impl == 'hip'):
            # both batches through the VGG16 stack in one pass (per-sample layers: same taps as two passes)
            from torch_utils.ops import vgg_hip
            convs = [m for k in range(1, 6) for m in getattr(net, f"slice{k}") if isinstance(m, nn.Conv2d)]
            outs0, outs1 = vgg_hip.vgg16_taps_pair(self.scaling_layer(input), self.scaling_layer(target), convs)
        else:
            outs0 = self.net(self.scaling_layer(input))
            outs1 = self.net(self.scaling_layer(target))
        val = None
        for kk in range(len(self.chns)):
            lin = getattr(self, f"lin{kk}").model
            if outs0[kk].is_cuda and self.head_impl == 'cuda' and not (self.training and len(lin) > 1):
                # normalise -> diff -> square -> lin -> mean in one HIP pass (torch_utils/ops/lpips_ops.py)
                r = lpips_ops.lpips_head(outs0[kk], outs1[kk], lin[-1].weight)
            else:
                d = (normalize_tensor(outs0[kk]) - normalize_tensor(outs1[kk])) ** 2
                r = spatial_average(lin(d), keepdim=True)
            val = r if val is None else val + r
        return val
