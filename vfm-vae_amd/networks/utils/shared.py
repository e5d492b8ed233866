"""Shared building blocks: FC layer with learning-rate multiplier, MLP,
fp32-upcasting GroupNorm, StyleSplit, scale-adaptive pooling.

Same classes, constructor arguments and parameter names as the reference
`networks/utils/shared.py` (:17-189) so checkpoints load unchanged.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F


class ResidualBlock(nn.Module):
    """(fn(x) + x) / sqrt(2)."""

    def __init__(self, fn: nn.Module):
        super().__init__()
        self.fn = fn

    def forward(self, x):
        return (self.fn(x) + x) * (1.0 / math.sqrt(2))


class FullyConnectedLayer(nn.Module):
    """y = act(x @ (W * lr/sqrt(in))^T + b * lr). Weights are stored divided by
    the learning-rate multiplier (equalised learning rate)."""

    def __init__(self, in_features, out_features, bias=True, activation='linear', lr_multiplier=1.0,
                 weight_init=1.0, bias_init=0.0):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.activation = activation
        self.weight = nn.Parameter(torch.randn(out_features, in_features) * (weight_init / lr_multiplier))
        if bias:
            init = torch.as_tensor(bias_init, dtype=torch.float32)
            self.bias = nn.Parameter(torch.broadcast_to(init, [out_features]).clone() / lr_multiplier)
        else:
            self.bias = None
        self.weight_gain = lr_multiplier / math.sqrt(in_features)
        self.bias_gain = lr_multiplier

    def forward(self, x):
        w = self.weight.to(x.dtype) * self.weight_gain
        b = self.bias.to(x.dtype) * self.bias_gain if self.bias is not None else None
        if x.is_cuda and x.dtype == torch.float32:
            # the product (and its gradients) on our exact-fp32 GEMM (torch_utils/ops/linear.py -> csrc/sgemm.hip)
            from torch_utils.ops.linear import linear
            if self.activation == 'linear':
                return linear(x, w, b)
            y = linear(x, w, None)
        elif self.activation == 'linear':
            return torch.addmm(b.unsqueeze(0), x, w.t()) if b is not None else x.matmul(w.t())
        else:
            y = x.matmul(w.t())
        if self.activation in ('relu', 'lrelu') and y.is_cuda:
            # bias + activation in one HIP bias_act pass (gain 1: F.relu / F.leaky_relu(0.2) semantics)
            from torch_utils.ops import bias_act
            return bias_act.bias_act(y, b, act=self.activation, alpha=0.2 if self.activation == 'lrelu' else None,
                                     gain=1.0)
        if b is not None:
            y = y + b
        if self.activation == 'relu':
            return F.relu(y)
        if self.activation == 'lrelu':
            return F.leaky_relu(y, negative_slope=0.2)
        if self.activation == 'gelu':
            return F.gelu(y)
        raise NotImplementedError(f"Activation '{self.activation}' not implemented.")

    def extra_repr(self):
        return f'in_features={self.in_features}, out_features={self.out_features}, activation={self.activation}'


class MLP(nn.Module):
    """Stack of FullyConnectedLayers named fc0..fc{n-1}; accepts [B, C] or [B, K, C]."""

    def __init__(self, features_list, activation='linear', lr_multiplier=1.0, linear_out=False):
        super().__init__()
        self.num_layers = len(features_list) - 1
        self.out_dim = features_list[-1]
        for i in range(self.num_layers):
            act = 'linear' if (linear_out and i == self.num_layers - 1) else activation
            self.add_module(f'fc{i}', FullyConnectedLayer(features_list[i], features_list[i + 1], bias=True,
                                                          activation=act, lr_multiplier=lr_multiplier))

    def forward(self, x):
        lead = x.shape[:-1] if x.ndim == 3 else None
        if lead is not None:
            x = x.flatten(0, 1)
        for i in range(self.num_layers):
            x = getattr(self, f'fc{i}')(x)
        if lead is not None:
            x = x.reshape(*lead, -1)
        return x


class GroupNorm32(nn.GroupNorm):
    """GroupNorm evaluated in fp32, result cast back to the input dtype."""

    def forward(self, x):
        from torch_utils.ops import decoder_ops
        return decoder_ops.group_norm(x, self.num_groups, self.weight, self.bias, self.eps, out_dtype=x.dtype)


def _conv_dtype(x):
    """The dtype nn.Conv2d would compute in: autocast's dtype inside a CUDA autocast region."""
    if x.is_cuda and torch.is_autocast_enabled('cuda'):
        return torch.get_autocast_dtype('cuda')
    return x.dtype


class DepthwiseConv2d(nn.Conv2d):
    """nn.Conv2d(C, C, k, padding=p, groups=C) (same parameters / state-dict keys) on the HIP
    depthwise kernel (decoder_ops.dwconv2d); the z-conv stems' 3x3 (reference generator.py:839-868)."""

    def forward(self, x):
        if not x.is_cuda or self.groups != x.shape[1] or self.stride != (1, 1) or self.dilation != (1, 1) \
                or self.padding_mode != 'zeros' or self.padding[0] != self.padding[1]:
            return super().forward(x)
        from torch_utils.ops import decoder_ops
        return decoder_ops.dwconv2d(x.to(_conv_dtype(x)), self.weight, self.bias, self.padding[0])


class Conv1x1(nn.Conv2d):
    """nn.Conv2d(I, O, 1) as the decoder's 1x1 GEMM (decoder_ops.pointwise: HIP f32x6 / bf16 MFMA GEMM
    forward, data and weight gradient)."""

    def forward(self, x):
        if not x.is_cuda or self.kernel_size != (1, 1) or self.stride != (1, 1) or self.groups != 1 \
                or self.padding != (0, 0):
            return super().forward(x)
        from torch_utils.ops import decoder_ops
        B, C, H, W = x.shape
        x = x.to(_conv_dtype(x))
        y = decoder_ops.pointwise(self.weight.reshape(self.out_channels, C), x.reshape(B, C, H * W))
        y = y.reshape(B, self.out_channels, H, W)
        return y + self.bias.to(y.dtype)[None, :, None, None] if self.bias is not None else y


class LeakyReLU(nn.LeakyReLU):
    """nn.LeakyReLU on the HIP bias_act kernel (gain 1)."""

    def forward(self, x):
        from torch_utils.ops import bias_act
        return bias_act.bias_act(x, act='lrelu', alpha=self.negative_slope, gain=1.0)


class StyleSplit(nn.Module):
    """FC to 3*C features split as m1 * m2 + m3."""

    def __init__(self, in_channels, out_channels, **kwargs):
        super().__init__()
        self.proj = FullyConnectedLayer(in_channels, 3 * out_channels, **kwargs)

    def forward(self, x):
        m1, m2, m3 = self.proj(x).chunk(3, dim=1)
        return m1 * m2 + m3


class ScaleAdaptiveAvgPool2d(nn.Module):
    def __init__(self, scale_factor: float):
        super().__init__()
        self.scale_factor = scale_factor

    def forward(self, x):
        h = max(1, int(x.shape[2] * self.scale_factor))
        w = max(1, int(x.shape[3] * self.scale_factor))
        return F.adaptive_avg_pool2d(x, (h, w))
