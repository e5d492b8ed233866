"""Grouped spectral norm of the D heads (torch_utils/ops/specnorm_group.py, csrc/specnorm.hip
vfm_specnorm_group_*) against the per-weight path (vfm_specnorm_fwd / _bwd, itself pinned against torch's
SpectralNorm by tests/test_specnorm_gpu.py): W / sigma, the updated u / v buffers and the weight gradients,
bit-identical, over several training forwards (the first one records the plan)."""
import copy

import pytest
import torch

from networks.discriminator import SpectralConv1d
from torch_utils.ops import specnorm_group

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


class _Heads(torch.nn.Module):
    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.convs = torch.nn.ModuleList([SpectralConv1d(24, 40, 1), SpectralConv1d(40, 32, 9, padding=4,
                                                                                    padding_mode='circular'),
                                          SpectralConv1d(32, 16, 3, padding=1), SpectralConv1d(16, 1, 1)])

    def forward(self, x):
        for c in self.convs:
            x = torch.nn.functional.leaky_relu(c(x), 0.2)
        return x


def _step(net, x, group):
    for p in net.parameters():
        p.grad = None
    if group:
        with specnorm_group.SpecNormGroup(net):
            y = net(x)
    else:
        y = net(x)
    (y * torch.linspace(-1, 1, y.numel(), device=DEV).reshape(y.shape)).sum().backward()
    return y.detach()


def test_specnorm_group_matches_per_weight():
    a = _Heads().to(DEV).train()
    b = copy.deepcopy(a)
    g = torch.Generator().manual_seed(1)
    for it in range(4):
        x = torch.randn(3, 24, 50, generator=g).to(DEV)
        ya, yb = _step(a, x, False), _step(b, x, True)
        assert torch.equal(ya, yb), it
        for ca, cb in zip(a.convs, b.convs):
            assert torch.equal(ca.weight_u, cb.weight_u) and torch.equal(ca.weight_v, cb.weight_v), it
            assert torch.equal(ca.weight_orig.grad, cb.weight_orig.grad), it
    assert specnorm_group._PLANS.get(b) is not None and len(specnorm_group._PLANS[b]) == 4
