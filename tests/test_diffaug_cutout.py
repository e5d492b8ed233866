"""DiffAugment cutout (training/diffaug.py rand_cutout: hole mask from range comparisons, no device scatter)
against the reference's clamped-grid scatter (reference training/diffaug.py:89-104, restated below) on the same
seeded draws: identical output (the mask is 0/1), every offset including the clamped edges, odd and even hole
sizes, square and non-square planes; CPU."""
import pytest
import torch


def _reference_cutout(x, ratio=0.2):
    cs = int(x.size(2) * ratio + 0.5), int(x.size(3) * ratio + 0.5)
    ox = torch.randint(0, x.size(2) + (1 - cs[0] % 2), size=[x.size(0), 1, 1], device=x.device)
    oy = torch.randint(0, x.size(3) + (1 - cs[1] % 2), size=[x.size(0), 1, 1], device=x.device)
    gb, gx, gy = torch.meshgrid(torch.arange(x.size(0)), torch.arange(cs[0]), torch.arange(cs[1]), indexing='ij')
    gx = torch.clamp(gx + ox - cs[0] // 2, min=0, max=x.size(2) - 1)
    gy = torch.clamp(gy + oy - cs[1] // 2, min=0, max=x.size(3) - 1)
    mask = torch.ones(x.size(0), x.size(2), x.size(3), dtype=x.dtype)
    mask[gb, gx, gy] = 0
    return x * mask.unsqueeze(1)


@pytest.mark.parametrize("B,C,H,W", [(64, 3, 32, 32), (64, 2, 20, 36), (128, 1, 7, 5), (32, 3, 224, 224)])
@pytest.mark.parametrize("ratio", [0.2, 0.5])
def test_cutout_matches_reference_scatter(B, C, H, W, ratio):
    from training import diffaug
    x = torch.randn(B, C, H, W, generator=torch.Generator().manual_seed(H * W + B))
    for seed in range(3):
        torch.manual_seed(seed)
        a = diffaug.rand_cutout(x, ratio)
        torch.manual_seed(seed)
        b = _reference_cutout(x, ratio)
        assert torch.equal(a, b), (seed, (a != b).sum())
