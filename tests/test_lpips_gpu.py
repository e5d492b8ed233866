"""LPIPS distance head (csrc/lpips.hip) against the reference expression of training/lpips.py
(`normalize_tensor` → diff² → `lin` 1×1 → `spatial_average`) evaluated in float64 by torch.
Tolerance: fp32 kernel vs fp64 reference, relative 2e-5 on the head value and 1e-4 (max-abs
over max-abs) on the feature gradients."""
import pytest
import torch

from torch_utils.ops import lpips_ops


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / (b.double().abs().max() + 1e-30))


def test_head_ref_is_the_reference_expression():
    from training.lpips import normalize_tensor, spatial_average
    g = torch.Generator().manual_seed(0)
    f0, f1 = torch.rand(2, 16, 5, 7, generator=g), torch.rand(2, 16, 5, 7, generator=g)
    w = torch.rand(1, 16, 1, 1, generator=g)
    d = (normalize_tensor(f0) - normalize_tensor(f1)) ** 2
    exp = spatial_average(torch.nn.functional.conv2d(d, w), keepdim=True)
    assert torch.allclose(lpips_ops.head_ref(f0, f1, w), exp, rtol=1e-6, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["nchw", "nhwc"])
@pytest.mark.parametrize("B,C,H,W", [(3, 64, 33, 31), (2, 130, 16, 16), (4, 512, 16, 16), (2, 64, 256, 256),
                                     (2, 256, 9, 7)])
def test_lpips_head_matches_reference(B, C, H, W, layout):
    """nhwc: channels_last features (the HIP VGG16 stack's taps) run the NHWC kernels in place
    (C = 130 is not covered and takes the NCHW kernel through a contiguous copy)."""
    dev = torch.device("cuda:0")
    fmt = torch.channels_last if layout == "nhwc" else torch.contiguous_format
    g = torch.Generator().manual_seed(B * C + H)
    # ReLU-like features (non-negative, some exact zeros) as the VGG taps are
    f0 = torch.relu(torch.randn(B, C, H, W, generator=g))
    f1 = torch.relu(f0 + 0.3 * torch.randn(B, C, H, W, generator=g))
    w = torch.rand(C, generator=g) / C
    x0 = f0.to(dev).to(memory_format=fmt).requires_grad_(True)
    x1 = f1.to(dev).to(memory_format=fmt).requires_grad_(True)
    out = lpips_ops.lpips_head(x0, x1, w.to(dev))
    gout = torch.rand(B, 1, 1, 1, generator=g)
    out.backward(gout.to(dev))
    r0 = f0.double().requires_grad_(True)
    r1 = f1.double().requires_grad_(True)
    ref = lpips_ops.head_ref(r0, r1, w.double())
    ref.backward(gout.double())
    assert out.shape == (B, 1, 1, 1)
    assert _rel(out.cpu(), ref) < 2e-5
    assert _rel(x1.grad.cpu(), r1.grad) < 1e-4
    assert _rel(x0.grad.cpu(), r0.grad) < 1e-4


@pytest.mark.gpu
def test_lpips_head_only_target_grad_and_zero_pixel():
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(5)
    f0 = torch.relu(torch.randn(2, 64, 8, 8, generator=g))
    f1 = torch.relu(torch.randn(2, 64, 8, 8, generator=g))
    f1[0, :, 3, 4] = 0.0                                    # all-zero pixel: gradient defined as finite
    w = torch.rand(64, generator=g) / 64
    x1 = f1.to(dev).requires_grad_(True)
    out = lpips_ops.lpips_head(f0.to(dev), x1, w.to(dev))
    out.sum().backward()
    assert torch.isfinite(x1.grad).all()
    m = torch.ones_like(f1, dtype=torch.bool)
    m[0, :, 3, 4] = False
    r1 = f1.double().requires_grad_(True)
    lpips_ops.head_ref(f0.double(), r1, w.double()).sum().backward()
    assert _rel(out.cpu(), lpips_ops.head_ref(f0.double(), f1.double(), w.double())) < 2e-5
    assert _rel(x1.grad.cpu()[m], r1.grad[m]) < 1e-4


@pytest.mark.gpu
def test_lpips_module_hip_head_matches_torch_head():
    """Whole LPIPS on cuda:0 with the HIP head vs the same module with the torch head. Both run
    the same HIP VGG16 stack (torch_utils/ops/vgg_hip.py: fixed accumulation order, so the
    features and the backward chain are identical) and only the head differs: value 1e-5,
    input gradient 1e-4 of max. Against the CPU module: value 1e-4; the input gradient in
    relative L2 norm (1e-2), since the GPU stack's ~2^-16 forward rounding flips the odd ReLU /
    max-pool decision of the CPU's fp32 stack, which moves single gradient entries by O(their
    size); the kernels themselves are checked through the same decisions in test_vgg_gpu.py."""
    from training.lpips import LPIPS
    torch.manual_seed(0)
    m = LPIPS().eval()
    g = torch.Generator().manual_seed(1)
    a = torch.rand(2, 3, 64, 64, generator=g) * 2 - 1
    b = (a + 0.2 * torch.randn(2, 3, 64, 64, generator=g)).clamp(-1, 1)
    bc = b.clone().requires_grad_(True)
    ref = m(a, bc)
    ref.sum().backward()
    md = m.to("cuda:0")
    res = {}
    for impl in ("ref", "cuda"):
        md.head_impl = impl
        bg = b.to("cuda:0").requires_grad_(True)
        out = md(a.to("cuda:0"), bg)
        out.sum().backward()
        res[impl] = (out.detach().cpu(), bg.grad.cpu())
    md.head_impl = "cuda"
    assert _rel(res["cuda"][0], res["ref"][0]) < 1e-5
    assert _rel(res["cuda"][1], res["ref"][1]) < 1e-4
    assert _rel(res["cuda"][0], ref) < 1e-4
    l2 = float((res["cuda"][1].double() - bc.grad.double()).norm() / bc.grad.double().norm())
    assert l2 < 1e-2, l2


@pytest.mark.gpu
def test_lpips_module_under_no_grad():
    """LPIPS under torch.no_grad() (tools/reconstruct/evaluate.py): the paired VGG16 pass runs its
    forward outside autograd (custom_ops.FastFunction's stand-in ctx) and gives the grad-mode value."""
    from training.lpips import LPIPS
    torch.manual_seed(0)
    m = LPIPS().eval().to("cuda:0")
    g = torch.Generator().manual_seed(3)
    a = (torch.rand(2, 3, 64, 64, generator=g) * 2 - 1).to("cuda:0")
    b = (a.cpu() + 0.2 * torch.randn(2, 3, 64, 64, generator=g)).clamp(-1, 1).to("cuda:0")
    with torch.no_grad():
        v0 = m(a, b)
    v1 = m(a, b.clone().requires_grad_(True)).detach()
    assert v0.shape == v1.shape and _rel(v0.cpu(), v1.cpu()) < 1e-6
