"""conv2d / conv_transpose2d on our kernels (torch_utils/ops/conv2d_hip.py: csrc/im2col2d.hip + the exact-fp32 GEMM
csrc/sgemm.hip) -- the convolution inside conv2d_resample (reference torch_utils/ops/conv2d_resample.py:46-141) and
modulated_conv2d's grouped per-sample form (reference networks/generator.py:46-103) -- against torch's fp64
convolution: output, input, weight and bias gradients, strided / padded / grouped / transposed with output padding,
fp32 and bf16 inputs. Tolerances: fp32 max |err| <= 2e-6 of max |ref| (exact-fp32 products in another summation
order); bf16 inputs: one bf16 rounding of the output (8e-3), gradients in fp32 then rounded (1e-2)."""
import pytest
import torch
import torch.nn.functional as F

from torch_utils.ops import conv2d_hip, conv2d_gradfix

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / (b.double().abs().max() + 1e-30))


CONV = [  # B, Cin, H, W, O, k, stride, pad, groups
    (2, 8, 17, 19, 12, 3, 1, 1, 1),
    (3, 8, 16, 16, 8, 3, 2, 0, 2),
    (2, 6, 15, 13, 9, 4, 2, 1, 3),
    (1, 16, 9, 9, 20, 3, 1, 1, 4),       # modulated_conv2d: [1, B Cin, H, W], groups = B
    (4, 5, 8, 8, 7, 1, 1, 0, 1),
]


@pytest.mark.parametrize("case", CONV)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("bias", [False, True])
def test_conv2d_matches_torch(case, dtype, bias):
    B, C, H, W, O, k, s, p, G = case
    g = torch.Generator().manual_seed(B * 100 + C + O + k)
    x = torch.randn(B, C, H, W, generator=g).to(DEV, dtype)
    w = (torch.randn(O, C // G, k, k, generator=g) / (C // G * k * k) ** 0.5).to(DEV, dtype)
    b = torch.randn(O, generator=g).to(DEV, dtype) if bias else None
    leaves = [t.clone().requires_grad_(True) for t in (x, w) + ((b,) if bias else ())]
    y = conv2d_hip.conv2d(leaves[0], leaves[1], leaves[2] if bias else None, stride=s, padding=p, groups=G)
    ref_leaves = [t.detach().double().requires_grad_(True) for t in leaves]
    yr = F.conv2d(ref_leaves[0], ref_leaves[1], ref_leaves[2] if bias else None, stride=s, padding=p, groups=G)
    assert y.shape == yr.shape and y.dtype == dtype
    dy = torch.randn(yr.shape, generator=g).to(DEV)
    y.backward(dy.to(dtype))
    yr.backward(dy.double())
    tol_y, tol_g = (2e-6, 2e-6) if dtype == torch.float32 else (8e-3, 1e-2)
    assert _rel(y, yr) < tol_y
    for a, r in zip(leaves, ref_leaves):
        assert _rel(a.grad, r.grad) < tol_g, (a.shape, _rel(a.grad, r.grad))


TCONV = [  # B, Cin, H, W, Og, k, stride, pad, output_padding, groups
    (2, 8, 9, 7, 6, 3, 2, 0, 0, 1),
    (2, 8, 8, 8, 4, 4, 2, 1, 1, 2),
    (1, 12, 6, 6, 5, 3, 2, 1, 1, 3),
]


@pytest.mark.parametrize("case", TCONV)
@pytest.mark.parametrize("bias", [False, True])
def test_conv_transpose2d_matches_torch(case, bias):
    B, C, H, W, Og, k, s, p, op, G = case
    g = torch.Generator().manual_seed(B * 7 + C + Og + k)
    x = torch.randn(B, C, H, W, generator=g).to(DEV)
    w = (torch.randn(C, Og, k, k, generator=g) / (C * k * k) ** 0.5).to(DEV)
    b = torch.randn(Og * G, generator=g).to(DEV) if bias else None
    leaves = [t.clone().requires_grad_(True) for t in (x, w) + ((b,) if bias else ())]
    y = conv2d_hip.conv_transpose2d(leaves[0], leaves[1], leaves[2] if bias else None, stride=s, padding=p,
                                    output_padding=op, groups=G)
    ref_leaves = [t.detach().double().requires_grad_(True) for t in leaves]
    yr = F.conv_transpose2d(ref_leaves[0], ref_leaves[1], ref_leaves[2] if bias else None, stride=s, padding=p,
                            output_padding=op, groups=G)
    assert y.shape == yr.shape
    dy = torch.randn(yr.shape, generator=g).to(DEV)
    y.backward(dy)
    yr.backward(dy.double())
    assert _rel(y, yr) < 2e-6
    for a, r in zip(leaves, ref_leaves):
        assert _rel(a.grad, r.grad) < 2e-6, (a.shape, _rel(a.grad, r.grad))


def test_no_weight_gradients_switch():
    """conv2d_gradfix.no_weight_gradients() (reference conv2d_gradfix.py:22-35): no weight gradient, input
    gradient unchanged."""
    x = torch.randn(2, 4, 8, 8, device=DEV, requires_grad=True)
    w = torch.randn(6, 4, 3, 3, device=DEV, requires_grad=True)
    with conv2d_gradfix.no_weight_gradients():
        conv2d_hip.conv2d(x, w, padding=1).square().sum().backward()
    assert w.grad is None and x.grad is not None


def test_conv2d_resample_runs_own_convolution():
    """conv2d_resample on ROCm tensors: the convolution is ours (no aten convolution call), all four resampling
    branches (down, up via the transposed conv, 1x1 decimate / interpolate, plain)."""
    from torch.utils._python_dispatch import TorchDispatchMode
    from torch_utils.ops import conv2d_resample, upfirdn2d

    class Rec(TorchDispatchMode):
        hits = []

        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            if "convolution" in str(func):
                Rec.hits.append(str(func))
            return func(*args, **(kwargs or {}))

    f = upfirdn2d.setup_filter([1, 3, 3, 1], device=DEV)
    x = torch.randn(2, 8, 16, 16, device=DEV, requires_grad=True)
    with Rec():
        for w, up, down in ((torch.randn(6, 8, 3, 3, device=DEV), 1, 2), (torch.randn(6, 8, 3, 3, device=DEV), 2, 1),
                            (torch.randn(6, 8, 1, 1, device=DEV), 1, 2), (torch.randn(6, 8, 1, 1, device=DEV), 2, 1),
                            (torch.randn(6, 8, 3, 3, device=DEV), 1, 1)):
            y = conv2d_resample.conv2d_resample(x, w, f=f, up=up, down=down, padding=1)
            y.square().sum().backward()
    assert not Rec.hits, Rec.hits
