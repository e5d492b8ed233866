"""LayerNorm with a backward to its input through frozen parameters (csrc/vit.hip ln2_fwd / ln2_bwd;
the DINOv2 discriminator backbone's norm1 / norm2 in the G phase, reference HF Dinov2Layer): forward
and input gradient against torch's fp32 LayerNorm evaluated in fp64, within 2e-5 (fp32 forward) /
1e-4 (gradient) of the reference's max magnitude, bf16 outputs within one bf16 rounding; the native
kernels asserted to have run, and the routing through vit_ops.layer_norm."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


@pytest.mark.parametrize("rows,D", [(6304, 384), (1, 128), (37, 256), (1000, 768), (5, 1024), (130, 640)])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("affine", [True, False])
def test_layer_norm_grad(rows, D, out_dtype, affine):
    from torch_utils.ops import kernel_timer as kt, vit_hip
    torch.manual_seed(rows + D)
    ln = torch.nn.LayerNorm(D, eps=1e-6, elementwise_affine=affine).to(DEV)
    if affine:
        with torch.no_grad():
            ln.weight.copy_(1 + 0.2 * torch.randn(D))
            ln.bias.copy_(0.1 * torch.randn(D))
    ln.requires_grad_(False)
    x = (torch.randn(rows, D, device=DEV) * 2 + 0.5).requires_grad_(True)
    assert vit_hip.layer_norm_grad_supported(x, ln)
    kt.enable(True)
    y = vit_hip.layer_norm_grad(x, ln, out_dtype)
    dy = torch.randn(rows, D, device=DEV).to(out_dtype)
    y.backward(dy)
    torch.cuda.synchronize()
    names = {k.split("<")[0] for k in kt.summary()}
    kt.enable(False)
    assert {"layer_norm_fwd", "layer_norm_bwd"} <= names, names
    xr = x.detach().double().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (D,), None if not affine else ln.weight.double(),
                                        None if not affine else ln.bias.double(), 1e-6)
    yr.backward(dy.double())
    assert y.dtype == out_dtype
    assert _rel(y, yr) < (2e-5 if out_dtype == torch.float32 else 8e-3)
    assert _rel(x.grad, xr.grad) < 1e-4, _rel(x.grad, xr.grad)


def test_vit_ops_layer_norm_routes_grad_inputs(monkeypatch):
    """With VFM_LN_GRAD on, vit_ops.layer_norm: an input that needs a gradient through frozen parameters takes the native
    op (3-D stream as in the DINO blocks); trainable parameters keep torch's LayerNorm."""
    from torch_utils.ops import kernel_timer as kt, vit_hip, vit_ops
    monkeypatch.setattr(vit_hip, "LN_GRAD", True)         # the routing switch (off by default)
    torch.manual_seed(0)
    ln = torch.nn.LayerNorm(384, eps=1e-6).to(DEV).requires_grad_(False)
    h = torch.randn(2, 197, 384, device=DEV, requires_grad=True)
    R = torch.randn(2, 197, 384, device=DEV)
    kt.enable(True)
    y = vit_ops.layer_norm(h, ln, torch.float32)
    (y * R).sum().backward()
    torch.cuda.synchronize()
    assert any(k.startswith("layer_norm_fwd") for k in kt.summary())
    kt.enable(False)
    hr = h.detach().clone().requires_grad_(True)
    (torch.nn.functional.layer_norm(hr.double(), (384,), ln.weight.double(), ln.bias.double(), 1e-6)
     * R.double()).sum().backward()
    assert _rel(h.grad, hr.grad) < 1e-4
    ln.requires_grad_(True)
    kt.enable(True)
    vit_ops.layer_norm(h, ln, torch.float32)
    assert not any(k.startswith("layer_norm_fwd") for k in kt.summary())
    kt.enable(False)


def test_vit_ops_layer_norm_frozen_input_trainable_affine(monkeypatch):
    """An input that needs no gradient through a TRAINABLE LayerNorm (grad enabled) keeps torch's LayerNorm, so the
    weight and bias gradients exist (the native ops' affine parameters are frozen)."""
    from torch_utils.ops import kernel_timer as kt, vit_hip, vit_ops
    monkeypatch.setattr(vit_hip, "LN_GRAD", True)
    torch.manual_seed(1)
    ln = torch.nn.LayerNorm(384, eps=1e-6).to(DEV)
    h = torch.randn(2, 197, 384, device=DEV)
    kt.enable(True)
    y = vit_ops.layer_norm(h, ln, torch.float32)
    y.square().sum().backward()
    torch.cuda.synchronize()
    names = set(kt.summary())
    kt.enable(False)
    assert not any(k.startswith("layer_norm_fwd") or k.startswith("residual_layer_norm") for k in names), names
    assert ln.weight.grad is not None and ln.bias.grad is not None
    w = ln.weight.detach().double().requires_grad_(True)
    torch.nn.functional.layer_norm(h.double(), (384,), w, ln.bias.double(), 1e-6).square().sum().backward()
    assert _rel(ln.weight.grad, w.grad) < 1e-4
