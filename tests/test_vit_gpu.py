"""GPU parity of the frozen-ViT fusions (csrc/vit.hip + the hipBLASLt GELU_BIAS epilogue)
against the plain PyTorch fp32 formulation of the same ops.

Tolerances: the residual stream h' = h + delta is fp32 and must be bit-identical; the
normalised output is compared after both sides round to the output dtype (bf16: 1 ulp =
2^-8 relative, so 1e-2 of the max magnitude; fp32: 1e-5).
"""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


@pytest.mark.parametrize("D", [256, 768, 1024, 2048])
@pytest.mark.parametrize("delta_dt", [None, torch.bfloat16, torch.float32])
@pytest.mark.parametrize("out_dt", [torch.bfloat16, torch.float32])
def test_residual_layer_norm(D, delta_dt, out_dt):
    from torch_utils.ops import vit_hip, kernel_timer
    torch.manual_seed(D)
    h = (torch.randn(3, 37, D, device=DEV) * 2 + 0.5)
    ln = nn.LayerNorm(D, eps=1e-6).to(DEV)
    with torch.no_grad():
        ln.weight.normal_(1.0, 0.1)
        ln.bias.normal_(0.0, 0.1)
    delta = None if delta_dt is None else torch.randn(3, 37, D, device=DEV).to(delta_dt)
    kernel_timer.enable(True)
    with torch.no_grad():
        h2, y = vit_hip.residual_layer_norm(h, delta, ln, out_dt)
    torch.cuda.synchronize()
    assert "residual_layer_norm" in kernel_timer.summary()
    kernel_timer.enable(False)
    href = h if delta is None else h + delta.float()
    assert torch.equal(h2, href)
    yref = F.layer_norm(href, (D,), ln.weight, ln.bias, ln.eps)
    assert y.dtype == out_dt
    assert _rel(y.float(), yref.to(out_dt).float()) < (1e-2 if out_dt == torch.bfloat16 else 1e-5)


def test_residual_layer_norm_rejects_autograd():
    from torch_utils.ops import vit_hip
    h = torch.randn(2, 256, device=DEV, requires_grad=True)
    with pytest.raises(RuntimeError):
        vit_hip.residual_layer_norm(h, None, nn.LayerNorm(256).to(DEV), torch.bfloat16)


def test_linear_gelu_tanh_epilogue():
    from torch_utils.ops import vit_ops
    torch.manual_seed(0)
    x = torch.randn(4, 64, 256, device=DEV).to(torch.bfloat16)
    w = (torch.randn(1024, 256, device=DEV) / 16).to(torch.bfloat16)
    b = torch.randn(1024, device=DEV) * 0.1
    with torch.no_grad():
        y = vit_ops.linear_gelu_tanh(x, w, b)
    ref = F.gelu(x.float() @ w.float().t() + b, approximate="tanh")
    assert y.dtype == torch.bfloat16
    assert _rel(y.float(), ref) < 1.5e-2


def test_siglip_fused_layers_match_unfused():
    """forward_features (LayerNorms fused into the residual adds) vs the layer-by-layer
    forward() formulation, same weights, bf16 GEMMs."""
    from networks.utils.vfms.siglip2_utils import SiglipVisionModel
    cfg = dict(hidden_size=256, num_hidden_layers=3, num_attention_heads=4, intermediate_size=1024,
               image_size=64, patch_size=16, num_channels=3, layer_norm_eps=1e-6, vision_use_head=False)
    m = SiglipVisionModel(cfg)
    m.reset_parameters(7)
    m = m.to(DEV).eval()
    px = torch.randn(2, 3, 64, 64, device=DEV)
    saved, last, _ = m.forward_features(px, [0, 2], want_last=True, want_pooled=False)
    vm = m.vision_model
    with torch.no_grad():
        h = vm.embeddings(px, torch.bfloat16)
        ref = {0: h}
        for i, layer in enumerate(vm.encoder.layers, start=1):
            h = layer(h, torch.bfloat16)
            ref[i] = h
        ref_last = F.layer_norm(h, (256,), vm.post_layernorm.weight, vm.post_layernorm.bias, vm.post_layernorm.eps)
    assert torch.equal(saved[0], ref[0])
    assert _rel(saved[2], ref[2]) < 2e-2
    assert last.dtype == torch.float32
    assert _rel(last, ref_last) < 3e-2
