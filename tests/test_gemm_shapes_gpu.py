"""The HIP GEMM on the exact operand shapes/strides the training path hands it (through
decoder_ops.pointwise and ops.linear autograd), against the torch fp32 formulation:
projected-discriminator heads (1x1 and unfolded k=9 circular convs over 196 tokens),
fusion-adapter projections, decoder fp32 1x1 convs. Tolerance 5e-5 of max |ref| (the
3-term split), on outputs and every gradient."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / (b.double().abs().max() + 1e-30))


@pytest.mark.parametrize("B,O,I,P", [(2, 64, 384, 196), (2, 64, 576, 196), (2, 384, 3456, 196), (3, 256, 512, 1024),
                                     (2, 2048, 512, 64), (2, 512, 2048, 256), (4, 512, 256, 16), (4, 256, 512, 144),
                                     (32, 2048, 512, 4)])
def test_pointwise_autograd_shapes(B, O, I, P):
    from torch_utils.ops import decoder_ops
    g = torch.Generator().manual_seed(O + I + P)
    w = (torch.randn(O, I, generator=g) / I ** 0.5).to(DEV).requires_grad_(True)
    x = torch.randn(B, I, P, generator=g).to(DEV).requires_grad_(True)
    dy = torch.randn(B, O, P, generator=g).to(DEV)
    y = decoder_ops.pointwise(w, x)
    y.backward(dy)
    wr = w.detach().clone().requires_grad_(True)
    xr = x.detach().clone().requires_grad_(True)
    yr = torch.matmul(wr, xr)
    yr.backward(dy)
    assert _rel(y, yr) < 5e-5
    assert _rel(x.grad, xr.grad) < 5e-5
    assert _rel(w.grad, wr.grad) < 5e-5


@pytest.mark.parametrize("N,K,Nout", [(2 * 1024, 1024, 3072), (2 * 1024, 1024, 64), (2 * 256, 768, 3072),
                                      (2 * 196, 384, 1152)])
def test_linear_autograd_shapes(N, K, Nout):
    from torch_utils.ops.linear import linear
    g = torch.Generator().manual_seed(N + K + Nout)
    x = torch.randn(N, K, generator=g).to(DEV).requires_grad_(True)
    w = (torch.randn(Nout, K, generator=g) / K ** 0.5).to(DEV).requires_grad_(True)
    b = torch.randn(Nout, generator=g).to(DEV).requires_grad_(True)
    dy = torch.randn(N, Nout, generator=g).to(DEV)
    y = linear(x, w, b)
    y.backward(dy)
    xr, wr, br = (t.detach().clone().requires_grad_(True) for t in (x, w, b))
    yr = torch.nn.functional.linear(xr, wr, br)
    yr.backward(dy)
    for a, r in ((y, yr), (x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert _rel(a, r) < 5e-5
