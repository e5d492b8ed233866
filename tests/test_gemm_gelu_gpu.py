"""ConvNeXt-MLP GEMMs with the GELU in the epilogue (csrc/gemm9.hip vfm_gemm9_gelu) against the plain
PyTorch fp32 reference of the same ops (reference networks/utils/convnext_utils.py:135-142:
pwconv1 -> GELU(h * s + b1) -> ..., and its backward).

Tolerances (max |err| / max |ref|): h and dg are bf16 roundings of fp32-accumulated products, so a
different summation order moves them by at most one bf16 ulp (2^-8 relative): 8e-3. g is compared
against GELU of OUR h (the epilogue's own arithmetic, exact-erf GELU to ~1e-7): 8e-3 (one output
rounding). dh / the row sums are compared against an fp32 chain fed with a bf16-rounded dg:
8e-3 / 2e-3 (sums over hundreds of columns of terms that carry one bf16 rounding each).
The layer test runs the fused autograd Function against the unfused chain of HIP ops
(gemm9 1x1s + scale_bias_gelu + layer_scale_residual) at the two widths it serves (C = 256, 512)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / (b.double().abs().max() + 1e-30))


def _bf(t):
    return t.to(torch.bfloat16).float()


@pytest.mark.parametrize("O,I,P,B", [(1024, 256, 4096, 2), (2048, 512, 1024, 3), (320, 128, 200, 2),
                                     (512, 64, 264, 1), (1024, 256, 16384, 2)])
@pytest.mark.parametrize("with_s", [True, False])
def test_gemm_gelu_forward(O, I, P, B, with_s):
    from torch_utils.ops import decoder_hip
    g0 = torch.Generator().manual_seed(O + I + P)
    w = (torch.randn(O, I, generator=g0) / I ** 0.5).to(torch.bfloat16).to(DEV)
    m = torch.randn(B, I, P, generator=g0).to(torch.bfloat16).to(DEV)
    s = (torch.rand(B, O, generator=g0) + 0.5).to(DEV) if with_s else None
    b1 = torch.randn(O, generator=g0).to(DEV)
    h, g = decoder_hip.gemm_gelu_fwd(w, m, s, b1, want_h=True)
    href = w.float() @ m.float()
    assert _rel(h.float(), href) < 8e-3
    z = h.float() * (s[:, :, None] if s is not None else 1.0) + b1[None, :, None]
    assert _rel(g.float(), F.gelu(z)) < 8e-3
    _, g2 = decoder_hip.gemm_gelu_fwd(w, m, s, b1, want_h=False)
    assert torch.equal(g, g2)


@pytest.mark.parametrize("O,C,P,B", [(1024, 256, 4096, 2), (2048, 512, 1024, 2), (320, 128, 200, 3),
                                     (1024, 256, 16384, 2)])
@pytest.mark.parametrize("with_s", [True, False])
def test_gemm_gelu_backward(O, C, P, B, with_s):
    from torch_utils.ops import decoder_hip
    g0 = torch.Generator().manual_seed(7 * O + C + P)
    w2 = (torch.randn(C, O, generator=g0) / O ** 0.5).to(torch.bfloat16).to(DEV)
    dy = torch.randn(B, C, P, generator=g0).to(torch.bfloat16).to(DEV)
    h = torch.randn(B, O, P, generator=g0).to(torch.bfloat16).to(DEV)
    s = (torch.rand(B, O, generator=g0) + 0.5).to(DEV) if with_s else None
    b1 = torch.randn(O, generator=g0).to(DEV)
    dh, ds, db1 = decoder_hip.gemm_gelu_bwd(w2.t().contiguous(), dy, h, s, b1)
    dg = _bf(w2.t().float() @ dy.float())
    sc = s[:, :, None] if s is not None else 1.0
    zz = (h.float() * sc + b1[None, :, None]).requires_grad_(True)
    gz, = torch.autograd.grad(F.gelu(zz), zz, dg)
    assert _rel(dh.float(), gz * sc) < 8e-3
    assert _rel(db1, gz.sum((0, 2))) < 2e-3
    if with_s:
        assert _rel(ds, (gz * h.float()).sum(2)) < 2e-3
    else:
        assert ds is None


@pytest.mark.parametrize("C,H", [(256, 32), (512, 16)])
def test_convnext_mlp_gemm_layer_matches_unfused(C, H):
    """Fused (gemm9 + GELU epilogues) vs unfused HIP chain, forward output and every gradient."""
    from torch_utils.ops import decoder_hip
    assert C in decoder_hip.GEMM_MLP_TESTED
    g0 = torch.Generator().manual_seed(C)
    B, P = 2, H * H
    m = torch.randn(B, C, P, generator=g0).to(torch.bfloat16).to(DEV)
    x_in = torch.randn(B, C, P, generator=g0).to(torch.bfloat16).to(DEV)
    w1 = (torch.randn(4 * C, C, generator=g0) / C ** 0.5).to(DEV)
    w2 = (torch.randn(C, 4 * C, generator=g0) / (2 * C ** 0.5)).to(DEV)
    dcoef = (torch.rand(B, 4 * C, generator=g0) + 0.5).to(DEV)
    b1, b2 = torch.randn(4 * C, generator=g0).to(DEV), torch.randn(C, generator=g0).to(DEV)
    gamma = torch.rand(C, generator=g0).to(DEV)
    dout = torch.randn(B, C, P, generator=g0).to(torch.bfloat16).to(DEV)
    leaves = [m, w1, dcoef, b1, w2, b2, gamma, x_in]

    def run(fused):
        ts = [t.detach().clone().requires_grad_(True) for t in leaves]
        if fused:
            out = decoder_hip.convnext_mlp(*ts)
        else:
            h = decoder_hip.pointwise(ts[1], ts[0])
            gg = decoder_hip.scale_bias_gelu(h, ts[2], ts[3])
            y = decoder_hip.pointwise(ts[4], gg)
            out = decoder_hip.layer_scale_residual(y, ts[5], ts[6], ts[7])
        out.backward(dout)
        return out.detach().float(), [t.grad.float() for t in ts]

    with torch.no_grad():
        nog = decoder_hip.convnext_mlp_nograd(*leaves)
    o1, g1 = run(True)
    o0, g0_ = run(False)
    assert torch.equal(nog, o1.to(torch.bfloat16))
    assert _rel(o1, o0) < 8e-3
    names = ["m", "w1", "dcoef", "b1", "w2", "b2", "gamma", "x_in"]
    for n, a, b in zip(names, g1, g0_):
        # bf16 intermediate roundings land on different products: norms within 1e-2, entries 3e-2
        assert float((a - b).norm() / (b.norm() + 1e-30)) < 1e-2, n
        assert _rel(a, b) < 3e-2, n
