"""Spectral normalisation of the D heads' SpectralConv1d weights on csrc/specnorm.hip (training mode,
one power iteration, dim 0) against torch.nn.utils.spectral_norm's own computation in float64
(reference networks/discriminator.py SpectralConv1d: SpectralNorm.apply(self, 'weight', 1, 0, 1e-12)):
the updated u / v buffers, the normalised weight and the weight gradient, including two forwards
before one backward (the GAN pattern torch's u / v clones exist for).

Tolerances (max |err| / max |ref|): fp32 dot products of <= 3456 terms against fp64: 2e-5 for u, v and
the weight, 1e-4 for the gradient."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return float((a.double().cpu() - b.double().cpu()).abs().max() / (b.double().abs().max().cpu() + 1e-30))


def _ref_step(W, u, v, eps=1e-12):
    """torch SpectralNorm.compute_weight(do_power_iteration=True) in float64 (u, v new values, W / sigma)."""
    Wm = W.reshape(W.shape[0], -1)
    v = torch.nn.functional.normalize(torch.mv(Wm.t(), u), dim=0, eps=eps)
    u = torch.nn.functional.normalize(torch.mv(Wm, v), dim=0, eps=eps)
    sigma = torch.dot(u, torch.mv(Wm, v))
    return u, v, W / sigma


@pytest.mark.parametrize("O,I,k", [(384, 384, 9), (384, 384, 1), (1, 384, 1), (70, 33, 3)])
def test_spectral_norm_matches_torch(O, I, k):
    from networks.discriminator import SpectralConv1d
    from torch_utils.ops import kernel_timer
    torch.manual_seed(O + I + k)
    m = SpectralConv1d(I, O, kernel_size=k, padding=k // 2, padding_mode='circular' if k > 1 else 'zeros').to(DEV)
    m.train()
    W64 = m.weight_orig.detach().double().requires_grad_(True)
    u0, v0 = m.weight_u.detach().double(), m.weight_v.detach().double()
    x1, x2 = torch.randn(2, I, 17, device=DEV), torch.randn(2, I, 17, device=DEV)
    g1, g2 = torch.randn(2, O, 17, device=DEV), torch.randn(2, O, 17, device=DEV)
    kernel_timer.enable(True)
    y1 = m(x1)
    w1 = m.weight.detach().clone()
    y2 = m(x2)                                               # second forward before the backward
    ((y1 * g1).sum() + (y2 * g2).sum()).backward()
    torch.cuda.synchronize()
    names = set(kernel_timer.summary())
    kernel_timer.enable(False)
    assert {'specnorm_fwd<f32>', 'specnorm_bwd<f32>'} <= names
    u1, v1, ws1 = _ref_step(W64, u0, v0)
    u2, v2, ws2 = _ref_step(W64, u1.detach(), v1.detach())
    assert _rel(w1, ws1) < 2e-5
    assert _rel(m.weight_u, u2) < 2e-5 and _rel(m.weight_v, v2) < 2e-5
    # the reference's weight gradient through both normalised weights (u, v detached per forward)
    u1d, v1d, u2d, v2d = u1.detach(), v1.detach(), u2.detach(), v2.detach()
    Wm = W64.reshape(O, -1)
    s1 = torch.dot(u1d, torch.mv(Wm, v1d))
    s2 = torch.dot(u2d, torch.mv(Wm, v2d))
    conv = lambda x, w: torch.nn.functional.conv1d(                    # noqa: E731
        torch.nn.functional.pad(x.double(), (k // 2, k // 2), mode='circular') if k > 1 else x.double(), w)
    ref = (conv(x1, W64 / s1) * g1.double()).sum() + (conv(x2, W64 / s2) * g2.double()).sum()
    gw, = torch.autograd.grad(ref, [W64])
    assert _rel(m.weight_orig.grad, gw) < 1e-4


def test_spectral_norm_eval_uses_torch_hook():
    """Outside training mode (no power iteration) the torch hook runs: same weight as torch's."""
    from networks.discriminator import SpectralConv1d
    torch.manual_seed(0)
    m = SpectralConv1d(64, 32, kernel_size=1).to(DEV).eval()
    ref = copy.deepcopy(m)
    with torch.no_grad():
        m(torch.randn(1, 64, 5, device=DEV))
    Wm = ref.weight_orig.reshape(32, -1)
    sigma = torch.dot(ref.weight_u, torch.mv(Wm, ref.weight_v))
    assert torch.allclose(m.weight, ref.weight_orig / sigma, rtol=1e-6, atol=0)


@pytest.mark.parametrize("B,C,L,k,p,circ", [(4, 384, 257, 9, 4, True), (2, 16, 5, 5, 2, True), (3, 8, 10, 3, 1, False),
                                            (2, 8, 10, 4, 2, False), (1, 4, 3, 7, 3, True)])
def test_im2col1d_matches_torch(B, C, L, k, p, circ):
    """The D heads' 1-D conv im2col (csrc/im2col1d.hip) vs F.pad + unfold + permute + reshape: the gather
    bit-exact, its adjoint (a sum of k terms) within 1e-6."""
    from torch_utils.ops import patchgan_hip
    import torch.nn.functional as F
    g0 = torch.Generator().manual_seed(B * L + k)
    x = torch.randn(B, C, L, generator=g0).to(DEV)
    assert patchgan_hip.im2col1d_supported(x, k, p, circ)
    xa = x.clone().requires_grad_(True)
    xb = x.clone().requires_grad_(True)
    cols = patchgan_hip.im2col1d(xa, k, p, circ)
    xp = F.pad(xb, (p, p), mode='circular' if circ else 'constant')
    ref = xp.unfold(2, k, 1).permute(0, 1, 3, 2).reshape(B, C * k, -1)
    assert cols.shape == ref.shape and torch.equal(cols, ref)
    g = torch.randn(ref.shape, generator=g0).to(DEV)
    cols.backward(g)
    ref.backward(g)
    assert _rel(xa.grad, xb.grad) < 1e-6


@pytest.mark.parametrize("B,C,O,L,k,p,circ,bias", [(32, 384, 384, 196, 9, 4, True, True), (8, 384, 384, 196, 1, 0, False, True),
                                                   (8, 384, 64, 196, 1, 0, False, False), (3, 8, 5, 10, 3, 1, False, True),
                                                   (2, 16, 7, 5, 5, 2, True, False)])
@pytest.mark.parametrize("own", ["sgemm", "torch", "hip"], ids=["sgemm", "hipblaslt", "f32x6"])
def test_conv1d_folded_matches_conv1d(B, C, O, L, k, p, circ, bias, own, monkeypatch):
    """The D heads' Conv1d as batch-folded GEMMs (patchgan_hip.conv1d_folded: cols [C k, B Lo] from
    vfm_im2col1d_cbl_f32, the exact-fp32 MFMA GEMM (csrc/sgemm.hip, default) -- or, for A/B, hipBLASLt's exact
    fp32 / our f32x6 GEMM -- folded col2im) vs F.conv1d (circular padding through
    F.pad) in fp32 and in fp64: output and every gradient within 1e-5 of max |ref| (exact fp32 products
    in another summation order: the k = 9 input gradient sums 3456 products; measured 3.2e-6 against
    F.conv1d's fp32 and 3.0e-6 against fp64, where MIOpen's own fp32 is 6e-7 from fp64), and within
    5e-6 of the fp64 result; the folded gather bit-identical to the per-sample one transposed."""
    from torch_utils.ops import patchgan_hip
    import torch.nn.functional as F
    monkeypatch.setattr(patchgan_hip, "_DHEAD", own)
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    g0 = torch.Generator().manual_seed(B * O + k)
    x = torch.randn(B, C, L, generator=g0).to(DEV)
    w = (torch.randn(O, C, k, generator=g0) / (C * k) ** 0.5).to(DEV)
    b = torch.randn(O, generator=g0).to(DEV) if bias else None
    gy = torch.randn(B, O, L + 2 * p - k + 1, generator=g0).to(DEV)
    assert patchgan_hip.conv1d_folded_supported(x, k, p, circ)
    leaves = [t.clone().requires_grad_(True) for t in (x, w) + ((b,) if bias else ())]
    ref_leaves = [t.clone().requires_grad_(True) for t in (x, w) + ((b,) if bias else ())]
    y = patchgan_hip.conv1d_folded(leaves[0], leaves[1].reshape(O, -1), leaves[2] if bias else None, k, p, circ)
    def ref(leaves_):
        xr = F.pad(leaves_[0], (p, p), mode='circular') if circ else leaves_[0]
        return F.conv1d(xr, leaves_[1], leaves_[2] if bias else None, padding=0 if circ else p)

    yr = ref(ref_leaves)
    l64 = [t.detach().double().requires_grad_(True) for t in ref_leaves]
    y64 = ref(l64)
    assert y.shape == yr.shape and _rel(y, yr) < 1e-5
    y.backward(gy)
    yr.backward(gy)
    y64.backward(gy.double())
    assert _rel(y, y64) < 5e-6
    for a, r, r64 in zip(leaves, ref_leaves, l64):
        assert _rel(a.grad, r.grad) < 1e-5
        assert _rel(a.grad, r64.grad) < 5e-6
    cols = torch.empty(C * k, B, L + 2 * p - k + 1, device=DEV)
    assert patchgan_hip._lib.vfm_im2col1d_cbl_f32(x.data_ptr(), cols.data_ptr(), B, C, L, k, p, int(circ),
                                                  patchgan_hip._stream()) == 0
    assert torch.equal(cols.transpose(0, 1), patchgan_hip.im2col1d(x, k, p, circ).view(B, C * k, -1))
