"""The decoder's style path (csrc/style.hip: StyleSplit(FullyConnectedLayer) + demodulation, reference
networks/utils/shared.py StyleSplit / FullyConnectedLayer and networks/utils/convnext_utils.py:60-66)
and channel RMS norm (csrc/rmsnorm.hip, reference networks/utils/gigagan_utils.py:31-39) against a
plain PyTorch float64 restatement of the same ops, forward and every gradient.

Tolerances (max |err| / max |ref|): both are fp32 FMA chains (dots of <= 2048 terms) against fp64:
2e-5 forward, 1e-4 for the gradients (two chained dots)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _recording():
    from torch_utils.ops import kernel_timer
    kernel_timer.enable(True)
    return kernel_timer


def _recorded(kt):
    torch.cuda.synchronize()
    names = set(kt.summary())
    kt.enable(False)
    return names


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / (b.double().abs().max() + 1e-30))


def _style_ref(w, A, ab, W1, wg, bg, eps):
    m = F.linear(w, A * wg, ab * bg)
    m1, m2, m3 = m.chunk(3, dim=1)
    s = m1 * m2 + m3
    d = torch.rsqrt(s.square() @ W1.square().t() + eps) if W1 is not None else None
    return s, d


@pytest.mark.parametrize("B,C,WD,demod", [(32, 512, 512, True), (32, 128, 512, True), (5, 40, 72, True),
                                          (3, 16, 24, False), (33, 64, 100, True)])
def test_style_demod_matches_fp64(B, C, WD, demod):
    from torch_utils.ops import decoder_hip
    g = torch.Generator().manual_seed(B * 1000 + C)
    nws = 3
    ws = torch.randn(B, nws, WD, generator=g).to(DEV)
    A = torch.randn(3 * C, WD, generator=g).to(DEV)
    ab = (torch.randn(3 * C, generator=g) * 0.3 + 1).to(DEV)
    W1 = (torch.randn(4 * C, C, generator=g) * 0.02).to(DEV) if demod else None
    wg, bg, eps = 1 / math.sqrt(WD), 1.0, 1e-8
    leaves = [ws, A, ab] + ([W1] if demod else [])
    ts = [t.clone().requires_grad_(True) for t in leaves]
    w = ts[0].unbind(1)[1]                                   # a strided row slice, as the synthesis feeds it
    kt = _recording()
    s, d = decoder_hip.style_demod(w, ts[1], ts[2], ts[3] if demod else None, wg, bg, eps)
    t64 = [t.detach().double().requires_grad_(True) for t in leaves]
    s0, d0 = _style_ref(t64[0].unbind(1)[1], t64[1], t64[2], t64[3] if demod else None, wg, bg, eps)
    assert _rel(s, s0) < 2e-5
    gs = torch.randn(s.shape, generator=g).to(DEV)
    outs, outs0, grads = [s], [s0], [gs]
    if demod:
        assert d.shape == (B, 4 * C) and _rel(d, d0) < 2e-5
        gd = torch.randn(d.shape, generator=g).to(DEV)
        outs.append(d)
        outs0.append(d0)
        grads.append(gd)
    got = torch.autograd.grad(outs, ts, grads)
    assert {'style_demod_fwd<f32>', 'style_demod_bwd<f32>'} <= _recorded(kt)
    ref = torch.autograd.grad(outs0, t64, [x.double() for x in grads])
    for name, a, b in zip(["ws", "A", "ab", "W1"], got, ref):
        assert _rel(a, b) < 1e-4, name


def test_style_demod_layer_matches_torch_path():
    """The ConvNeXt layer's style path through decoder_ops (HIP) vs its torch formulation."""
    from networks.utils.shared import StyleSplit
    from torch_utils.ops import decoder_ops
    decoder_ops.STYLE_HIP, prev = True, decoder_ops.STYLE_HIP
    torch.manual_seed(0)
    aff = StyleSplit(512, 256, bias_init=1).to(DEV)
    w1 = (torch.randn(1024, 256) * 0.02).to(DEV)
    w = torch.randn(8, 512, device=DEV)
    s, d = decoder_ops.style_and_demod(aff, w, w1)
    s0 = aff(w).float()
    d0 = decoder_ops.demod_coefficients(w1, s0)
    decoder_ops.STYLE_HIP = prev
    assert _rel(s, s0) < 2e-5 and _rel(d, d0) < 2e-5


@pytest.mark.parametrize("B,C,H,W", [(4, 512, 8, 8), (2, 512, 16, 16), (3, 256, 32, 32), (2, 40, 5, 7)])
def test_channel_rms_norm_matches_fp64(B, C, H, W):
    from networks.utils.gigagan_utils import ChannelRMSNorm
    g = torch.Generator().manual_seed(C + H)
    x = torch.randn(B, C, H, W, generator=g)
    x[0, :, 0, 0] = 0                                        # a clamped (zero-norm) column
    norm = ChannelRMSNorm(C).to(DEV)
    with torch.no_grad():
        norm.gamma.copy_(torch.rand(C, 1, 1, generator=g) + 0.5)
    xg = x.to(DEV).requires_grad_(True)
    kt = _recording()
    y = norm(xg)
    x64 = x.double().requires_grad_(True)
    g64 = norm.gamma.detach().double().cpu().requires_grad_(True)
    y0 = F.normalize(x64, dim=1) * norm.scale * g64
    assert _rel(y.cpu(), y0) < 2e-5
    dy = torch.randn(y.shape, generator=g)
    gx, gg = torch.autograd.grad(y, [xg, norm.gamma], dy.to(DEV))
    assert {'channel_rms_norm_fwd<f32>', 'channel_rms_norm_bwd<f32>'} <= _recorded(kt)
    gx0, gg0 = torch.autograd.grad(y0, [x64, g64], dy.double())
    assert _rel(gx.cpu(), gx0) < 1e-4 and _rel(gg.cpu(), gg0) < 1e-4
