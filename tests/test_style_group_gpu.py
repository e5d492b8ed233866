"""Grouped style path (torch_utils/ops/style_group.py, csrc/style.hip vfm_style_group_*) against the per-layer
path (csrc/style.hip single-layer calls) and the torch formulation (reference networks/utils/shared.py StyleSplit /
FullyConnectedLayer, networks/utils/convnext_utils.py:60-66 demodulation): styles, demodulation coefficients and
the gradients of ws, the affine weights / biases and the demodulated weights. Same per-layer arithmetic as the
single-layer calls, so against them the outputs and gradients are bit-identical; against fp64 torch within 1e-5
of max |ref|. The whole generator's grouped path is pinned against the reference's vectors by
tests/test_networks_gpu.py::test_generator_forward_backward_gpu (its checked forward runs grouped)."""
import pytest
import torch

from networks.utils.shared import StyleSplit
from torch_utils.ops import decoder_ops, style_group

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
B, NW, WD = 5, 7, 48
LAYERS = [(64, 256, 0), (32, 128, 2), (16, 64, 3), (64, None, 5), (24, 96, 6)]     # C, O (None: ToRGB), ws column


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.aff = torch.nn.ModuleList([StyleSplit(WD, C, bias_init=1) for C, _, _ in LAYERS])
        self.w1 = torch.nn.ParameterList([torch.nn.Parameter(torch.randn(O, C, 1, 1) * 0.1) if O else
                                          torch.nn.Parameter(torch.zeros(1)) for C, O, _ in LAYERS])

    def styles(self, ws):
        outs = []
        for (C, O, j), aff, w1 in zip(LAYERS, self.aff, self.w1):
            w = ws[:, j]
            if O:
                outs += list(decoder_ops.style_and_demod(aff, w, w1.reshape(O, C)))
            else:
                outs.append(decoder_ops.style_and_demod(aff, w, None)[0])
        return outs


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / (b.double().abs().max() + 1e-30))


def _run(net, ws, group, dys):
    ws = ws.detach().clone().requires_grad_(True)
    for p in net.parameters():
        p.grad = None
    ctx = style_group.StyleGroup(net, ws) if group else None
    if ctx is not None:
        ctx.__enter__()
    try:
        outs = net.styles(ws)
    finally:
        if ctx is not None:
            ctx.__exit__(None, None, None)
    sum((o * dy).sum() for o, dy in zip(outs, dys)).backward()
    grads = [ws.grad] + [p.grad for p in net.parameters()]
    return [o.detach() for o in outs], grads, ctx


def test_style_group_matches_per_layer_and_torch():
    net = _Net().to(DEV)
    g = torch.Generator().manual_seed(3)
    ws = torch.randn(B, NW, WD, generator=g).to(DEV)
    with torch.no_grad():
        shapes = [o.shape for o in net.styles(ws)]
    dys = [torch.randn(s, generator=g).to(DEV) for s in shapes]
    ref_out, ref_grads, _ = _run(net, ws, False, dys)                  # per-layer path
    rec_out, rec_grads, ctx = _run(net, ws, True, dys)                 # first forward: records the plan
    assert ctx.record is not None and len(ctx.record) == len(LAYERS)
    grp_out, grp_grads, ctx = _run(net, ws, True, dys)                 # grouped launches
    assert ctx.record is None and not ctx.results, "every layer took its grouped outputs"
    # the same kernels' per-layer arithmetic: bit-identical outputs and gradients
    for a, b in zip(grp_out, ref_out):
        assert torch.equal(a, b)
    names = ["ws"] + [n for n, _ in net.named_parameters()]
    bad = [(n, _rel(a, b)) for n, a, b in zip(names, grp_grads, ref_grads)
           if not ((a is None and b is None) or torch.equal(a, b))]
    if bad:
        cols = [(j, _rel(grp_grads[0][:, j], ref_grads[0][:, j])) for j in range(NW)]
        print("differing gradients:", bad, "ws columns:", cols, flush=True)
    assert not bad, bad
    # the torch formulation in fp64
    ws64 = ws.double().requires_grad_(True)
    outs = []
    for (C, O, j), aff in zip(LAYERS, net.aff):
        fc = aff.proj
        m = ws64[:, j] @ (fc.weight.double() * fc.weight_gain).t() + fc.bias.double() * fc.bias_gain
        m1, m2, m3 = m.chunk(3, dim=1)
        s = m1 * m2 + m3
        outs.append(s)
    k = 0
    for (C, O, j), s64, w1 in zip(LAYERS, outs, net.w1):
        assert float((grp_out[k].double() - s64).abs().max() / s64.abs().max()) < 1e-5
        if O:
            d64 = torch.rsqrt((s64[:, None, :] * w1.double().reshape(O, C)[None]).square().sum(2) + 1e-8)
            assert float((grp_out[k + 1].double() - d64).abs().max() / d64.abs().max()) < 1e-5
            k += 2
        else:
            k += 1


def test_style_group_falls_back_on_foreign_w():
    """A layer whose w is not the recorded ws column takes the per-layer path."""
    net = _Net().to(DEV)
    ws = torch.randn(B, NW, WD, device=DEV)
    for _ in range(2):
        with style_group.StyleGroup(net, ws):
            net.styles(ws)
    with style_group.StyleGroup(net, ws) as ctx:
        C, O, j = LAYERS[0]
        other = torch.randn(B, WD, device=DEV)
        s, d = decoder_ops.style_and_demod(net.aff[0], other, net.w1[0].reshape(O, C))
        s_ref, d_ref = decoder_ops.style_and_demod(net.aff[0], other, net.w1[0].reshape(O, C))
    assert torch.equal(s, s_ref) and torch.equal(d, d_ref)
