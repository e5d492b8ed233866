"""GPU parity of the HIP multi-scale PatchGAN (torch_utils/ops/patchgan_hip.py, csrc/patchgan.hip)
against the same module evaluated in fp64 on the CPU through the reference formulation
(nn.Conv2d / BatchNormLocal2d / LeakyReLU; reference networks/discriminator.py:75-99, :180-268).

Module level: every intermediate feature of every scale (the feature-matching loss reads them),
the logits, the input gradient and every parameter gradient of a random projection of all outputs.
Features / logits match at 1e-4 of max magnitude (fp32 products through the 3-term bf16 split,
~2^-15.5 per product, fp32 accumulation). Gradients are compared in relative L2 norm at 1e-2: the
fp32 forward flips the odd LeakyReLU decision of the fp64 one (pre-activations within ~1e-6 of 0),
and each flip changes that element's gradient by O(1) of itself; a flip fraction f gives a relative
L2 error ~sqrt(f) (3e-3 measured at f ~ 1e-5). The conv-bias gradients of the layers followed by
BatchNorm are analytically zero (the normalisation removes a per-channel shift), so they are checked
in absolute terms against the layer's weight-gradient norm. The kernels themselves are pinned
without activations in between (test_conv_nhwc_kernel, test_bn_local_lrelu_kernel) at 1e-5 / 2e-5.
Each kernel name is asserted in the timer, so a torch fallback fails.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def _rel2(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("B,res", [(16, 64), (2, 48), (8, 40)])
def test_patchgan_matches_fp64(B, res):
    from networks.discriminator import MultiscaleDiscriminator, weights_init
    from torch_utils.ops import kernel_timer
    torch.manual_seed(B + res)
    D = MultiscaleDiscriminator(input_nc=3, num_D=3, get_interm_feat=True)
    D.apply(weights_init)
    for m in D.modules():                       # non-trivial affine BN parameters
        if hasattr(m, 'virtual_bs') and m.affine:
            m.weight.data.normal_(1.0, 0.2)
            m.bias.data.normal_(0.0, 0.2)
    x = torch.randn(B, 3, res, res)
    Dg = D.cuda()
    xg = x.cuda().requires_grad_()
    kernel_timer.enable(True)
    out = Dg(xg)
    feats = [f for scale in out for f in scale]
    gen = torch.Generator().manual_seed(7)
    R = [torch.randn(f.shape, generator=gen) for f in feats]
    loss = sum((f * r.cuda()).sum() for f, r in zip(feats, R))
    loss.backward()
    torch.cuda.synchronize()
    names = {k.split('<')[0] for k in kernel_timer.summary()}
    kernel_timer.enable(False)
    for n in ("im2col_nhwc", "col2im_nhwc", "rowdot", "coldot", "bnl_lrelu_fwd", "bnl_lrelu_bwd"):
        assert n in names, (n, names)
    assert any(n.startswith("gemm") for n in names), names

    Dc = MultiscaleDiscriminator(input_nc=3, num_D=3, get_interm_feat=True).double()
    Dc.load_state_dict({k: v.detach().cpu().double() for k, v in Dg.state_dict().items()})
    xc = x.double().requires_grad_()
    outc = Dc(xc)
    featc = [f for scale in outc for f in scale]
    lossc = sum((f * r.double()).sum() for f, r in zip(featc, R))
    lossc.backward()
    assert len(feats) == len(featc)
    for f, fc in zip(feats, featc):
        assert f.shape == fc.shape
        assert _rel(f, fc) < 1e-4, (tuple(f.shape), _rel(f, fc))
    assert _rel2(xg.grad, xc.grad) < 1e-2, _rel2(xg.grad, xc.grad)
    pc = dict(Dc.named_parameters())
    for n, p in Dg.named_parameters():
        assert p.grad is not None, n
        if n.endswith(".0.bias") and not n.split(".")[0].endswith(("layer0", "layer4")):
            wn = float(pc[n[:-4] + "weight"].grad.norm())
            assert float((p.grad.cpu().double() - pc[n].grad).norm()) < 1e-4 * wn, n
            continue
        assert _rel2(p.grad, pc[n].grad) < 1e-2, (n, _rel2(p.grad, pc[n].grad))


@pytest.mark.parametrize("B,H,W,C,O,stride", [(4, 33, 33, 64, 128, 2), (3, 10, 9, 256, 512, 1), (2, 7, 6, 512, 1, 1),
                                             (5, 20, 21, 3, 64, 2)])
def test_conv_nhwc_kernel(B, H, W, C, O, stride):
    """k4 / pad 2 conv on NHWC (im2col + MFMA GEMM / rowdot, col2im, split-K weight gradient / coldot)
    vs fp64 torch: y, dx, dw, db."""
    from torch_utils.ops import patchgan_hip
    g = torch.Generator().manual_seed(B * H + O)
    x = torch.randn(B, H, W, C, generator=g)
    w = torch.randn(O, C, 4, 4, generator=g) * (C * 16) ** -0.5
    b = torch.randn(O, generator=g)
    xg, wg, bg = (t.cuda().requires_grad_() for t in (x, w, b))
    y = patchgan_hip.conv_nhwc(xg, wg, bg, stride, 2)
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy.cuda())
    xd, wd, bd = (t.double().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.conv2d(xd.permute(0, 3, 1, 2), wd, bd, stride=stride, padding=2).permute(0, 2, 3, 1)
    yr.backward(dy.double())
    assert y.shape == yr.shape
    assert _rel(y, yr) < 1e-5
    assert _rel(xg.grad, xd.grad) < 1e-5
    assert _rel(wg.grad, wd.grad) < 1e-5
    assert _rel(bg.grad, bd.grad) < 1e-5


def test_bn_local_lrelu_kernel():
    """The fused BatchNormLocal2d + LeakyReLU alone (fp32 NHWC) vs fp64 torch, G = 2 groups."""
    from torch_utils.ops import patchgan_hip
    g = torch.Generator().manual_seed(3)
    x = (3 + 2 * torch.randn(16, 9, 7, 128, generator=g)).requires_grad_()
    w = (1 + 0.3 * torch.randn(128, generator=g)).requires_grad_()
    b = (0.2 * torch.randn(128, generator=g)).requires_grad_()
    dy = torch.randn(16, 9, 7, 128, generator=g)
    xg, wg, bg = (t.detach().cuda().requires_grad_() for t in (x, w, b))
    y = patchgan_hip.bn_local_lrelu(xg, wg, bg, 2, 1e-5, 0.2)
    y.backward(dy.cuda())
    xd, wd, bd = (t.detach().double().requires_grad_() for t in (x, w, b))
    v = xd.view(2, 8, 9, 7, 128)
    var, mean = torch.var_mean(v, dim=[1, 2, 3], keepdim=True, unbiased=False)
    z = ((v - mean) / torch.sqrt(var + 1e-5) * wd + bd).view(16, 9, 7, 128)
    yr = torch.nn.functional.leaky_relu(z, 0.2)
    yr.backward(dy.double())
    assert _rel(y, yr) < 2e-6
    assert _rel(xg.grad, xd.grad) < 2e-5
    assert _rel(wg.grad, wd.grad) < 2e-5
    assert _rel(bg.grad, bd.grad) < 2e-5


@pytest.mark.parametrize("B,C,L,k", [(16, 384, 196, 9), (2, 384, 197, 1), (8, 64, 33, 9)])
def test_head_block_fused_bn_lrelu(B, C, L, k):
    """The projected discriminator's head block (SpectralConv1d -> BatchNormLocal -> LeakyReLU) with
    the fused HIP BatchNormLocal + LeakyReLU (csrc/patchgan.hip bn1d_*) vs the same module's torch
    formulation in fp64: output, input and parameter gradients."""
    from networks.discriminator import make_block
    from torch_utils.ops import kernel_timer
    torch.manual_seed(B + L)
    blk = make_block(C, k)
    blk[1].weight.data.normal_(1.0, 0.2)
    blk[1].bias.data.normal_(0.0, 0.2)
    x = torch.randn(B, C, L)
    r = torch.randn(B, C, L)
    # LeakyReLU's slope switches at 0: an output within rounding of 0 takes either slope, so the upstream
    # gradient is zeroed where the fp64 pre-activation is that close (one flipped element moved the input
    # gradient by 2e-3 relative at B = 16, L = 196 -- a draw, not a kernel error)
    with torch.no_grad():
        pre = torch.nn.Sequential(*list(make_block(C, k).double().eval().children())[:2])
        pre.load_state_dict({kk: v.detach().clone().double() for kk, v in blk[:2].state_dict().items()})
        r = r * (pre(x.double()).abs() > 1e-4).float()
    # eval(): the spectral norm uses its stored power-iteration vectors without updating them (so both
    # copies normalise the same weight); BatchNormLocal always normalises with the batch statistics
    state = {kk: v.detach().clone().double() for kk, v in blk.state_dict().items()}
    bg = blk.cuda().eval()
    xg = x.cuda().requires_grad_()
    kernel_timer.enable(True)
    y = bg(xg)
    (y * r.cuda()).sum().backward()
    torch.cuda.synchronize()
    names = set(kernel_timer.summary())
    kernel_timer.enable(False)
    assert "bnl1d_lrelu_fwd<f32>" in names and "bnl1d_lrelu_bwd<f32>" in names, names
    bc = make_block(C, k).double().eval()
    bc.load_state_dict(state)
    xc = x.double().requires_grad_()
    yc = torch.nn.Sequential.forward(bc, xc)
    (yc * r.double()).sum().backward()
    assert _rel(y, yc) < 1e-5, _rel(y, yc)
    assert _rel2(xg.grad, xc.grad) < 1e-3, _rel2(xg.grad, xc.grad)
    pw = dict(bc.named_parameters())
    for (n, p), (_, q) in zip(bg.named_parameters(), bc.named_parameters()):
        if p.grad is None:
            continue
        if n == "0.bias":       # conv bias under BatchNorm: analytically zero gradient, compare absolutely
            wn = float(pw["0.weight_orig"].grad.norm()) if "0.weight_orig" in pw else float(q.grad.abs().max() + 1)
            assert float((p.grad.cpu().double() - q.grad).norm()) < 1e-4 * wn, n
            continue
        assert _rel2(p.grad, q.grad) < 1e-3, (n, _rel2(p.grad, q.grad))
