"""LPIPS VGG16 stack on the HIP implicit-GEMM conv (csrc/conv.hip, torch_utils/ops/vgg_hip.py)
against fp64 torch convolutions of the same weights: single conv3x3 layers (image layer with
3 -> 4 padded channels, ragged spatial sizes, the fused ReLU-derivative mask) and the whole
relu1_2..relu5_3 tap stack forward + input gradient (reference training/lpips.py:126-163).

Tolerance (the default fp32-equivalent f32x6 products): 3e-6 of max |ref| per conv layer and
within 2x (+1e-7) of the exact-fp32 torch convolution's own error, 3e-5 on the 13-layer taps,
1e-4 on the input gradient against the fp64 chain through the same ReLU / pool decisions."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max())


@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 16, 16, 3, 64), (2, 12, 20, 64, 64), (1, 7, 9, 128, 256),
                                            (3, 8, 8, 512, 512), (2, 33, 5, 256, 128)])
def test_conv3x3_layer(B, H, W, Cin, Cout):
    from torch_utils.ops import vgg_hip
    g = torch.Generator(device=DEV).manual_seed(H * W + Cin)
    x = torch.randn(B, Cin, H, W, generator=g, device=DEV)
    conv = torch.nn.Conv2d(Cin, Cout, 3, padding=1).to(DEV)
    wf, wb, b, w = vgg_hip.prepare([conv])[0]
    cp = max(Cin, 4)
    xh = torch.zeros(B, H, W, cp, device=DEV)
    xh[..., :Cin] = x.permute(0, 2, 3, 1)
    ref = F.conv2d(x.double(), w.double(), b.double(), padding=1).relu()
    y = vgg_hip.conv3x3(xh, wf, b, relu=True)
    e_ours = _rel(y.permute(0, 3, 1, 2), ref)
    with torch.backends.cudnn.flags(enabled=False):      # torch's direct fp32 conv (exact products)
        yt = F.conv2d(x, w, b, padding=1).relu()
    assert e_ours < 3e-6, e_ours
    assert e_ours <= 2 * _rel(yt, ref) + 1e-7, (e_ours, _rel(yt, ref))
    if Cin >= 64:
        # data gradient with the layer-below mask, as the backward runs it
        dz = torch.randn(B, H, W, Cout, generator=g, device=DEV)
        mask = torch.randn(B, H, W, Cin, generator=g, device=DEV)
        gx = vgg_hip.conv3x3(dz, wb, None, relu=False, mask=mask)
        ref = torch.nn.grad.conv2d_input((B, Cin, H, W), w.double(), dz.permute(0, 3, 1, 2).double(), padding=1)
        ref = ref * (mask.permute(0, 3, 1, 2) > 0)
        assert _rel(gx.permute(0, 3, 1, 2), ref) < 3e-6


def _conv64(x, w, bias=None, relu=False, mask=None):
    """fp64 torch stand-in for vgg_hip.conv3x3 (same NHWC conventions; w = the bf16 pieces in the kernel's
    k order, whose sum is the fp32 weight exactly)."""
    from torch_utils.ops import vgg_hip
    B, H, W, Cin = x.shape
    w = vgg_hip.tap_major(w.double().sum(0)[:, :9 * Cin], Cin)
    y = F.conv2d(x.permute(0, 3, 1, 2).double(), w.reshape(w.shape[0], 3, 3, Cin).permute(0, 3, 1, 2),
                 None if bias is None else bias.double(), padding=1)
    y = (y.relu() if relu else y).permute(0, 2, 3, 1)
    return (y * (mask > 0) if mask is not None else y).contiguous()


@pytest.mark.parametrize("res", [64, 48])
def test_vgg16_taps_forward_backward(res):
    """Taps vs an independent fp64 stack; the input gradient vs the fp64 backward chain taken
    through the same ReLU masks and pool choices (a 2^-16 forward difference flips the odd ReLU
    or max-pool decision of an fp64 stack, which moves single gradient entries by O(1) of their
    size -- that comparison is made in relative L2 norm instead)."""
    from training.lpips import vgg16
    from torch_utils.ops import vgg_hip
    net = vgg16(pretrained=False).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(res)
    x = torch.randn(2, 3, res, res, generator=g, device=DEV).requires_grad_(True)
    outs = net(x)
    gs = [torch.randn(o.shape, generator=g, device=DEV) for o in outs]
    torch.autograd.backward(list(outs), gs)
    ref_net = vgg16(pretrained=False).to(DEV).double()
    ref_net.load_state_dict(net.state_dict())
    xr = x.detach().double().requires_grad_(True)
    h, refs = xr, []
    for k in range(1, 6):
        h = getattr(ref_net, f"slice{k}")(h)
        refs.append(h)
    torch.autograd.backward(refs, [t.double() for t in gs])
    for o, r in zip(outs, refs):
        assert o.shape == r.shape
        assert _rel(o, r) < 3e-5
    convs = [m for k in range(1, 6) for m in getattr(net, f"slice{k}") if isinstance(m, torch.nn.Conv2d)]
    prep = vgg_hip.prepare(convs)
    _, ys, pools = vgg_hip.forward_chain(x.detach(), prep)
    gx = vgg_hip.backward_chain([y.double() for y in ys], pools, prep, x.shape, [t.double() for t in gs],
                                conv=_conv64)
    assert _rel(x.grad, gx) < 1e-4
    l2 = float((x.grad.double() - xr.grad).norm() / xr.grad.norm())
    assert l2 < 2e-2, l2


@pytest.mark.parametrize("B,H,W", [(2, 37, 70), (1, 64, 64), (3, 5, 130)])
def test_image_layer_input_gradient(B, H, W):
    """The VGG16 image layer's input gradient (3 <- 64 channels) on the VALU kernel
    vfm_conv3x3_dgrad_small_f32 vs the fp64 torch conv2d_input: fp32 FMAs over 576 terms, 2e-6 of
    max |ref|, and within 2x of the exact-fp32 torch conv's own error (+1e-7)."""
    from torch_utils.ops import vgg_hip
    g = torch.Generator(device=DEV).manual_seed(B * H + W)
    w = torch.randn(64, 3, 3, 3, generator=g, device=DEV) * 0.1
    dz = torch.randn(B, H, W, 64, generator=g, device=DEV)
    out = vgg_hip.image_grad(dz, w, (B, 3, H, W))
    ref = torch.nn.grad.conv2d_input((B, 3, H, W), w.double(), dz.permute(0, 3, 1, 2).double(), padding=1)
    with torch.backends.cudnn.flags(enabled=False):
        t32 = torch.nn.grad.conv2d_input((B, 3, H, W), w, dz.permute(0, 3, 1, 2).contiguous(), padding=1)
    e = _rel(out, ref)
    assert e < 2e-6, e
    assert e <= 2 * _rel(t32, ref) + 1e-7, (e, _rel(t32, ref))


@pytest.mark.parametrize("B,H,W,C", [(2, 16, 16, 64), (3, 8, 12, 128), (1, 2, 2, 4)])
@pytest.mark.parametrize("with_tap", [True, False])
def test_maxpool2x2_fused_bit_exact(B, H, W, C, with_tap):
    """csrc/pool.hip against torch: the forward (no indices) equals F.max_pool2d, and the fused backward
    (pool backward + tap gradient + ReLU derivative, argmax recomputed from the input) equals torch's
    max_pool2d_with_indices_backward -> add -> * (x > 0) chain bit for bit, ties (ReLU zeros, repeated
    values) included."""
    from torch_utils.ops import vgg_hip
    g0 = torch.Generator().manual_seed(B * H + W * C)
    x = torch.randn(B, H, W, C, generator=g0).relu()                     # ~half zeros: all-zero windows
    x[:, ::2, ::2, : C // 2] = x[:, 1::2, 1::2, : C // 2]                # exact ties inside windows
    x = x.to(DEV)
    out = vgg_hip.maxpool2x2(x)
    ref, idx = F.max_pool2d(x.permute(0, 3, 1, 2), 2, 2, return_indices=True)
    assert torch.equal(out, ref.permute(0, 2, 3, 1))
    g = torch.randn(B, H // 2, W // 2, C, generator=g0).to(DEV)
    gt = torch.randn(B, H, W, C, generator=g0).to(DEV) if with_tap else None
    got = vgg_hip.maxpool2x2_bwd(g, x, gt)
    r = torch.ops.aten.max_pool2d_with_indices_backward(g.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2), [2, 2], [2, 2],
                                                        [0, 0], [1, 1], False, idx).permute(0, 2, 3, 1)
    if gt is not None:
        r = r + gt
    r = r * (x > 0)
    assert torch.equal(got, r)


@pytest.mark.parametrize("res", [64, 48])
def test_vgg16_taps_pair_matches_two_passes(res):
    """LPIPS's input and target through one VGG16 pass of 2B images (vgg_hip.vgg16_taps_pair): taps bit-
    identical to two single-batch passes (every layer is per-sample), the input gradient identical to the
    single-batch backward, and no gradient work for the target (no grad requested)."""
    from training.lpips import vgg16
    from torch_utils.ops import vgg_hip
    net = vgg16(pretrained=False).to(DEV)
    convs = [m for k in range(1, 6) for m in getattr(net, f"slice{k}") if isinstance(m, torch.nn.Conv2d)]
    g = torch.Generator(device=DEV).manual_seed(res + 1)
    x0 = torch.randn(3, 3, res, res, generator=g, device=DEV).requires_grad_(True)
    x1 = torch.randn(3, 3, res, res, generator=g, device=DEV)
    t0, t1 = vgg_hip.vgg16_taps_pair(x0, x1, convs)
    r0 = vgg_hip.vgg16_taps(x0.detach().requires_grad_(True), convs)
    r1 = vgg_hip.vgg16_taps(x1, convs)
    for a, b in zip(list(t0) + list(t1), list(r0) + list(r1)):
        assert torch.equal(a, b)
    gs = [torch.randn(o.shape, generator=g, device=DEV) for o in t0]
    gx, = torch.autograd.grad(list(t0), [x0], gs)
    xr = x0.detach().requires_grad_(True)
    gr, = torch.autograd.grad(list(vgg_hip.vgg16_taps(xr, convs)), [xr], gs)
    assert torch.equal(gx, gr)
