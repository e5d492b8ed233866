"""GPU parity of the gfx950 decoder kernels (csrc/decoder.hip) against the plain
PyTorch fp32 formulation of the same ops (decoder_ops.*(impl='ref')), forward
and backward, on the shapes the decoder runs plus ragged edge cases.

The native path is asserted to have run (kernel_timer records each native
launch by name), so a silent torch fallback fails the test.

Tolerances: fp32 I/O 2e-5 of the reference's max magnitude (different summation
order); bf16/fp16 I/O 1.5e-2 (one output rounding of 2^-8 plus bf16-rounded
intermediates between the ops).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ops():
    from torch_utils.ops import decoder_ops, kernel_timer
    return decoder_ops, kernel_timer


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def _tol(dt):
    return 2e-5 if dt == torch.float32 else 1.5e-2


def _run(fn_hip, fn_ref, inputs, dt, names, out_grad_seed=0):
    """inputs: list of fp32 CPU tensors (None allowed); the first `len(dt_mask)` get dtype dt."""
    _, kt = _ops()
    hip_in = [None if t is None else t.detach().to(DEV).requires_grad_(t.requires_grad) for t in inputs]
    kt.enable(True)
    out = fn_hip(*hip_in)
    torch.manual_seed(out_grad_seed)
    g = torch.randn(out.shape, device=DEV)
    out.backward(g.to(out.dtype))
    torch.cuda.synchronize()
    recorded = set(kt.summary())
    kt.enable(False)
    # region names carry <dtype,taps>; the banded-MFMA dwconv (bf16) counts as the dwconv op
    base = {r.split('<')[0].replace('dwconv2d_mfma', 'dwconv2d') for r in recorded}
    for n in names:
        assert n in base, (n, recorded)
    ref_in = [None if t is None else t.detach().to(DEV).double().float().requires_grad_(t.requires_grad)
              for t in hip_in]
    ref = fn_ref(*ref_in)
    ref.backward(g.float())
    tol = _tol(dt)
    assert _rel(out.float(), ref) < tol
    for a, b in zip(hip_in, ref_in):
        if a is not None and a.requires_grad:
            assert a.grad is not None
            assert _rel(a.grad.float(), b.grad) < 4 * tol, (a.shape, _rel(a.grad.float(), b.grad))


# Row-streaming kernel: same-size odd K, W in {16..256} a power-of-two multiple of 4;
# LDS-tile kernel: everything else (ragged widths, narrow planes).
DW_CASES = [(2, 8, 16, 16, 3), (2, 8, 16, 16, 5), (2, 6, 16, 16, 7), (1, 4, 64, 70, 3), (2, 5, 13, 9, 3),
            (1, 3, 33, 130, 7), (3, 2, 4, 4, 3), (1, 2, 1, 5, 3), (2, 3, 37, 128, 7), (1, 2, 20, 256, 5),
            (2, 4, 9, 32, 3), (1, 3, 300, 64, 7), (2, 2, 256, 256, 7),
            # several samples per wave (narrow planes), multi-band units, partial last wave
            (20, 3, 16, 16, 5), (33, 2, 32, 64, 7), (9, 3, 64, 64, 7), (5, 2, 8, 16, 3)]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("case", DW_CASES)
def test_dwconv2d(case, dt):
    ops, _ = _ops()
    B, C, H, W, K = case
    torch.manual_seed(1)
    x = torch.randn(B, C, H, W).to(dt).float().requires_grad_(True)
    w = (torch.randn(C, 1, K, K) * 0.2).requires_grad_(True)
    b = (torch.randn(C) * 0.1).requires_grad_(True)
    noise = torch.randn(H, W).requires_grad_(True)
    hip = lambda x, w, b, n: ops.dwconv2d(x.to(dt), w, b, K // 2, noise=n)
    ref = lambda x, w, b, n: ops.dwconv2d(x, w, b, K // 2, noise=n, impl='ref')
    _run(hip, ref, [x, w, b, noise], dt, ["dwconv2d_fwd", "dwconv2d_bwd_data", "dwconv2d_bwd_weight"])


@pytest.mark.parametrize("case", [(2, 8, 16, 16, 3), (2, 6, 16, 16, 5), (2, 5, 20, 64, 7), (1, 3, 64, 256, 7),
                                  (3, 4, 37, 48, 7), (2, 3, 8, 128, 5), (1, 2, 5, 32, 3)])
def test_dwconv2d_mfma(case):
    """The banded-MFMA depthwise kernel (csrc/dwconv_mfma.hip): bf16 planes, no noise, forward and
    data gradient (both on MFMA; the weight gradient stays on the row kernel) vs the fp32 torch
    formulation with the taps rounded to bf16, as the reference's autocast conv uses them."""
    ops, kt = _ops()
    B, C, H, W, K = case
    torch.manual_seed(2)
    x = torch.randn(B, C, H, W).to(torch.bfloat16).float().requires_grad_(True)
    w = (torch.randn(C, 1, K, K) * 0.2).to(torch.bfloat16).float().requires_grad_(True)
    b = (torch.randn(C) * 0.1).requires_grad_(True)
    hip = lambda x, w, b: ops.dwconv2d(x.to(torch.bfloat16), w, b, K // 2)
    ref = lambda x, w, b: ops.dwconv2d(x, w, b, K // 2, impl='ref')
    _run(hip, ref, [x, w, b], torch.bfloat16, ["dwconv2d_fwd", "dwconv2d_bwd_data", "dwconv2d_bwd_weight"])
    kt.enable(True)
    ops.dwconv2d(x.detach().to(DEV, torch.bfloat16), w.detach().to(DEV), b.detach().to(DEV), K // 2)
    torch.cuda.synchronize()
    assert any(n.startswith("dwconv2d_mfma_fwd") for n in kt.summary()), kt.summary()
    kt.enable(False)
    # the weight gradient on MFMA as well (bf16 x / dy)
    kt.enable(True)
    xg = x.detach().to(DEV, torch.bfloat16).requires_grad_(False)
    wg = w.detach().to(DEV).requires_grad_(True)
    bg = b.detach().to(DEV).requires_grad_(True)
    dyg = torch.randn(B, C, H, W).to(DEV, torch.bfloat16)
    ops.dwconv2d(xg, wg, bg, K // 2).backward(dyg)
    torch.cuda.synchronize()
    assert any(n.startswith("dwconv2d_mfma_bwd_weight") for n in kt.summary()), kt.summary()
    kt.enable(False)
    xr = x.detach().double().requires_grad_(False)
    wr = w.detach().double().requires_grad_(True)
    br = b.detach().double().requires_grad_(True)
    torch.nn.functional.conv2d(xr, wr, br, padding=K // 2, groups=C).backward(dyg.double().cpu())
    assert _rel(wg.grad, wr.grad) < 1e-5, _rel(wg.grad, wr.grad)
    assert _rel(bg.grad, br.grad) < 1e-5


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", [(2, 8, 16, 16, 3), (3, 4, 64, 64, 7), (2, 5, 37, 48, 7), (4, 6, 32, 128, 5),
                                  (1, 3, 5, 16, 3)])
def test_dwconv2d_noise_strength(case, dt):
    """The legacy noise as plane * strength (reference convnext_utils.py: noise_const * noise_strength
    added after the dwconv): the strength's gradient sum dY * plane comes from the data-gradient
    kernel's per-wave partials on bf16 planes (vfm_dwconv2d_fwd_mfma_nz) and from a torch dot
    otherwise; against an fp64 dot of the same dY within 1e-5 (fp32 partial sums), the forward and the
    other gradients as the torch formulation (decoder tolerances), and the plane's own gradient
    strength * sum_{b,c} dY when it is asked for."""
    ops, kt = _ops()
    B, C, H, W, K = case
    torch.manual_seed(3)
    x = torch.randn(B, C, H, W, device=DEV).to(dt)
    w = (torch.randn(C, 1, K, K, device=DEV) * 0.2)
    b = (torch.randn(C, device=DEV) * 0.1)
    plane = torch.randn(H, W, device=DEV)
    strength = torch.tensor(0.37, device=DEV)
    dy = torch.randn(B, C, H, W, device=DEV).to(dt)
    leaves = [t.clone().requires_grad_(True) for t in (x, w, b, strength)]
    kt.enable(True)
    y = ops.dwconv2d(leaves[0], leaves[1], leaves[2], K // 2, noise=plane, noise_strength=leaves[3])
    y.backward(dy)
    torch.cuda.synchronize()
    names = set(kt.summary())
    kt.enable(False)
    if dt == torch.bfloat16 and W % 16 == 0:
        assert any(n.startswith("dwconv2d_mfma_bwd_data") for n in names), names
    ref_leaves = [t.detach().float().clone().requires_grad_(True) for t in (x, w, b, strength)]
    yr = ops.dwconv2d(ref_leaves[0], ref_leaves[1], ref_leaves[2], K // 2, noise=plane,
                      noise_strength=ref_leaves[3], impl='ref')
    yr.backward(dy.float())
    tol = _tol(dt)
    assert _rel(y.float(), yr) < tol
    for a, r in zip(leaves[:3], ref_leaves[:3]):
        assert _rel(a.grad.float(), r.grad) < 4 * tol
    exact = (dy.double() * plane.double()).sum()
    assert abs(float(leaves[3].grad) - float(exact)) <= 1e-5 * float((dy.double().abs() * plane.double().abs()).sum())
    # the plane itself with a gradient (not the model's use): d plane = strength * sum_{b,c} dY
    pl = plane.clone().requires_grad_(True)
    ops.dwconv2d(x, w, b, K // 2, noise=pl, noise_strength=strength).backward(dy)
    assert _rel(pl.grad, 0.37 * dy.float().sum((0, 1))) < 1e-5


def test_dwconv2d_no_bias_valid_padding():
    ops, _ = _ops()
    torch.manual_seed(2)
    x = torch.randn(2, 4, 12, 20).requires_grad_(True)
    w = torch.randn(4, 1, 3, 3).requires_grad_(True)
    _run(lambda x, w: ops.dwconv2d(x, w, None, 0), lambda x, w: ops.dwconv2d(x, w, None, 0, impl='ref'),
         [x, w], torch.float32, ["dwconv2d_fwd"])


GN_CASES = [(2, 64, 16, 16, 16), (2, 12, 5, 7, 3), (3, 32, 8, 8, 32), (1, 256, 32, 32, 32), (2, 8, 1, 1, 2),
            # flat forms: 2-lane channel segments, channels spanning many chunk rounds; channel-loop
            # fallbacks: HW / 8 not a power of two, more than 128 channels per group
            (2, 8, 4, 4, 1), (2, 64, 128, 128, 32), (1, 16, 24, 24, 4), (1, 512, 16, 16, 2)]


@pytest.mark.parametrize("dt_in,dt_out", [(torch.float32, torch.float32), (torch.float32, torch.bfloat16),
                                          (torch.bfloat16, torch.bfloat16), (torch.float16, torch.float16)])
@pytest.mark.parametrize("case", GN_CASES)
@pytest.mark.parametrize("with_style", [False, True])
def test_group_norm(case, dt_in, dt_out, with_style):
    ops, _ = _ops()
    B, C, H, W, G = case
    torch.manual_seed(3)
    x = (torch.randn(B, C, H, W) * 3 + 1.5).to(dt_in).float().requires_grad_(True)
    w = (1 + 0.1 * torch.randn(C)).requires_grad_(True)
    b = (0.1 * torch.randn(C)).requires_grad_(True)
    s = (1 + 0.3 * torch.randn(B, C)).requires_grad_(True) if with_style else None
    hip = lambda x, w, b, s: ops.group_norm(x.to(dt_in), G, w, b, 1e-5, out_dtype=dt_out, style=s)
    ref = lambda x, w, b, s: ops.group_norm(x, G, w, b, 1e-5, out_dtype=torch.float32, style=s, impl='ref')
    worst = dt_out if dt_out != torch.float32 else dt_in
    _run(hip, ref, [x, w, b, s], worst, ["group_norm_fwd", "group_norm_bwd"])


def test_group_norm_large_mean_is_stable():
    """Shifted sums: a group with |mean| >> std still normalises accurately."""
    ops, _ = _ops()
    torch.manual_seed(4)
    x = torch.randn(2, 16, 16, 16) * 0.01 + 300.0
    y = ops.group_norm(x.to(DEV), 4, None, None, 1e-5)
    r = ops.group_norm(x.double(), 4, None, None, 1e-5, impl='ref')
    assert _rel(y.cpu(), r) < 5e-3


# (B, C, H, W, K, G): both MFMA tile widths, partial row bands, one-band planes, many units per group
GS_CASES = [(2, 64, 16, 16, 7, 32), (2, 32, 37, 48, 7, 8), (3, 16, 64, 64, 5, 4), (1, 128, 128, 128, 7, 32),
            (4, 8, 8, 16, 3, 2), (2, 256, 32, 32, 7, 32), (1, 12, 100, 64, 3, 3),
            # more than GN_FLAT_MAX channels per group: the one-block-per-group form of the stats mode
            (1, 256, 16, 16, 3, 1)]


@pytest.mark.parametrize("case", GS_CASES)
@pytest.mark.parametrize("offset", [0.0, 40.0])
def test_group_norm_stats_from_dwconv(case, offset):
    """GroupNorm statistics from the dwconv's per-wave partials (vfm_dwconv2d_fwd_mfma_gs ->
    vfm_group_norm_fwd_stats, the ConvNeXt block's dwconv -> norm): an fp32-output GroupNorm of the
    bf16 conv output against an fp64 GroupNorm of the same bf16 values within 2e-5 (also with a large
    common offset: the shifted partial sums), the bf16-output form and both gradients against the
    unfused path, and the fused kernels asserted to have run."""
    from torch_utils.ops import decoder_hip
    ops, kt = _ops()
    B, C, H, W, K, G = case
    torch.manual_seed(5)
    x = torch.randn(B, C, H, W, device=DEV).to(torch.bfloat16)
    w = torch.randn(C, 1, K, K, device=DEV) * 0.2
    b = torch.randn(C, device=DEV) * 0.1 + offset
    plane = torch.randn(H, W, device=DEV)
    gw = 1 + 0.1 * torch.randn(C, device=DEV)
    gb = 0.1 * torch.randn(C, device=DEV)
    st = 1 + 0.3 * torch.randn(B, C, device=DEV)
    kt.enable(True)
    d = ops.dwconv2d(x, w, b, K // 2, noise=plane)
    y32 = ops.group_norm(d, G, gw, gb, 1e-5, out_dtype=torch.float32, style=st)
    torch.cuda.synchronize()
    names = set(kt.summary())
    kt.enable(False)
    assert any(n.startswith("dwconv2d_mfma_fwd") for n in names), names
    assert any(n.startswith("group_norm_fwd_stats") for n in names), names
    ref = torch.nn.functional.group_norm(d.double(), G, gw.double(), gb.double(), 1e-5) * st.double()[:, :, None, None]
    assert _rel(y32, ref) < 2e-5, _rel(y32, ref)

    def fwd_bwd(fused):
        decoder_hip.GN_STATS = fused
        try:
            leaves = [t.clone().requires_grad_(True) for t in (x, w, b, gw, gb, st)]
            kt.enable(True)
            out = ops.group_norm(ops.dwconv2d(leaves[0], leaves[1], leaves[2], K // 2, noise=plane), G, leaves[3],
                                 leaves[4], 1e-5, out_dtype=torch.bfloat16, style=leaves[5])
            torch.manual_seed(6)
            out.backward(torch.randn(out.shape, device=DEV).to(out.dtype))
            torch.cuda.synchronize()
            used = any(n.startswith("group_norm_fwd_stats") for n in kt.summary())
            kt.enable(False)
            assert used == fused
            return out, [t.grad for t in leaves]
        finally:
            decoder_hip.GN_STATS = True

    yf, gf = fwd_bwd(True)
    yu, gu = fwd_bwd(False)
    assert _rel(yf.float(), yu.float()) < 1.5e-2
    for a, r in zip(gf, gu):
        assert _rel(a.float(), r.float()) < 3e-2, _rel(a.float(), r.float())


def test_group_norm_stats_need_the_unchanged_output():
    """The partials are used only by a GroupNorm of the dwconv's own, unmodified output."""
    from torch_utils.ops import decoder_hip
    ops, kt = _ops()
    torch.manual_seed(7)
    x = torch.randn(2, 32, 32, 64, device=DEV).to(torch.bfloat16)
    w = torch.randn(32, 1, 7, 7, device=DEV) * 0.2
    kt.enable(True)
    d = ops.dwconv2d(x, w, None, 3)
    d.mul_(2.0)                                    # in-place change after the conv: version differs
    y = ops.group_norm(d, 8, None, None, 1e-5, out_dtype=torch.float32)
    d2 = ops.dwconv2d(x, w, None, 3)
    other = d2.clone()                             # a different tensor of the same shape
    y2 = ops.group_norm(other, 8, None, None, 1e-5, out_dtype=torch.float32)
    torch.cuda.synchronize()
    names = set(kt.summary())
    kt.enable(False)
    assert not any(n.startswith("group_norm_fwd_stats") for n in names), names
    for inp, out in ((d, y), (other, y2)):
        ref = torch.nn.functional.group_norm(inp.double(), 8, None, None, 1e-5)
        assert _rel(out, ref) < 2e-5
    e = getattr(decoder_hip._gn_tls, "e", None)     # per-thread handoff slot: d2's partials or cleared
    assert e is None or (e[0]() is d2 and e[1] == d2.device)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(2, 32, 64), (4, 256, 256), (1, 8, 8), (3, 40, 1000)])
@pytest.mark.parametrize("with_scale", [True, False])
def test_scale_bias_gelu(shape, dt, with_scale):
    ops, _ = _ops()
    B, O, P = shape
    torch.manual_seed(5)
    h = (torch.randn(B, O, P) * 2).to(dt).float().requires_grad_(True)
    s = (torch.rand(B, O) + 0.5).requires_grad_(True) if with_scale else None
    b = (torch.randn(O) * 0.3).requires_grad_(True)
    hip = lambda h, s, b: ops.scale_bias_gelu(h.to(dt), s, b)
    ref = lambda h, s, b: ops.scale_bias_gelu(h, s, b, impl='ref')
    _run(hip, ref, [h, s, b], dt, ["scale_bias_gelu_fwd", "scale_bias_gelu_bwd"])


@pytest.mark.parametrize("dt_y,dt_x", [(torch.float32, torch.float32), (torch.bfloat16, torch.float32),
                                       (torch.bfloat16, torch.bfloat16), (torch.float16, torch.float16)])
@pytest.mark.parametrize("shape", [(2, 16, 64), (4, 128, 256), (1, 3, 8)])
def test_layer_scale_residual(shape, dt_y, dt_x):
    ops, _ = _ops()
    B, C, P = shape
    torch.manual_seed(6)
    y = torch.randn(B, C, P).to(dt_y).float().requires_grad_(True)
    b = (0.1 * torch.randn(C)).requires_grad_(True)
    g = (0.5 + 0.2 * torch.randn(C)).requires_grad_(True)
    x = torch.randn(B, C, P).to(dt_x).float().requires_grad_(True)
    hip = lambda y, b, g, x: ops.layer_scale_residual(y.to(dt_y), b, g, x.to(dt_x))
    ref = lambda y, b, g, x: ops.layer_scale_residual(y, b, g, x, impl='ref')
    worst = dt_y if dt_y != torch.float32 else dt_x
    _run(hip, ref, [y, b, g, x], worst, ["layer_scale_residual_fwd", "layer_scale_residual_bwd"])


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("taps", [[1, 1], [1, 2, 1], [1, 3, 3, 1], [1, 4, 6, 4, 1], [1, 7, 21, 35, 35, 21, 7, 1]])
@pytest.mark.parametrize("shape,r", [((2, 16, 8, 8), 2), ((1, 12, 5, 7), 2), ((2, 4, 9, 6), 1), ((1, 4, 1, 1), 2),
                                     ((1, 2, 16, 32), 1), ((1, 8, 40, 70), 2), ((1, 3, 70, 130), 1),
                                     # 16-B vector forms (W % 8 == 0) with partial edge tiles
                                     ((2, 8, 40, 48), 2), ((1, 3, 72, 136), 1), ((1, 4, 3, 8), 2),
                                     # forward strips of BSTRIP tiles: several strips, a partial last one
                                     ((1, 4, 136, 16), 2), ((1, 2, 300, 64), 1), ((2, 12, 64, 64), 2)])
def test_shuffle_blur(shape, r, taps, dt):
    ops, _ = _ops()
    torch.manual_seed(7)
    x = torch.randn(*shape).to(dt).float().requires_grad_(True)
    if r == 1:
        hip = lambda x: ops.blur_replicate(x.to(dt), taps)
        ref = lambda x: ops.blur_replicate(x, taps, impl='ref')
    else:
        hip = lambda x: ops.shuffle_blur(x.to(dt), taps, r)
        ref = lambda x: ops.shuffle_blur(x, taps, r, impl='ref')
    _run(hip, ref, [x], dt, ["shuffle_blur_fwd", "shuffle_blur_bwd"])


def test_convnext_layer_hip_matches_torch_formulation():
    """One ConvNeXt synthesis layer end to end (fwd + grads of every parameter),
    HIP decoder ops vs the torch formulation, fp32."""
    from networks.utils.convnext_utils import ConvNeXtSynthesisLayer
    ops, _ = _ops()
    torch.manual_seed(8)
    layer = ConvNeXtSynthesisLayer(64, 32, 7, layer_scale_init=0.5).to(DEV)
    x = torch.randn(2, 64, 16, 16, device=DEV)
    w = torch.randn(2, 32, device=DEV)
    outs, grads = [], []
    for force in (False, True):
        ops.set_force_ref(force)
        try:
            layer.zero_grad(set_to_none=True)
            y = layer(x, w)
            (y * torch.linspace(-1, 1, y.numel(), device=DEV).view_as(y)).sum().backward()
        finally:
            ops.set_force_ref(False)
        outs.append(y.detach())
        grads.append({n: p.grad.detach().clone() for n, p in layer.named_parameters() if p.grad is not None})
    assert _rel(outs[0], outs[1]) < 2e-5
    assert grads[0].keys() == grads[1].keys()
    for n in grads[0]:
        assert _rel(grads[0][n], grads[1][n]) < 1e-4, n


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 64, 32, 256), (3, 24, 40, 64), (1, 8, 3, 5)])
def test_pointwise_gemm(shape, dt):
    """Copy-free 1x1 conv GEMM (stride-0 batch bmm) vs torch.matmul in fp32; weight grads fp32."""
    ops, _ = _ops()
    B, O, I, P = shape
    torch.manual_seed(9)
    w = (torch.randn(O, I) / I ** 0.5).to(DEV).requires_grad_(True)
    x = torch.randn(B, I, P).to(dt).to(DEV).requires_grad_(True)
    y = ops.pointwise(w, x)
    assert y.dtype == dt and y.is_contiguous()
    g = torch.randn_like(y)
    y.backward(g)
    assert w.grad.dtype == torch.float32 and x.grad.is_contiguous()
    w2 = w.detach().clone().requires_grad_(True)
    x2 = x.detach().float().requires_grad_(True)
    y2 = torch.matmul(w2, x2)
    y2.backward(g.float())
    tol = _tol(dt)
    assert _rel(y.float(), y2) < tol
    assert _rel(w.grad, w2.grad) < 4 * tol
    assert _rel(x.grad.float(), x2.grad) < 4 * tol


@pytest.mark.parametrize("k", [1, 9])
def test_spectral_conv1d_gemm_path(k):
    """Discriminator heads' Conv1d (circular padding) as one batched GEMM vs F.conv1d."""
    import torch.nn.functional as F
    from networks.discriminator import SpectralConv1d
    torch.manual_seed(10)
    m = SpectralConv1d(24, 16, kernel_size=k, padding=k // 2, padding_mode='circular').to(DEV)
    m(torch.randn(2, 24, 37, device=DEV))              # one power iteration in train mode
    m.eval()
    x = torch.randn(4, 24, 37, device=DEV, requires_grad=True)
    y = m(x)
    w = m.weight.detach()
    x2 = x.detach().clone().requires_grad_(True)
    xp = F.pad(x2, (k // 2, k // 2), mode='circular') if k > 1 else x2
    y2 = F.conv1d(xp, w, m.bias)
    assert _rel(y, y2) < 1e-5
    g = torch.randn_like(y)
    y.backward(g)
    y2.backward(g)
    assert _rel(x.grad, x2.grad) < 1e-5


def test_input_only_grad_skips_parameter_work():
    """torch.autograd.grad(loss, [x]) through a ConvNeXt layer (the adaptive-VF-weight pass,
    reference training/loss.py:262-271): same input gradient as a full backward, and no
    parameter-gradient kernels (depthwise weight grad) are launched for it."""
    from networks.utils.convnext_utils import ConvNeXtSynthesisLayer
    ops, kt = _ops()
    torch.manual_seed(11)
    layer = ConvNeXtSynthesisLayer(64, 32, 7, layer_scale_init=0.5).to(DEV)
    x = torch.randn(2, 64, 32, 32, device=DEV, requires_grad=True)
    w = torch.randn(2, 32, device=DEV)
    r = torch.randn(2, 64, 32, 32, device=DEV)
    y = layer(x, w)
    kt.enable(True)
    (gx,) = torch.autograd.grad((y * r).sum(), x, retain_graph=True)
    torch.cuda.synchronize()
    rec = set(kt.summary())
    kt.enable(False)
    assert any(n.startswith("dwconv2d_bwd_data") for n in rec)
    assert not any(n.startswith("dwconv2d_bwd_weight") for n in rec), rec
    assert all(p.grad is None for p in layer.parameters())
    (y * r).sum().backward()
    assert _rel(gx, x.grad) == 0.0
    assert layer.dwconv.weight.grad is not None and layer.pwconv1.weight.grad is not None


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,C,H,W,O", [(4, 128, 16, 16, 3), (2, 512, 8, 8, 3), (3, 256, 32, 24, 1), (2, 16, 4, 2, 4)])
def test_torgb(dt, B, C, H, W, O):
    """ToRGB (csrc/torgb.hip) vs (W @ (style * x)) + bias in fp32: output, dx, dstyle, dweight, dbias."""
    ops, _ = _ops()
    g = torch.Generator().manual_seed(B * C + H)
    x = torch.randn(B, C, H, W, generator=g).to(dt).float().requires_grad_()
    w2 = (0.1 * torch.randn(O, C, generator=g)).requires_grad_()
    st = (1 + 0.3 * torch.randn(B, C, generator=g)).requires_grad_()
    bias = torch.randn(1, O, 1, 1, generator=g).requires_grad_()

    def hip(x, w2, st, bias):
        return ops.torgb(x.to(dt), w2, st, bias)

    def ref(x, w2, st, bias):
        return torch.einsum('oc,bchw->bohw', w2, x * st[:, :, None, None]) + bias

    _run(hip, ref, [x, w2, st, bias], dt, ['torgb_fwd', 'torgb_bwd'])


@pytest.mark.parametrize("B,C,H", [(4, 32, 16), (3, 8, 5)])
def test_posterior_sample_kl(B, C, H):
    """Fused posterior sample + KL (csrc/posterior.hip) vs DiagonalGaussianDistribution's torch ops
    (reference kl_utils.py:30-56) on the same epsilon: z, kl, and the moment gradients of a loss on
    both outputs (logvar values beyond the clamp included, whose gradient is zero)."""
    from networks.utils import kl_utils
    _, kt = _ops()
    g = torch.Generator().manual_seed(B * C + H)
    params = torch.randn(B, 2 * C, H, H, generator=g)
    params[:, C:, 0, 0] = 25.0              # clamped above
    params[:, C:, 1, 0] = -35.0             # clamped below
    eps = torch.randn(B, C, H, H, generator=g)
    wz = torch.randn(B, C, H, H, generator=g)
    wk = torch.randn(B, generator=g)
    kl_utils.set_noise_source(lambda shape: eps.clone())
    try:
        pg = params.to(DEV).requires_grad_()
        kt.enable(True)
        z, kl = kl_utils.sample_and_kl(pg)
        ((z * wz.to(DEV)).sum() + (kl * wk.to(DEV)).sum()).backward()
        torch.cuda.synchronize()
        names = set(kt.summary())
        kt.enable(False)
        assert "posterior_fwd<f32>" in names and "posterior_bwd<f32>" in names, names
        pr = params.double().requires_grad_()
        post = kl_utils.DiagonalGaussianDistribution(pr)
        zr = post.sample()
        klr = post.kl()
        ((zr * wz.double()).sum() + (klr * wk.double()).sum()).backward()
    finally:
        kl_utils.set_noise_source(None)
    assert _rel(z, zr) < 1e-6
    assert _rel(kl, klr) < 1e-6
    assert _rel(pg.grad, pr.grad) < 1e-5


def test_posterior_nan_logvar_passes_through():
    """torch.clamp passes NaN through: a NaN logvar gives a NaN sample and KL (as the reference's
    DiagonalGaussianDistribution), not the clamped -30 that fminf / fmaxf would produce."""
    from networks.utils import kl_utils
    params = torch.randn(2, 8, 4, 4)
    params[0, 4, 1, 2] = float("nan")
    eps = torch.randn(2, 4, 4, 4)
    kl_utils.set_noise_source(lambda shape: eps.clone())
    try:
        z, kl = kl_utils.sample_and_kl(params.to(DEV))
        post = kl_utils.DiagonalGaussianDistribution(params.double())
        zr, klr = post.sample(), post.kl()
    finally:
        kl_utils.set_noise_source(None)
    assert torch.isnan(z[0, 0, 1, 2]) and torch.isnan(zr[0, 0, 1, 2])
    assert torch.isnan(kl[0]) and torch.isnan(klr[0])
    assert torch.isfinite(kl[1]) and torch.isfinite(z[1]).all()


@pytest.mark.parametrize("C,res", [(128, 32), (64, 48)])
def test_convnext_layer_residual_fusion(C, res, monkeypatch):
    """The residual-branch gradient handed to the dwconv data-gradient kernel (decoder_hip.ResidualSlot)
    gives the layer the same input / parameter gradients as autograd's separate add (bf16 layer:
    one rounding of the sum instead of two, hence 1e-2 of max)."""
    from networks.utils.convnext_utils import ConvNeXtSynthesisLayer
    from torch_utils.ops import decoder_hip
    _, kt = _ops()
    torch.manual_seed(C + res)
    layer = ConvNeXtSynthesisLayer(C, 32, 7, layer_scale_init=0.5).to(DEV)
    x0 = torch.randn(2, C, res, res, device=DEV).to(torch.bfloat16)
    w = torch.randn(2, 32, device=DEV)
    r = torch.randn(2, C, res, res, device=DEV)
    grads = []
    for fused in (True, False):
        monkeypatch.setattr(decoder_hip, "RESIDUAL_FUSION", fused)
        layer.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        kt.enable(True)
        y = layer(x, w, compute_dtype=torch.bfloat16)
        (y.float() * r).sum().backward()
        torch.cuda.synchronize()
        names = set(kt.summary())
        kt.enable(False)
        assert any(n.startswith("dwconv2d_mfma_bwd_data") for n in names), names
        grads.append([x.grad.float()] + [p.grad.float() for p in layer.parameters() if p.grad is not None])
    assert len(grads[0]) == len(grads[1])
    for a, b in zip(*grads):
        assert _rel(a, b) < 1e-2, _rel(a, b)
