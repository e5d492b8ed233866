"""`vfm_pw_gemm_gelu` (csrc/pwgemm.hip): the ConvNeXt MLP channel GEMM with the GELU fused
into its epilogue, against the unfused formulation in fp32 torch
(reference convnext_utils.py:135-138: modulated 1x1 conv -> GELU(erf); backward: the 4C->C
conv's data gradient -> GELU backward).

Tolerances (max error relative to max |ref|): 1e-2 for bf16 outputs (one bf16 ulp is
3.9e-3 relative; the MFMA and the fp32 reference sum in different orders, which can flip
a rounding). MFMA fragment-layout errors show up as O(1) errors."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CASES = [(2, 512, 128, 256), (3, 1024, 256, 384), (2, 2048, 512, 128), (1, 512, 128, 4096), (2, 1024, 256, 2304)]


def _native():
    from torch_utils import custom_ops
    return custom_ops.get_native(), custom_ops


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def _inputs(B, M, K, N, seed):
    g = torch.Generator().manual_seed(seed)
    A = (torch.randn(M, K, generator=g) / K ** 0.5).bfloat16().cuda()
    X = torch.randn(B, K, N, generator=g).bfloat16().cuda()
    s = (torch.rand(B, M, generator=g) + 0.5).cuda()
    bias = torch.randn(M, generator=g).cuda()
    return A, X, s, bias


@pytest.mark.parametrize("B,M,K,N", CASES)
@pytest.mark.parametrize("write_h", [True, False])
def test_forward_gemm_gelu(B, M, K, N, write_h):
    lib, co = _native()
    A, X, s, bias = _inputs(B, M, K, N, 0)
    h = torch.empty(B, M, N, dtype=torch.bfloat16, device="cuda")
    g = torch.empty_like(h)
    rc = lib.vfm_pw_gemm_gelu(A.data_ptr(), X.data_ptr(), s.data_ptr(), bias.data_ptr(), None,
                              h.data_ptr() if write_h else None, g.data_ptr(), None, None, 0, B, M, K, N,
                              co.stream_ptr())
    torch.cuda.synchronize()
    assert rc == 0
    href = torch.matmul(A.float(), X.float())
    gref = F.gelu(href.bfloat16().float() * s[:, :, None] + bias[None, :, None])
    if write_h:
        assert _rel(h.float(), href) < 1e-2
        gref = F.gelu(h.float() * s[:, :, None] + bias[None, :, None])
    assert _rel(g.float(), gref) < 1e-2


@pytest.mark.parametrize("B,M,K,N", CASES)
def test_backward_gemm_gelu(B, M, K, N):
    lib, co = _native()
    A, X, s, bias = _inputs(B, M, K, N, 1)
    hin = torch.randn(B, M, N, generator=torch.Generator().manual_seed(2)).bfloat16().cuda()
    tiles = lib.vfm_pw_gemm_gelu_tiles(N)
    assert tiles == N // 64
    dh = torch.empty(B, M, N, dtype=torch.bfloat16, device="cuda")
    p0 = torch.empty(B, tiles, M, device="cuda")
    p1 = torch.empty_like(p0)
    rc = lib.vfm_pw_gemm_gelu(A.data_ptr(), X.data_ptr(), s.data_ptr(), bias.data_ptr(), hin.data_ptr(),
                              dh.data_ptr(), None, p0.data_ptr(), p1.data_ptr(), 1, B, M, K, N, co.stream_ptr())
    torch.cuda.synchronize()
    assert rc == 0
    dg = torch.matmul(A.float(), X.float()).bfloat16().float()
    z = (hin.float() * s[:, :, None] + bias[None, :, None]).requires_grad_(True)
    F.gelu(z).backward(dg)
    dz = z.grad
    assert _rel(dh.float(), dz * s[:, :, None]) < 1e-2
    assert _rel(p0.sum(1), (dz * hin.float()).sum(-1)) < 1e-2
    assert _rel(p1.sum(1), dz.sum(-1)) < 1e-2


def test_unsupported_shapes_report_no_kernel():
    lib, co = _native()
    assert lib.vfm_pw_gemm_gelu_tiles(100) == co.VFM_NO_KERNEL
    A, X, s, bias = _inputs(1, 512, 128, 128, 3)
    out = torch.empty(1, 512, 128, dtype=torch.bfloat16, device="cuda")
    for (M, K, N) in [(512, 64, 128), (500, 128, 128), (512, 128, 100)]:
        rc = lib.vfm_pw_gemm_gelu(A.data_ptr(), X.data_ptr(), None, None, None, None, out.data_ptr(), None,
                                  None, 0, 1, M, K, N, co.stream_ptr())
        assert rc == co.VFM_NO_KERNEL


@pytest.mark.parametrize("B,C,N", [(2, 128, 256), (3, 256, 384), (1, 128, 4096), (2, 256, 2304)])
def test_convnext_mlp_forward(B, C, N):
    """vfm_convnext_mlp_fwd vs the unfused chain with the same bf16 roundings
    (pointwise -> scale_bias_gelu -> pointwise -> layer_scale_residual)."""
    lib, co = _native()
    g = torch.Generator().manual_seed(4)
    W1 = (torch.randn(4 * C, C, generator=g) / C ** 0.5).bfloat16().cuda()
    W2 = (torch.randn(C, 4 * C, generator=g) / (4 * C) ** 0.5).bfloat16().cuda()
    m = torch.randn(B, C, N, generator=g).bfloat16().cuda()
    x = torch.randn(B, C, N, generator=g).bfloat16().cuda()
    s = (torch.rand(B, 4 * C, generator=g) + 0.5).cuda()
    b1 = torch.randn(4 * C, generator=g).cuda()
    b2 = torch.randn(C, generator=g).cuda()
    gamma = torch.randn(C, generator=g).cuda()
    out = torch.empty_like(x)
    rc = lib.vfm_convnext_mlp_fwd(W1.data_ptr(), m.data_ptr(), s.data_ptr(), b1.data_ptr(), W2.data_ptr(),
                                  b2.data_ptr(), gamma.data_ptr(), x.data_ptr(), out.data_ptr(), None, None, None, B, C, N,
                                  co.stream_ptr())
    torch.cuda.synchronize()
    assert rc == 0
    h = torch.matmul(W1.float(), m.float()).bfloat16().float()
    gv = F.gelu(h * s[:, :, None] + b1[None, :, None]).bfloat16().float()
    y = torch.matmul(W2.float(), gv).bfloat16().float()
    ref = x.float() + gamma[None, :, None] * (y + b2[None, :, None])
    assert _rel(out.float(), ref) < 1e-2
    assert lib.vfm_convnext_mlp_fwd(W1.data_ptr(), m.data_ptr(), None, None, W2.data_ptr(), None, None,
                                    x.data_ptr(), out.data_ptr(), None, None, None, B, 512, N, co.stream_ptr()) == co.VFM_NO_KERNEL


@pytest.mark.parametrize("res", [16, 32])
def test_convnext_layer_nograd_uses_fused_mlp(res):
    """ConvNeXtSynthesisLayer (C=128, bf16) without autograd takes the fused MLP kernel and
    matches the unfused forward to bf16 rounding."""
    from networks.utils.convnext_utils import ConvNeXtSynthesisLayer
    from torch_utils.ops import decoder_hip, kernel_timer
    torch.manual_seed(0)
    lyr = ConvNeXtSynthesisLayer(128, 512, 7, layer_scale_init=0.5, block_index=2, legacy=True).cuda()
    with torch.no_grad():
        for p in lyr.parameters():
            p.add_(torch.randn_like(p) * 0.05)
    x = torch.randn(2, 128, res, res, device="cuda").bfloat16()
    w = torch.randn(2, 512, device="cuda")
    saved = decoder_hip.MLP_CHANNELS
    decoder_hip.MLP_CHANNELS = ()
    with torch.enable_grad():
        ref = lyr(x, w, torch.bfloat16)          # unfused chain
    decoder_hip.MLP_CHANNELS = saved
    kernel_timer.enable(True)
    with torch.no_grad():
        got = lyr(x, w, torch.bfloat16)
    names = set(kernel_timer._records)
    kernel_timer.enable(False)
    assert any(n.startswith("convnext_mlp_fwd") for n in names), names
    assert _rel(got.float(), ref.float()) < 2e-2


def test_convnext_layer_grad_fused_matches_unfused():
    """Autograd path at C=128: fused forward (h, g, y saved) + residual backward + fused
    GELU-backward GEMM, against the unfused Functions; output and every gradient."""
    from networks.utils.convnext_utils import ConvNeXtSynthesisLayer
    from torch_utils.ops import decoder_hip, kernel_timer
    torch.manual_seed(1)
    lyr = ConvNeXtSynthesisLayer(128, 512, 7, layer_scale_init=0.5, block_index=2, legacy=True).cuda()
    with torch.no_grad():
        for p in lyr.parameters():
            p.add_(torch.randn_like(p) * 0.05)
    x0 = torch.randn(2, 128, 32, 32, device="cuda").bfloat16()
    w0 = torch.randn(2, 512, device="cuda")
    dout = torch.randn(2, 128, 32, 32, device="cuda").bfloat16()

    def run(fused):
        saved = decoder_hip.MLP_CHANNELS
        decoder_hip.MLP_CHANNELS = (128,) if fused else ()
        try:
            lyr.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            w = w0.clone().requires_grad_(True)
            kernel_timer.enable(True)
            out = lyr(x, w, torch.bfloat16)
            out.backward(dout)
            names = set(kernel_timer._records)
            kernel_timer.enable(False)
            grads = {n: p.grad.detach().clone() for n, p in lyr.named_parameters() if p.grad is not None}
            return out.detach(), x.grad.detach(), w.grad.detach(), grads, names
        finally:
            decoder_hip.MLP_CHANNELS = saved

    o1, gx1, gw1, g1, n1 = run(True)
    o0, gx0, gw0, g0, n0 = run(False)
    assert any(n.startswith("convnext_mlp_fwd") for n in n1) and any(n.startswith("pw_gemm_gelu_bwd") for n in n1)
    assert not any(n.startswith("convnext_mlp_fwd") for n in n0)
    assert _rel(o1.float(), o0.float()) < 2e-2
    assert _rel(gx1.float(), gx0.float()) < 3e-2
    assert _rel(gw1.float(), gw0.float()) < 3e-2
    assert set(g1) == set(g0)
    for k in g0:
        assert _rel(g1[k].float(), g0[k].float()) < 3e-2, k
