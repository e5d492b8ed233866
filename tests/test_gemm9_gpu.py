"""The LDS-DMA one-wave-per-SIMD bf16 GEMM (csrc/gemm9.hip, `vfm_gemm9`) against an fp32 product of the
same bf16 operands: every operand layout (K- or M/N-contiguous A and B), bf16 and fp32 outputs, the
bias / GELU / alpha-beta epilogues, ragged M / N edges, one and two K-tiles, batched and shared (stride-0)
operands. Tolerances: fp32 output 2e-5 of max |ref| (fp32 accumulation order); bf16 output one bf16
rounding of the result, 8e-3 of max |ref|."""
import pytest
import torch

from torch_utils.ops import gemm_hip

DEV = "cuda:0"


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / (b.double().abs().max() + 1e-30))


def _rnd(*shape, g):
    return (torch.rand(*shape, generator=g) * 2 - 1).to(torch.bfloat16).to(DEV)


def _operand(t, kcont_inner):
    """The same values with the other memory layout when kcont_inner is False (transposed storage)."""
    return t if kcont_inner else t.transpose(-1, -2).contiguous().transpose(-1, -2)


@pytest.mark.gpu
@pytest.mark.parametrize("a_kc", [True, False])
@pytest.mark.parametrize("b_kc", [True, False])
@pytest.mark.parametrize("M,N,K", [(512, 512, 256), (304, 264, 64), (264, 520, 128), (1024, 768, 1024), (257, 136, 192)])
@pytest.mark.parametrize("out_f32", [False, True])
@pytest.mark.parametrize("persistent", [1, 0])
def test_gemm9_layouts(a_kc, b_kc, M, N, K, out_f32, persistent):
    if M % 8 and not a_kc:
        pytest.skip("M-contiguous A needs M % 8 == 0 (16-B DMA chunks)")
    g = torch.Generator().manual_seed(M + N + K)
    A = _rnd(M, K, g=g)
    Bt = _rnd(N, K, g=g)                       # B = Bt^T: [K, N]
    a = A if a_kc else _operand(A, False)
    b = Bt.t() if b_kc else Bt.t().contiguous()
    ref = A.float() @ Bt.float().t()
    prev = gemm_hip._lib.vfm_gemm9_set_mode(persistent)
    try:
        out = gemm_hip.try_gemm(a, b, route=("g9", 0), out_dtype=torch.float32 if out_f32 else None)
    finally:
        gemm_hip._lib.vfm_gemm9_set_mode(prev)
    assert out is not None and out.shape == (M, N)
    assert _rel(out, ref) < (2e-5 if out_f32 else 8e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("act", [None, "gelu_tanh", "gelu"])
@pytest.mark.parametrize("bias_dim", [None, 0, 1])
def test_gemm9_epilogues(act, bias_dim):
    g = torch.Generator().manual_seed(7)
    M, N, K = 384, 520, 192
    A, Bt = _rnd(M, K, g=g), _rnd(N, K, g=g)
    bias = None
    ref = A.float() @ Bt.float().t()
    if bias_dim is not None:
        bias = torch.randn(M if bias_dim == 0 else N, generator=g).to(DEV)
        ref = ref + (bias[:, None] if bias_dim == 0 else bias[None, :])
    if act == "gelu_tanh":
        ref = torch.nn.functional.gelu(ref, approximate="tanh")
    elif act == "gelu":
        ref = torch.nn.functional.gelu(ref)
    out = gemm_hip.try_gemm(A, Bt.t(), bias=bias, bias_dim=bias_dim, act=act, route=("g9", 0),
                            out_dtype=torch.float32)
    assert _rel(out, ref) < 2e-5
    # alpha / beta on an fp32 output
    c0 = torch.randn(M, N, generator=g).to(DEV)
    out2 = c0.clone()
    gemm_hip.try_gemm(A, Bt.t(), out=out2, alpha=0.5, beta=-2.0, route=("g9", 0), out_dtype=torch.float32)
    assert _rel(out2, 0.5 * (A.float() @ Bt.float().t()) - 2.0 * c0) < 2e-5


@pytest.mark.gpu
@pytest.mark.parametrize("shared", ["A", "B", None])
def test_gemm9_batched(shared):
    """Batched products as the decoder's 1x1 convs run them: W [O, I] shared (stride 0) against per-sample
    planes x[b] [I, P] (N-contiguous), and the data gradient's W^T (M-contiguous A)."""
    g = torch.Generator().manual_seed(11)
    z, O, I, P = 3, 256, 512, 1024
    W = _rnd(O, I, g=g)
    x = _rnd(z, I, P, g=g)
    if shared == "A":
        out = gemm_hip.try_gemm(W, x, route=("g9", 0))
        ref = torch.matmul(W.float(), x.float())
    elif shared == "B":
        dy = _rnd(z, O, P, g=g)
        out = gemm_hip.try_gemm(W.t(), dy, route=("g9", 0))
        ref = torch.matmul(W.t().float(), dy.float())
    else:
        Ws = _rnd(z, O, I, g=g)
        out = gemm_hip.try_gemm(Ws, x, route=("g9", 0))
        ref = torch.matmul(Ws.float(), x.float())
    assert out is not None and out.shape == ref.shape
    assert _rel(out, ref) < 8e-3


@pytest.mark.gpu
def test_gemm9_siglip_shape_bitwise_stable():
    """A full SigLIP2-L shape (32 x 1024 tokens, fc1 with the tanh-GELU epilogue): against fp32, and two
    launches bit-identical (no data race between the DMA ring and the fragment reads)."""
    g = torch.Generator().manual_seed(3)
    M, N, K = 32768, 4096, 1024
    A, W = _rnd(M, K, g=g), _rnd(N, K, g=g)
    b = torch.randn(N, generator=g).to(DEV)
    outs = [gemm_hip.try_gemm(A, W.t(), bias=b, bias_dim=1, act="gelu_tanh", route=("g9", 0)) for _ in range(2)]
    assert torch.equal(outs[0], outs[1])
    rows = torch.randint(0, M, (512,), generator=g).to(DEV)
    ref = torch.nn.functional.gelu(A[rows].float() @ W.float().t() + b, approximate="tanh")
    assert _rel(outs[0][rows], ref) < 8e-3


@pytest.mark.gpu
def test_gemm9_persistent_many_items_bitwise_stable():
    """The persistent form walks several output tiles per workgroup (a K-tile stream across tile boundaries,
    the stores of one tile in flight beside the next tile's first K-tile): a 4096-tile batched product twice,
    bit-identical, and against fp32 on sampled planes."""
    g = torch.Generator().manual_seed(5)
    z, O, I, P = 32, 512, 2048, 4096            # the decoder's b3 pwconv2 at batch 32: 8 K-tiles per tile
    W = _rnd(O, I, g=g)
    x = _rnd(z, I, P, g=g)
    outs = [gemm_hip.try_gemm(W, x, route=("g9", 0)) for _ in range(2)]
    assert torch.equal(outs[0], outs[1])
    for b in (0, 13, 31):
        assert _rel(outs[0][b], W.float() @ x[b].float()) < 8e-3


@pytest.mark.gpu
@pytest.mark.parametrize("O,I,P,z", [(2048, 512, 4096, 32), (256, 1024, 16384, 4), (512, 256, 1024, 3)])
@pytest.mark.parametrize("out_f32", [True, False])
def test_gemm9_batch_reduced_weight_grad(O, I, P, z, out_f32):
    """dW = sum_b dY[b] X[b]^T (the decoder's bf16 1x1 weight gradient) on gemm9's batch-reduced split-K
    (fp32 partials, fixed-order combine): against fp32 (2e-5 of max for fp32 C), deterministic."""
    g = torch.Generator().manual_seed(O + P + z)
    dy, x = _rnd(z, O, P, g=g), _rnd(z, I, P, g=g)
    od = torch.float32 if out_f32 else torch.bfloat16
    outs = [gemm_hip.try_gemm(dy, x.transpose(1, 2), reduce_batch=True, out_dtype=od, auto=True) for _ in range(2)]
    assert outs[0] is not None and outs[0].shape == (O, I)
    assert torch.equal(outs[0], outs[1])
    ref = torch.einsum("bop,bip->oi", dy.float(), x.float())
    assert _rel(outs[0], ref) < (2e-5 if out_f32 else 8e-3)


@pytest.mark.gpu
def test_gemm9_operands_past_2gib():
    """The b5 ConvNeXt layer's data gradient dm = W1^T dh at batch 32: dh is [32, 512, 65536] bf16 = 2 GiB, past
    a buffer descriptor's 31-bit record count. The persistent form moves 64-bit descriptor bases per K-tile and
    output slice; checked against fp32 on the first, a middle and the last sample (where a 32-bit offset would
    wrap), and the batch-reduced weight gradient over the same planes."""
    g = torch.Generator(device=DEV).manual_seed(9)
    z, C, O, P = 32, 128, 512, 65536
    W1 = (torch.rand(O, C, generator=g, device=DEV) * 2 - 1).to(torch.bfloat16)
    dh = (torch.rand(z, O, P, generator=g, device=DEV) * 2 - 1).to(torch.bfloat16)
    dm = gemm_hip.try_gemm(W1.t(), dh, route=("g9", 0))
    assert dm is not None and dm.shape == (z, C, P)
    for b in (0, 17, z - 1):
        assert _rel(dm[b], W1.t().float() @ dh[b].float()) < 8e-3
    m = (torch.rand(z, C, P, generator=g, device=DEV) * 2 - 1).to(torch.bfloat16)
    dw = gemm_hip.try_gemm(dh, m.transpose(1, 2), reduce_batch=True, out_dtype=torch.float32, auto=True)
    ref = torch.zeros(O, C, device=DEV)
    for b in range(z):
        ref += dh[b].float() @ m[b].float().t()
    assert dw is not None and _rel(dw, ref) < 2e-5


def _f32(*shape, g):
    return (torch.rand(*shape, generator=g) * 2 - 1).to(DEV)


def _route_f32(a, b, g9, **kw):
    """fp32 product on the 256-tile f32x6 route: gemm9's persistent kernel (vfm_gemm9_pieces) or gemm8's."""
    prev = gemm_hip.G9_F32, gemm_hip.G9F_BIAS
    gemm_hip.G9_F32 = gemm_hip.G9F_BIAS = g9
    try:
        return gemm_hip.try_gemm(a, b, route=("g8", 0), **kw)
    finally:
        gemm_hip.G9_F32, gemm_hip.G9F_BIAS = prev


@pytest.mark.gpu
@pytest.mark.parametrize("a_kc", [True, False])
@pytest.mark.parametrize("b_kc", [True, False])
@pytest.mark.parametrize("M,N,K,z", [(512, 512, 256, 1), (304, 264, 64, 1), (264, 520, 128, 2), (1024, 768, 1024, 1)])
def test_gemm9_f32x6_pieces(a_kc, b_kc, M, N, K, z):
    """f32x6 on gemm9 (six piece products of a real K-tile as consecutive virtual K-tiles, planar pieces of
    the whole fp32 tensors) against fp64: within twice hipBLASLt's exact-fp32 error, and equal to gemm8's f32x6
    route (same piece products, same K order, same MFMA)."""
    if M % 8 and not a_kc:
        pytest.skip("M-contiguous A needs M % 8 == 0 (16-B DMA chunks)")
    g = torch.Generator().manual_seed(M + N + K + z)
    A = _f32(z, M, K, g=g)
    Bt = _f32(z, N, K, g=g)
    a = A if a_kc else A.transpose(1, 2).contiguous().transpose(1, 2)
    b = Bt.transpose(1, 2) if b_kc else Bt.transpose(1, 2).contiguous()
    if z == 1:
        a, b = a[0], b[0]
    ref = (A.double() @ Bt.double().transpose(1, 2))
    vend = (A @ Bt.transpose(1, 2))
    out = _route_f32(a, b, True)
    out8 = _route_f32(a, b, False)
    assert out is not None and out.shape == out8.shape
    out = out.reshape(ref.shape)
    err, err_v = _rel(out, ref), _rel(vend, ref)
    assert err <= 2 * err_v + 1e-7, (err, err_v)
    assert _rel(out, out8.reshape(ref.shape)) < 1e-6


@pytest.mark.gpu
def test_gemm9_f32x6_bias_alpha_stacked():
    """The bias / alpha epilogue of the f32x6 form and the stacked piece layout (a view that does not cover its
    tensor: per-product split along K)."""
    g = torch.Generator().manual_seed(11)
    M, N, K = 520, 384, 320
    big = _f32(M, 2 * K, g=g)
    A = big[:, :K]                              # a column slice: stacked pieces, not planar
    Bt = _f32(N, K, g=g)
    bias = _f32(N, g=g)
    ref = 0.5 * (A.double() @ Bt.double().t()) + bias.double()
    out = _route_f32(A, Bt.t(), True, bias=bias, bias_dim=1, alpha=0.5)
    assert _rel(out, ref) < 2e-6


@pytest.mark.gpu
@pytest.mark.parametrize("a_kc,b_kc", [(True, False), (False, True), (True, True), (False, False)])
@pytest.mark.parametrize("O,I,P,Bn", [(512, 256, 1024, 6), (304, 264, 320, 3), (2048, 512, 256, 32)])
def test_gemm9_f32x6_batch_reduced(a_kc, b_kc, O, I, P, Bn):
    """sum_b dy[b] x[b]^T (the decoder's fp32 1x1 weight gradients) on gemm9's f32x6 form through the auto
    route: chunks of whole real K-tiles of the batch-concatenated reduction, fp32 partials, fixed-order combine;
    against fp64 and deterministic."""
    from torch_utils.ops import kernel_timer
    g = torch.Generator().manual_seed(O + I + P + Bn)
    dy = _f32(Bn, O, P, g=g)
    x = _f32(Bn, I, P, g=g)
    A = dy if a_kc else dy.transpose(1, 2).contiguous().transpose(1, 2)
    Bm = x.transpose(1, 2) if b_kc else x.transpose(1, 2).contiguous()
    kernel_timer.enable(True)
    prev = gemm_hip.G9F_PLAN
    gemm_hip.G9F_PLAN = True
    try:
        dW = gemm_hip.try_gemm(A, Bm, out_dtype=torch.float32, reduce_batch=True, auto=True)
        torch.cuda.synchronize()
        names = list(kernel_timer.summary())
        again = gemm_hip.try_gemm(A, Bm, out_dtype=torch.float32, reduce_batch=True, auto=True)
    finally:
        kernel_timer.enable(False)
        gemm_hip.G9F_PLAN = prev
    assert any(n.startswith("gemm9<f32x6") for n in names), names
    ref = (dy.double() @ x.double().transpose(1, 2)).sum(0)
    vend = (dy @ x.transpose(1, 2)).sum(0)
    assert _rel(dW, ref) <= 2 * _rel(vend, ref) + 1e-7
    assert torch.equal(dW, again)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(512, 384, 4096), (6304, 384, 1536), (3072, 1024, 8192)])
def test_gemm9_f32x6_split_k(M, N, K):
    """Single products with fewer 256-tiles than CUs (the DINO tower's narrow outputs, the token-major linears'
    weight gradients): K split into chunks of real K-tiles, fp32 partials, fixed-order combine."""
    g = torch.Generator().manual_seed(M + N + K)
    A = _f32(M, K, g=g)
    Bt = _f32(N, K, g=g)
    assert gemm_hip._splits9f(M, N, K, 1, False) > 1
    prev = gemm_hip.G9F_PLAN
    gemm_hip.G9F_PLAN = True
    try:
        out = gemm_hip.try_gemm(A, Bt.t(), out_dtype=torch.float32, auto=True)
        again = gemm_hip.try_gemm(A, Bt.t(), out_dtype=torch.float32, auto=True)
    finally:
        gemm_hip.G9F_PLAN = prev
    ref = A.double() @ Bt.double().t()
    vend = A @ Bt.t()
    assert _rel(out, ref) <= 2 * _rel(vend, ref) + 1e-7
    assert torch.equal(out, again)


@pytest.mark.gpu
@pytest.mark.parametrize("a_kc,b_kc", [(True, False), (False, True), (True, True), (False, False)])
@pytest.mark.parametrize("bias_dim", [0, 1, None])
@pytest.mark.parametrize("M,N,K,z,alpha", [(512, 256, 512, 1, 1.0), (1024, 512, 192, 1, 0.5), (384, 1024, 1024, 2, 1.0)])
def test_gemm9_f32x6_epilogue_layouts(a_kc, b_kc, bias_dim, M, N, K, z, alpha):
    """f32x6 on gemm9 through the pinned 256-tile route with a per-row / per-column bias and alpha, every layout,
    few output tiles (one workgroup per item)."""
    g = torch.Generator().manual_seed(M * 7 + N + K + z)
    A = _f32(z, M, K, g=g)
    Bt = _f32(z, N, K, g=g)
    a = A if a_kc else A.transpose(1, 2).contiguous().transpose(1, 2)
    b = Bt.transpose(1, 2) if b_kc else Bt.transpose(1, 2).contiguous()
    if z == 1:
        a, b = a[0], b[0]
    bias = None if bias_dim is None else _f32(M if bias_dim == 0 else N, g=g)
    ref = alpha * (A.double() @ Bt.double().transpose(1, 2))
    if bias_dim == 0:
        ref = ref + bias.double()[:, None]
    elif bias_dim == 1:
        ref = ref + bias.double()
    out = _route_f32(a, b, True, bias=bias, bias_dim=bias_dim, alpha=alpha)
    assert _rel(out.reshape(ref.shape), ref) < 2e-6


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K,z,b_kc", [(512, 256, 2048, 32, False), (512, 256, 1088, 8, True), (304, 264, 1024, 3, False)])
def test_gemm9_f32x6_batched_split(M, N, K, z, b_kc):
    """Batched products with few tiles per sample (the 16^2 decoder block's 1x1s) on gemm9's batched K-split: chunks
    of real K-tiles per sample into [z][S] fp32 partials, combined per sample in a fixed order; against fp64,
    deterministic."""
    g = torch.Generator().manual_seed(M + N + K + z)
    A = _f32(M, K, g=g)
    Bt = _f32(z, N, K, g=g)
    b = Bt.transpose(1, 2) if b_kc else Bt.transpose(1, 2).contiguous()
    S = max(2, min(256 // (-(-M // 256) * -(-N // 256) * z), (K // 64) // 4))
    ws = torch.empty(gemm_hip._lib.vfm_gemm9_workspace_floats(M, N, K, z, S, 0), dtype=torch.float32, device=DEV)
    pieces = lambda t: gemm_hip._planar(t.unsqueeze(0) if t.dim() == 2 else t, gemm_hip.custom_ops.stream_ptr(t.device))
    pa, pb = pieces(A), pieces(b)
    out = torch.empty(z, M, N, dtype=torch.float32, device=DEV)
    st = gemm_hip.custom_ops.stream_ptr(A.device)
    b_ld = K if b_kc else N
    rc = gemm_hip._lib.vfm_gemm9_pieces(pa[0].data_ptr(), pb[0].data_ptr(), out.data_ptr(), None, M, N, K, z, 1, K, 0,
                                       pa[2], int(b_kc), b_ld, K * N, pb[2], N, M * N, 1.0, 0, ws.data_ptr(), S, 0, st)
    assert rc == 0
    again = out.clone()
    rc = gemm_hip._lib.vfm_gemm9_pieces(pa[0].data_ptr(), pb[0].data_ptr(), again.data_ptr(), None, M, N, K, z, 1, K, 0,
                                       pa[2], int(b_kc), b_ld, K * N, pb[2], N, M * N, 1.0, 0, ws.data_ptr(), S, 0, st)
    ref = torch.matmul(A.double(), Bt.double().transpose(1, 2))
    vend = torch.matmul(A, Bt.transpose(1, 2))
    assert _rel(out, ref) <= 2 * _rel(vend, ref) + 1e-7
    assert torch.equal(out, again)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(64, 512, 256), (512, 48, 128), (40, 40, 4096), (64, 1024, 32768), (24, 96, 2048)])
@pytest.mark.parametrize("a_kc", [True, False])
def test_gemm9_narrow_routes(M, N, K, a_kc):
    """bf16 products narrower than a 128-wide output through try_gemm(auto=True): gemm9 unsplit, or its K split
    (few output tiles over a deep K: `_plan` -> "g9r"); fp32 output within the fp32 accumulation order."""
    if M % 8 and not a_kc:
        pytest.skip("M-contiguous A needs M % 8 == 0 (16-B DMA chunks)")
    g = torch.Generator().manual_seed(M * 3 + N + K)
    A = _rnd(M, K, g=g)
    Bt = _rnd(N, K, g=g)
    a = A if a_kc else _operand(A, False)
    out = gemm_hip.try_gemm(a, Bt.t(), auto=True, out_dtype=torch.float32)
    assert out is not None and out.shape == (M, N)
    assert _rel(out, A.float() @ Bt.float().t()) < 2e-5


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K,z", [(64, 520, 128, 1), (304, 40, 192, 1), (48, 64, 4096, 1), (32, 24, 8192, 1),
                                     (64, 1024, 256, 3), (40, 72, 2048, 2)])
@pytest.mark.parametrize("b_kc", [True, False])
def test_gemm9_narrow_default_route(M, N, K, z, b_kc):
    """bf16 products with an output side of 64 or less through the default routing (preferred() sends every
    bf16 product to gemm9; few-tile deep-K single products run K-split, `_plan` "g9r"): the narrow shapes of
    the bf16 linears' weight gradients (dy^T x over the tokens) and of narrow heads. fp32 output against the
    fp32 product of the same operands at 2e-5, bf16 output at one rounding (8e-3); deterministic."""
    g = torch.Generator().manual_seed(M * 7 + N + K + z)
    A = _rnd(z, M, K, g=g)
    Bt = _rnd(z, N, K, g=g)
    b = Bt.transpose(1, 2) if b_kc else Bt.transpose(1, 2).contiguous()
    ref = torch.matmul(A.float(), Bt.float().transpose(1, 2))
    assert gemm_hip.preferred(A, M, N)
    out = gemm_hip.try_gemm(A, b, out_dtype=torch.float32, auto=True)
    assert out is not None and out.shape == (z, M, N)
    assert _rel(out, ref) < 2e-5
    again = gemm_hip.try_gemm(A, b, out_dtype=torch.float32, auto=True)
    assert torch.equal(out, again)
    outb = gemm_hip.try_gemm(A, b, auto=True)
    assert outb is not None and outb.dtype == torch.bfloat16
    assert _rel(outb, ref) < 8e-3
