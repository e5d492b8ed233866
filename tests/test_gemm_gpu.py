"""MFMA GEMM (csrc/gemm.hip) against the plain PyTorch fp32 reference of the same product.

Tolerances (max |err| / max |ref|):
  bf16 operands, fp32 accumulation: 1e-5 for fp32 output (same products, other summation
  order), 8e-3 for bf16 output (one output rounding);
  fp32 operands (the default f32x6 mode: three exact bf16 pieces per operand, six piece
  products, dropped terms <= ~2^-23 per product, fp32 accumulation): 2e-6 against the fp32
  hipBLASLt product -- the size of fp32 accumulation differences at these depths, the
  reference's precision (TF32 off, training_loop.py:504-505); test_gemm_f32x6_matches_fp32
  additionally bounds the error against fp64 by twice hipBLASLt's own fp32 error;
  the opt-in f32x3 mode (hi / lo, three products, ~2^-15.5 per product): F32_TOL.
Layouts: every (A, B) contiguity combination, batched with shared and per-batch operands,
ragged M/N/K (tails inside a tile), bias per row / per column, tanh/erf GELU, alpha/beta
accumulation, split-K and the batch-reducing form used for 1x1-conv weight gradients."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


F32_TOL = 2e-6
F32X3_TOL = 5e-5


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / (b.double().abs().max() + 1e-30))


def _make(shape, dtype, g, kcont_last=True):
    t = torch.randn(*shape, generator=g)
    return t.to(dtype).to(DEV)


def _ref_epi(c, bias=None, bias_dim=1, act=None):
    if bias is not None:
        c = c + (bias[None, :] if bias_dim == 1 else bias[:, None])
    if act == "gelu_tanh":
        c = torch.nn.functional.gelu(c, approximate="tanh")
    elif act == "gelu":
        c = torch.nn.functional.gelu(c)
    return c


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("a_t,b_t", [(False, True), (False, False), (True, True), (True, False)])
@pytest.mark.parametrize("M,N,K", [(256, 384, 512), (200, 136, 72), (8, 520, 1024)])
def test_gemm_layouts(dtype, a_t, b_t, M, N, K):
    from torch_utils.ops import gemm_hip
    g = torch.Generator().manual_seed(M + N + K)
    A = _make((K, M) if a_t else (M, K), dtype, g)
    B = _make((N, K) if b_t else (K, N), dtype, g)
    Av = A.t() if a_t else A
    Bv = B.t() if b_t else B
    out = gemm_hip.gemm(Av, Bv, out_dtype=torch.float32)
    ref = Av.float() @ Bv.float()
    tol = 1e-5 if dtype == torch.bfloat16 else F32_TOL
    assert _rel(out, ref) < tol


@pytest.mark.parametrize("act", [None, "gelu_tanh", "gelu"])
@pytest.mark.parametrize("bias_dim", [None, 1, 0])
def test_gemm_epilogue_bf16(act, bias_dim):
    """The SigLIP2 fc1 form: x [M, K] @ W^T [K, N] + bias, tanh-GELU, bf16 out."""
    from torch_utils.ops import gemm_hip
    g = torch.Generator().manual_seed(3)
    M, N, K = 300, 264, 136
    x = _make((M, K), torch.bfloat16, g)
    w = _make((N, K), torch.bfloat16, g)
    bias = None if bias_dim is None else torch.randn(N if bias_dim == 1 else M, generator=g).to(DEV)
    out = gemm_hip.gemm(x, w.t(), bias=bias, bias_dim=bias_dim, act=act)
    assert out.dtype == torch.bfloat16
    ref = _ref_epi(x.float() @ w.float().t(), bias, bias_dim if bias_dim is not None else 1, act)
    assert _rel(out.float(), ref) < 8e-3


def test_gemm_alpha_beta_accumulate():
    from torch_utils.ops import gemm_hip
    g = torch.Generator().manual_seed(4)
    A = _make((96, 64), torch.float32, g)
    B = _make((64, 72), torch.float32, g)
    C = _make((96, 72), torch.float32, g)
    ref = 0.5 * (A @ B) + 2.0 * C
    gemm_hip.gemm(A, B, out=C, alpha=0.5, beta=2.0)
    assert _rel(C, ref) < F32_TOL


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_gemm_batched_1x1_conv_forms(dtype):
    """Decoder 1x1 conv: W [O, I] . x[b] [I, P] (shared weight); its data gradient
    W^T . dy[b]; its weight gradient sum_b dy[b] . x[b]^T (reduce_batch, split-K)."""
    from torch_utils.ops import gemm_hip
    g = torch.Generator().manual_seed(5)
    Bn, O, I, P = 3, 96, 64, 200
    W = _make((O, I), dtype, g)
    x = _make((Bn, I, P), dtype, g)
    dy = _make((Bn, O, P), dtype, g)
    tol = 1e-5 if dtype == torch.bfloat16 else F32_TOL
    y = gemm_hip.gemm(W, x, out_dtype=torch.float32)
    assert y.shape == (Bn, O, P) and _rel(y, W.float() @ x.float()) < tol
    dx = gemm_hip.gemm(W.t(), dy, out_dtype=torch.float32)
    assert _rel(dx, W.float().t() @ dy.float()) < tol
    for splits in (1, 3):
        dW = gemm_hip.gemm(dy, x.transpose(1, 2), out_dtype=torch.float32, reduce_batch=True, splits=splits)
        assert dW.shape == (O, I)
        assert _rel(dW, (dy.float() @ x.float().transpose(1, 2)).sum(0)) < tol


def test_gemm_split_k_deterministic():
    from torch_utils.ops import gemm_hip
    g = torch.Generator().manual_seed(6)
    A = _make((128, 4096), torch.float32, g)
    B = _make((4096, 256), torch.float32, g)
    o1 = gemm_hip.gemm(A, B, splits=8)
    o2 = gemm_hip.gemm(A, B, splits=8)
    assert torch.equal(o1, o2)
    assert _rel(o1, A @ B) < F32_TOL


@pytest.mark.parametrize("K", [64, 1024, 4096])
def test_gemm_f32x6_matches_fp32(K, monkeypatch):
    """fp32-equivalence of the default split on both kernels: error vs the fp64 product within its
    analytic bound (dropped terms 2^-22 + fp32 accumulation K 2^-24, relative to |A||B|) and, in
    norm, within twice the error of hipBLASLt's exact-fp32 GEMM on the same operands."""
    from torch_utils.ops import gemm_hip
    g = torch.Generator().manual_seed(7 + K)
    A = torch.randn(512, K, generator=g, dtype=torch.float64).float()
    B = torch.randn(K, 512, generator=g, dtype=torch.float64).float()
    exact = A.double() @ B.double()
    blas = (A.to(DEV) @ B.to(DEV)).double().cpu()
    eb = float((blas - exact).norm())
    for fast in (True, False):
        monkeypatch.setattr(gemm_hip, "FAST", fast)
        monkeypatch.setattr(gemm_hip, "FAST_MIN_MN", 0)
        out = gemm_hip.gemm(A.to(DEV), B.to(DEV)).double().cpu()
        bound = (A.double().abs() @ B.double().abs()) * (2.0 ** -22 + K * 2.0 ** -24)
        assert bool(((out - exact).abs() <= bound).all())
        assert float((out - exact).norm()) <= 2.0 * eb + 1e-30, (fast, float((out - exact).norm()), eb)


def test_gemm_f32x3_opt_in(monkeypatch):
    """The opt-in 3-term split (VFM_F32_PRODUCTS=f32x3): within its ~2^-15.5-per-product bound."""
    from torch_utils import custom_ops
    from torch_utils.ops import gemm_hip
    monkeypatch.setattr(custom_ops, "F32_PRODUCTS", "f32x3")
    g = torch.Generator().manual_seed(7)
    A = torch.randn(256, 1024, generator=g, dtype=torch.float64)
    B = torch.randn(1024, 256, generator=g, dtype=torch.float64)
    for fast in (True, False):
        monkeypatch.setattr(gemm_hip, "FAST", fast)
        monkeypatch.setattr(gemm_hip, "FAST_MIN_MN", 0)
        out = gemm_hip.gemm(A.float().to(DEV), B.float().to(DEV)).double().cpu()
        exact = A.float().double() @ B.float().double()
        bound = (A.abs() @ B.abs()) * 2.0 ** -15.5 + 1024 * 2.0 ** -24 * (A.abs() @ B.abs())
        assert bool(((out - exact).abs() <= bound).all())
        assert _rel(out, exact) < F32X3_TOL


def test_gemm_unsupported_shape_routes_exact_fp32(monkeypatch):
    """K = 7 (not a multiple of 4 fp32 elements): none of the bf16-piece kernels takes it; try_gemm hands it to the
    exact-fp32 kernel (csrc/sgemm.hip, scalar-load staging), and returns None only with that route off."""
    from torch_utils.ops import gemm_hip
    A = torch.randn(10, 7, device=DEV)
    B = torch.randn(7, 12, device=DEV)
    out = gemm_hip.try_gemm(A, B)
    assert out is not None and _rel(out, A.double() @ B.double()) < 1e-6
    monkeypatch.setattr(gemm_hip, "SGEMM", False)
    assert gemm_hip.try_gemm(A, B) is None


@pytest.fixture(params=[1, 0], ids=["deep", "one_ahead"])
def g8_schedule(request, monkeypatch):
    """Both K-tile staging schedules of gemm8 (two / one K-tiles ahead); bf16 products routed to gemm8
    rather than gemm9 (the default bf16 kernel, tests/test_gemm9_gpu.py)."""
    from torch_utils import custom_ops
    from torch_utils.ops import gemm_hip
    monkeypatch.setattr(gemm_hip, "G9", False)
    monkeypatch.setattr(gemm_hip, "G9_F32", False)
    lib = custom_ops.get_native()
    prev = lib.vfm_gemm8_set_schedule(request.param)
    yield request.param
    lib.vfm_gemm8_set_schedule(prev)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("a_t,b_t", [(False, True), (False, False), (True, True), (True, False)])
@pytest.mark.parametrize("M,N,K", [(512, 768, 256), (520, 776, 128), (256, 256, 64), (1000, 264, 704),
                                   (512, 512, 128)])
def test_gemm_fast_path_layouts(dtype, a_t, b_t, M, N, K, monkeypatch, g8_schedule):
    """The 256-tile LDS-DMA kernel (csrc/gemm8.hip, 4-phase pipeline) and, for fp32, the piece split
    walked as 6 product terms; bf16 K = 64 / 128 are the one- and two-K-tile paths of the prologue and
    tail."""
    from torch_utils.ops import gemm_hip, kernel_timer
    kernel = "gemm8"
    monkeypatch.setattr(gemm_hip, "FAST_MIN_MN", 0)
    g = torch.Generator().manual_seed(M * 3 + N + K)
    A = _make((K, M) if a_t else (M, K), dtype, g)
    B = _make((N, K) if b_t else (K, N), dtype, g)
    Av = A.t() if a_t else A
    Bv = B.t() if b_t else B
    kernel_timer.enable(True)
    out = gemm_hip.gemm(Av, Bv, out_dtype=torch.float32)
    torch.cuda.synchronize()
    assert any(k.startswith(kernel + "<") for k in kernel_timer.summary())
    kernel_timer.enable(False)
    tol = 1e-5 if dtype == torch.bfloat16 else F32_TOL
    assert _rel(out, Av.float() @ Bv.float()) < tol


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_gemm_fast_epilogue_batched(dtype):
    from torch_utils.ops import gemm_hip
    g = torch.Generator().manual_seed(9)
    Bn, O, I, P = 2, 256, 128, 1024
    W = _make((O, I), dtype, g)
    x = _make((Bn, I, P), dtype, g)
    bias = torch.randn(O, generator=g).to(DEV)
    y = gemm_hip.gemm(W, x, bias=bias, bias_dim=0, act="gelu", out_dtype=torch.float32, cache_a=True)
    ref = torch.nn.functional.gelu(W.float() @ x.float() + bias[:, None])
    assert _rel(y, ref) < (1e-5 if dtype == torch.bfloat16 else F32_TOL)
    y2 = gemm_hip.gemm(W, x, bias=bias, bias_dim=0, act="gelu", out_dtype=torch.float32, cache_a=True)
    assert torch.equal(y, y2)                                   # cached weight split reused
    with torch.no_grad():
        W.mul_(2.0)                                             # version bump invalidates the cache
    y3 = gemm_hip.gemm(W, x, bias=bias, bias_dim=0, act="gelu", out_dtype=torch.float32, cache_a=True)
    ref3 = torch.nn.functional.gelu(W.float() @ x.float() + bias[:, None])
    assert _rel(y3, ref3) < (1e-5 if dtype == torch.bfloat16 else F32_TOL)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("act", [None, "gelu_tanh"])
@pytest.mark.parametrize("bias_dim", [None, 1, 0])
def test_gemm8_fp32_output_epilogue(dtype, act, bias_dim, monkeypatch, g8_schedule):
    """gemm8's fp32-output epilogue: full 256 x 256 tiles go through the LDS-staged 16-B store form
    (alpha, row / column bias, GELU), the ragged last tiles through the per-element form."""
    from torch_utils.ops import gemm_hip
    monkeypatch.setattr(gemm_hip, "FAST_MIN_MN", 0)
    g = torch.Generator().manual_seed(11)
    Bn, M, N, K = 2, 512, 776, 192
    A = _make((M, K), dtype, g)
    x = _make((Bn, K, N), dtype, g)
    bias = None if bias_dim is None else torch.randn(N if bias_dim == 1 else M, generator=g).to(DEV)
    y = gemm_hip.gemm(A, x, bias=bias, bias_dim=bias_dim, act=act, alpha=0.75, out_dtype=torch.float32,
                      cache_a=True)
    ref = _ref_epi(0.75 * (A.float() @ x.float()), bias, bias_dim if bias_dim is not None else 1, act)
    assert _rel(y, ref) < (1e-5 if dtype == torch.bfloat16 else F32_TOL)


def test_gemm_generic_path_when_fast_off(monkeypatch):
    from torch_utils.ops import gemm_hip
    monkeypatch.setattr(gemm_hip, "FAST", False)
    g = torch.Generator().manual_seed(10)
    A = _make((512, 256), torch.float32, g)
    B = _make((256, 768), torch.float32, g)
    assert _rel(gemm_hip.gemm(A, B), A @ B) < F32_TOL


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("a_kc,b_kc", [(True, False), (False, True), (True, True)])
@pytest.mark.parametrize("O,I,P,Bn", [(512, 256, 1024, 6), (304, 264, 320, 3)])
def test_gemm8_batch_reduced_weight_gradient(dtype, a_kc, b_kc, O, I, P, Bn, monkeypatch, g8_schedule):
    """sum_b dy[b] . x[b]^T on gemm8's split-K over the batch-concatenated K (opt-in path,
    VFM_GEMM8_SPLIT=1): fp32 partials + fixed-order reduce; every operand layout; ragged M/N."""
    from torch_utils.ops import gemm_hip, kernel_timer
    monkeypatch.setattr(gemm_hip, "SPLIT8", True)
    g = torch.Generator().manual_seed(O + I + P)
    dy = _make((Bn, O, P), dtype, g)
    x = _make((Bn, I, P), dtype, g)
    A = dy if a_kc else dy.transpose(1, 2).contiguous().transpose(1, 2)
    Bm = x.transpose(1, 2) if b_kc else x.transpose(1, 2).contiguous()
    kernel_timer.enable(True)
    dW = gemm_hip.gemm(A, Bm, out_dtype=torch.float32, reduce_batch=True)
    torch.cuda.synchronize()
    assert any(k.startswith("gemm8<") for k in kernel_timer.summary())
    kernel_timer.enable(False)
    ref = (dy.double() @ x.double().transpose(1, 2)).sum(0)
    assert _rel(dW, ref) < (1e-5 if dtype == torch.bfloat16 else F32_TOL)
    assert torch.equal(dW, gemm_hip.gemm(A, Bm, out_dtype=torch.float32, reduce_batch=True))   # deterministic


@pytest.mark.parametrize("M,N,K", [(768, 512, 8192), (256, 300, 2048)])
def test_gemm8_split_k(M, N, K, monkeypatch, g8_schedule):
    """Few output tiles over a deep K (the adapter's weight gradients): split-K on gemm8 with a bias
    epilogue in the reduce pass."""
    from torch_utils.ops import gemm_hip
    monkeypatch.setattr(gemm_hip, "SPLIT8", True)
    g = torch.Generator().manual_seed(M + K)
    A = _make((M, K), torch.float32, g)
    B = _make((K, N), torch.float32, g)
    bias = torch.randn(N, generator=g).to(DEV)
    out = gemm_hip.gemm(A, B, bias=bias, splits=4)
    ref = A.double() @ B.double() + bias.double()
    assert _rel(out, ref) < F32_TOL


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("a_t,b_t", [(False, True), (True, False)])
@pytest.mark.parametrize("M,N,K,Z", [(4352, 4608, 192, 1), (520, 1000, 128, 40), (4400, 2056, 64, 1)])
@pytest.mark.parametrize("out_bf16", [False, True])
def test_gemm8_many_tiles(dtype, a_t, b_t, M, N, K, Z, out_bf16, g8_schedule):
    """More tiles than CUs (289-480 blocks), batched operands and ragged edges through the buffer-
    descriptor DMA offsets."""
    from torch_utils.ops import gemm_hip
    g = torch.Generator().manual_seed(M + N + K + Z)
    A = _make((Z, K, M) if a_t else (Z, M, K), dtype, g)
    B = _make((Z, N, K) if b_t else (Z, K, N), dtype, g)
    Av = A.transpose(1, 2) if a_t else A
    Bv = B.transpose(1, 2) if b_t else B
    odt = torch.bfloat16 if (out_bf16 and dtype == torch.bfloat16) else torch.float32
    out = gemm_hip.try_gemm(Av, Bv, out_dtype=odt, route=("g8", 0))
    assert out is not None
    ref = torch.bmm(Av.float(), Bv.float())
    tol = (8e-3 if odt == torch.bfloat16 else 1e-5) if dtype == torch.bfloat16 else F32_TOL
    assert _rel(out.float(), ref) < tol


def test_gemm8_split_k_ragged_chunks(g8_schedule):
    """Split-K over several chunks per tile, the last one shorter."""
    from torch_utils.ops import gemm_hip
    g = torch.Generator().manual_seed(11)
    A = _make((2048, 2432), torch.bfloat16, g)
    B = _make((2432, 2304), torch.bfloat16, g)
    out = gemm_hip.try_gemm(A, B, out_dtype=torch.float32, route=("g8", 10))
    assert _rel(out, A.float() @ B.float()) < 1e-5


@pytest.mark.parametrize("a_t", [False, True])
@pytest.mark.parametrize("O,I,P,Bn", [(512, 512, 64, 32), (2048, 512, 64, 5), (200, 136, 16, 9), (3, 40, 8, 17)])
@pytest.mark.parametrize("bias_dim", [None, 0])
def test_gemm_batch_folded_narrow_planes(a_t, O, I, P, Bn, bias_dim, monkeypatch):
    """Shared A (1x1-conv weight, or its transpose for the data gradient) times per-sample planes of
    P < 128 columns: one batch-folded product (vfm_gemm_fold, kernel timer region gemm_fold), f32x6
    products against the fp32 reference at the fp32 tolerance."""
    from torch_utils.ops import gemm_hip, kernel_timer
    monkeypatch.setattr(gemm_hip, "FOLD", True)          # opt-in on the network path (VFM_GEMM_FOLD=1)
    g = torch.Generator().manual_seed(O + I + P + Bn)
    W = torch.randn(I, O, generator=g).to(DEV) if a_t else torch.randn(O, I, generator=g).to(DEV)
    Wv = W.t() if a_t else W
    x = torch.randn(Bn, I, P, generator=g).to(DEV)
    bias = torch.randn(O, generator=g).to(DEV) if bias_dim is not None else None
    kernel_timer.enable(True)
    out = gemm_hip.try_gemm(Wv, x, bias=bias, bias_dim=bias_dim, auto=True)
    names = set(kernel_timer.summary())
    kernel_timer.enable(False)
    assert out is not None and out.shape == (Bn, O, P)
    if a_t and O % 4:
        # an MN-contiguous A needs its contiguous extent (M) % 4 == 0 for the f32x6 fold: the exact-fp32
        # kernel (csrc/sgemm.hip, scalar-load staging) takes the product
        assert any(n.startswith("sgemm<") for n in names), names
    else:
        assert any(n.startswith("gemm_fold<") for n in names), names
    ref = torch.matmul(Wv.double(), x.double())
    if bias is not None:
        ref = ref + bias.double()[None, :, None]
    assert _rel(out, ref) < F32_TOL


@pytest.mark.parametrize("a_t,b_t", [(False, True), (False, False), (True, True), (True, False)])
@pytest.mark.parametrize("M,N,K,Z,reduce", [(520, 776, 128, 3, False), (512, 256, 1024, 4, True),
                                            (256, 1000, 192, 1, False)])
def test_gemm8_planar_pieces_bit_identical(a_t, b_t, M, N, K, Z, reduce, monkeypatch):
    """Planar pieces ([3][tensor], one split per fp32 tensor, vfm_gemm8_pieces) against the per-product
    stacked split (vfm_split_f32 along K): the same pieces and term order, so bit-identical outputs;
    the split is reused by the transposed view and redone after an in-place update."""
    from torch_utils.ops import gemm_hip
    g = torch.Generator().manual_seed(M + N + K + Z)
    A = _make((Z, K, M) if a_t else (Z, M, K), torch.float32, g)
    B = _make((Z, N, K) if b_t else (Z, K, N), torch.float32, g)
    Av = A.transpose(1, 2) if a_t else A
    Bv = B.transpose(1, 2) if b_t else B
    route = ("g8", 4) if reduce else ("g8", 0)
    monkeypatch.setattr(gemm_hip, "PLANAR", True)
    planar = gemm_hip.try_gemm(Av, Bv, out_dtype=torch.float32, reduce_batch=reduce, route=route)
    assert getattr(A, "_vfm_planar", None) is not None and getattr(B, "_vfm_planar", None) is not None
    monkeypatch.setattr(gemm_hip, "PLANAR", False)
    stacked = gemm_hip.try_gemm(Av, Bv, out_dtype=torch.float32, reduce_batch=reduce, route=route)
    assert torch.equal(planar, stacked)
    ref = torch.bmm(Av.double(), Bv.double())
    ref = ref.sum(0) if reduce else ref
    assert _rel(planar, ref) < F32_TOL
    # the cached split follows the tensor's version
    monkeypatch.setattr(gemm_hip, "PLANAR", True)
    A.mul_(0.5)
    again = gemm_hip.try_gemm(Av, Bv, out_dtype=torch.float32, reduce_batch=reduce, route=route)
    assert torch.equal(again, planar * 0.5)
