"""The exact-fp32 GEMM on the fp32-input MFMA (csrc/sgemm.hip, `vfm_sgemm`) against an fp64 product of the
same fp32 operands: every operand layout, every tile, ragged M / N / K edges (not multiples of the 32-deep
K-tile or of the output tile), batched and shared (stride-0) operands, K splits, the batch reduction, the
batch-folded narrow planes, and the bias / GELU / alpha-beta epilogues; plus the product shapes the training
step sends it (D heads' batch-folded 1-D convs, the 8^2 / 4^2 decoder 1x1s, the adapter's 64-wide linears).

Tolerance: each output within 2e-5 * (|A| @ |B|) of the fp64 product -- an fp32 fmaf chain over K terms stays
within ~sqrt(K) * 2^-24 of sum |a b| in practice (K <= 6272 here: <= 5e-6), so this bound catches any wrong
operand, dropped K-tile or misplaced output while admitting the exact-fp32 rounding."""
import pytest
import torch

from torch_utils.ops import gemm_hip

DEV = "cuda:0"


def _rnd(*shape, g):
    return (torch.rand(*shape, generator=g, dtype=torch.float64) * 2 - 1).float().to(DEV)


def _store(t, kcont):
    """The same values with K-contiguous (kcont) or outer-contiguous storage of a [.., rows, cols] view whose
    last dim is k (kcont) -- i.e. transposed storage when not kcont."""
    return t if kcont else t.transpose(-1, -2).contiguous().transpose(-1, -2)


def _check(out, A, B, alpha=1.0, extra=None, reduce=False):
    A64, B64 = A.double(), B.double()
    ref = alpha * torch.matmul(A64, B64)
    bound = abs(alpha) * torch.matmul(A64.abs(), B64.abs())
    if reduce:
        ref, bound = ref.sum(0), bound.sum(0)
    if extra is not None:
        ref = ref + extra
        bound = bound + extra.abs()
    err = (out.double() - ref).abs()
    worst = float((err / (bound + 1e-30)).max())
    assert worst < 2e-5, f"worst error {worst:.3e} of |A||B|"


@pytest.mark.gpu
@pytest.mark.parametrize("a_kc", [True, False])
@pytest.mark.parametrize("b_kc", [True, False])
@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 5, 6, 7])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (200, 136, 100), (72, 520, 36), (384, 6272, 384)])
def test_sgemm_layouts_tiles(a_kc, b_kc, tile, M, N, K):
    g = torch.Generator().manual_seed(M * 7 + N + K)
    A = _rnd(M, K, g=g)
    Bt = _rnd(N, K, g=g)
    a = _store(A, a_kc)
    b = Bt.t() if b_kc else Bt.t().contiguous()
    out = gemm_hip.sgemm(a, b, tile=tile, splits=1)
    assert out is not None and out.shape == (M, N)
    _check(out, A, Bt.t())


@pytest.mark.gpu
@pytest.mark.parametrize("splits", [2, 5, 13])
@pytest.mark.parametrize("tile", [0, 7])
@pytest.mark.parametrize("M,N,K", [(384, 384, 6272), (384, 3456, 6272), (96, 200, 1000)])
def test_sgemm_split_k(splits, tile, M, N, K):
    g = torch.Generator().manual_seed(splits + M)
    A = _rnd(M, K, g=g)
    B = _rnd(N, K, g=g).t()                     # [K, N] K-contiguous (the dW = dY cols^T form)
    out = gemm_hip.sgemm(A, B, splits=splits, tile=tile)
    _check(out, A, B)
    auto = gemm_hip.sgemm(A, B)                 # shape-chosen split
    _check(auto, A, B)


@pytest.mark.gpu
@pytest.mark.parametrize("z,M,N,K,shared_a", [(32, 2048, 64, 512, True), (32, 512, 64, 2048, True),
                                               (5, 130, 72, 68, False), (3, 64, 256, 96, False)])
def test_sgemm_batched(z, M, N, K, shared_a):
    g = torch.Generator().manual_seed(z * M + K)
    A = _rnd(1 if shared_a else z, M, K, g=g)
    B = _rnd(z, K, N, g=g)
    out = gemm_hip.sgemm(A.expand(z, M, K) if not shared_a else A, B)
    assert out.shape == (z, M, N)
    _check(out, A.expand(z, M, K), B)


@pytest.mark.gpu
@pytest.mark.parametrize("P", [4, 16, 32])
@pytest.mark.parametrize("a_kc", [True, False])
def test_sgemm_batch_fold(P, a_kc):
    """Per-sample planes narrower than a 64-wide tile run as one product over N = z P columns (lgp folding)."""
    g = torch.Generator().manual_seed(P)
    z, M, K = 32, 512, 2048
    A = _rnd(M, K, g=g)
    B = _rnd(z, K, P, g=g)
    bias = _rnd(M, g=g)
    out = gemm_hip.sgemm(_store(A, a_kc), B, bias=bias, bias_dim=0)
    assert out.shape == (z, M, P)
    _check(out, A.expand(z, M, K), B, extra=bias.double()[:, None])


@pytest.mark.gpu
@pytest.mark.parametrize("z,M,N,K", [(32, 2048, 512, 64), (32, 512, 512, 16), (7, 100, 36, 44)])
def test_sgemm_reduce_batch(z, M, N, K):
    """Weight gradients dW = sum_b dY[b] X[b]^T: the batch inside the split reduction."""
    g = torch.Generator().manual_seed(M + K)
    dY = _rnd(z, M, K, g=g)
    X = _rnd(z, N, K, g=g)
    out = gemm_hip.sgemm(dY, X.transpose(1, 2), reduce_batch=True)
    assert out.shape == (M, N)
    _check(out, dY, X.transpose(1, 2), reduce=True)


@pytest.mark.gpu
@pytest.mark.parametrize("act", [None, "gelu_tanh", "gelu"])
@pytest.mark.parametrize("bias_dim", [None, 0, 1])
@pytest.mark.parametrize("splits", [1, 3])
def test_sgemm_epilogues(act, bias_dim, splits):
    g = torch.Generator().manual_seed(11)
    M, N, K = 200, 136, 260
    A, B = _rnd(M, K, g=g), _rnd(K, N, g=g)
    bias = None
    ref = A.double() @ B.double()
    if bias_dim is not None:
        bias = _rnd(N if bias_dim == 1 else M, g=g)
        ref = ref + (bias.double() if bias_dim == 1 else bias.double()[:, None])
    out = gemm_hip.sgemm(A, B, bias=bias, bias_dim=bias_dim, act=act, splits=splits)
    if act == "gelu_tanh":
        ref = torch.nn.functional.gelu(ref, approximate="tanh")
    elif act == "gelu":
        ref = torch.nn.functional.gelu(ref)
    assert float((out.double() - ref).abs().max() / ref.abs().max()) < 2e-6


@pytest.mark.gpu
def test_sgemm_alpha_beta():
    g = torch.Generator().manual_seed(3)
    M, N, K = 136, 264, 96
    A, B = _rnd(M, K, g=g), _rnd(K, N, g=g)
    C0 = _rnd(M, N, g=g)
    out = C0.clone()
    gemm_hip.sgemm(A, B, out=out, alpha=0.5, beta=-2.0)
    _check(out, A, B, alpha=0.5, extra=-2.0 * C0.double())


@pytest.mark.gpu
def test_sgemm_rank1_and_single_row():
    """The D heads' 1-channel logit layer: W [1, C] cols (M = 1) and its data gradient W^T dY (K = 1)."""
    g = torch.Generator().manual_seed(5)
    w = _rnd(1, 384, g=g)
    cols = _rnd(384, 6272, g=g)
    out = gemm_hip.sgemm(w, cols)
    _check(out, w, cols)
    gy = _rnd(1, 6272, g=g)
    out = gemm_hip.sgemm(w.t(), gy)
    _check(out, w.t(), gy)


@pytest.mark.gpu
def test_sgemm_routes_narrow_fp32_products():
    """try_gemm(auto=True) sends fp32 products narrower than 128 to sgemm (no library fallback)."""
    g = torch.Generator().manual_seed(9)
    W = _rnd(2048, 512, g=g)
    x = _rnd(32, 512, 64, g=g)
    out = gemm_hip.try_gemm(W, x, auto=True)
    assert out is not None and out.shape == (32, 2048, 64)
    _check(out, W.expand(32, 2048, 512), x)
    xs = _rnd(32768, 1024, g=g)
    wl = _rnd(64, 1024, g=g)
    out = gemm_hip.try_gemm(xs, wl.t(), auto=True)
    assert out is not None
    _check(out, xs, wl.t())


@pytest.mark.gpu
@pytest.mark.parametrize("P", [1, 3, 9, 36])
@pytest.mark.parametrize("splits", [1, 2])
def test_sgemm_ragged_planes(P, splits):
    """Per-sample planes whose width is not a multiple of 4 floats (the equivariance decodes' 1 x 1 .. 6 x 6 maps:
    scalar-load staging) forward and transposed, K splits over them (the split combine over N % 4 != 0)."""
    g = torch.Generator().manual_seed(P + splits)
    z, M, K = 8, 512, 520
    W = _rnd(M, K, g=g)
    x = _rnd(z, K, P, g=g)
    out = gemm_hip.sgemm(W, x, splits=splits)
    _check(out, W.expand(z, M, K), x)
    dy = _rnd(z, M, P, g=g)
    out = gemm_hip.sgemm(W.t(), dy, splits=splits)
    _check(out, W.t().expand(z, K, M), dy)
    out = gemm_hip.sgemm(dy, x.transpose(1, 2), reduce_batch=True, splits=splits)
    _check(out, dy, x.transpose(1, 2), reduce=True)
