"""Discrete-latent codebook lookup: int64 indices must be bit-exact.

* CPU: the C oracle (oracle/ops_oracle.c, fixed fp32 order) against the indices the
  reference itself produced (tests/golden/vq_golden.npz, make_golden_vq.py). The
  reference's fp32 GEMM may sum in another order, so a token may only differ where the
  reference's own top-1/top-2 cosine margin is within rounding (< 1e-6); the test asserts
  that no such token exists in the committed vectors, i.e. the match is exact.
* CPU: this package's VectorQuantizerM (torch path) reproduces the reference's indices,
  f_hat, vq_loss and vocab_usage.
* GPU: the HIP kernel `vfm_codebook_argmax` against the oracle, bit-exact (integer
  indices), including exact ties (first index wins), zero vectors, NaN rows, ragged N,
  strided (split) feature views, every supported width and the config-4 full size.
"""
import numpy as np
import pytest
import torch

import golden_io
from oracle import ops_oracle

G = "vq_golden.npz"
NEAR_TIE = 1e-6


def _a(k):
    return golden_io.load(G)[0][k]


def test_oracle_matches_reference_config4():
    f = _a("m/features").reshape(-1, 32)
    ref = _a("m/indices")                       # [B, 8, L]
    for i in range(8):
        idx = ops_oracle.codebook_argmax(f[:, 4 * i:4 * i + 4], _a(f"m/codebook{i}"))
        r = ref[:, i, :].reshape(-1)
        bad = np.nonzero(idx != r)[0]
        assert all(_a(f"m/margin{i}")[bad] < NEAR_TIE), bad
        assert len(bad) == 0


def test_oracle_matches_reference_wide_ties_zero():
    idx = ops_oracle.codebook_argmax(_a("w/features").reshape(-1, 32), _a("w/codebook"))
    assert np.array_equal(idx, _a("w/indices").reshape(-1))
    idx = ops_oracle.codebook_argmax(_a("t/features"), _a("t/codebook"))
    assert np.array_equal(idx, _a("t/indices").reshape(-1))
    assert idx[0] == 7 and idx[1] == 3          # duplicated / scaled rows: first index wins
    idx = ops_oracle.codebook_argmax(_a("z/features").reshape(-1, 4), _a("z/codebook"))
    assert np.array_equal(idx, _a("z/indices").reshape(-1))


def _vqm_from_golden(device):
    from networks.utils.quant_utils import VectorQuantizerM
    vq = VectorQuantizerM(vocab_size=32768, vocab_width=32, beta=0.25, num_codebooks=8)
    with torch.no_grad():
        for i, cb in enumerate(vq.codebooks):
            cb.codebook.weight.copy_(torch.from_numpy(_a(f"m/codebook{i}")))
    return vq.to(device)


def _check_vqm(device):
    vq = _vqm_from_golden(device)
    feats = torch.from_numpy(_a("m/features")).to(device)
    idx = vq.f_to_idx(feats)
    assert np.array_equal(idx.cpu().numpy(), _a("m/indices"))
    vq.train()
    f_hat, vq_loss, _, usage = vq(feats.clone().requires_grad_(True))
    assert np.allclose(f_hat.detach().cpu().numpy(), _a("m/f_hat"), atol=1e-6)
    assert abs(float(vq_loss) - float(_a("m/vq_loss"))) < 1e-6 * max(1.0, abs(float(_a("m/vq_loss"))))
    assert abs(float(usage) - float(_a("m/vocab_usage"))) < 1e-4


def test_vector_quantizer_cpu_matches_reference():
    _check_vqm("cpu")


# ------------------------------------------------------------------------------ GPU


def _hip(f, w):
    from torch_utils.ops import vq_ops
    return vq_ops.codebook_argmax(f, w).cpu().numpy()


@pytest.mark.gpu
def test_vector_quantizer_gpu_matches_reference():
    _check_vqm("cuda")


@pytest.mark.gpu
def test_hip_matches_oracle_on_golden_inputs():
    f = torch.from_numpy(_a("m/features").reshape(-1, 32)).cuda()
    for i in range(8):
        w = _a(f"m/codebook{i}")
        part = f[:, 4 * i:4 * i + 4]                     # strided view: row stride 32
        got = _hip(part, torch.from_numpy(w).cuda())
        assert np.array_equal(got, ops_oracle.codebook_argmax(part.cpu().numpy(), w))
    for k in ("w", "t", "z"):
        ff, w = _a(f"{k}/features"), _a(f"{k}/codebook")
        ff = ff.reshape(-1, w.shape[1])
        got = _hip(torch.from_numpy(ff).cuda(), torch.from_numpy(w).cuda())
        assert np.array_equal(got, _a(f"{k}/indices").reshape(-1))


@pytest.mark.gpu
@pytest.mark.parametrize("C", [1, 2, 3, 4, 8, 16, 32, 64])
def test_hip_bit_exact_vs_oracle_widths(C):
    g = torch.Generator().manual_seed(C)
    for N, V in ((1, 7), (63, 100), (1000, 3000), (257, 5000)):
        f = torch.randn(N, C, generator=g)
        w = torch.randn(V, C, generator=g)
        got = _hip(f.cuda(), w.cuda())
        assert np.array_equal(got, ops_oracle.codebook_argmax(f.numpy(), w.numpy())), (N, V)


@pytest.mark.gpu
def test_hip_edge_cases():
    g = torch.Generator().manual_seed(5)
    w = torch.randn(300, 4, generator=g)
    w[200] = w[10]                     # exact duplicate later in the book
    w[250] = 0.0                       # zero code (normalises to 0)
    f = torch.randn(40, 4, generator=g)
    f[0] = w[10] * 2.0                 # exact tie with a later duplicate -> 10
    f[1] = 0.0                         # zero feature: all scores 0 -> first index
    f[2, 1] = float("nan")             # NaN feature: every score NaN -> first index
    f[3] = torch.tensor([1e-30, 0, 0, 0])   # below the normalize eps
    got = _hip(f.cuda(), w.cuda())
    exp = ops_oracle.codebook_argmax(f.numpy(), w.numpy())
    assert np.array_equal(got, exp)
    assert got[0] == 10 and got[1] == 0 and got[2] == 0
    w2 = w.clone()
    w2[123, 2] = float("nan")          # a NaN code wins for every token that reaches it
    got = _hip(f.cuda(), w2.cuda())
    assert np.array_equal(got, ops_oracle.codebook_argmax(f.numpy(), w2.numpy()))
    assert _hip(torch.zeros(0, 4).cuda(), w.cuda()).shape == (0,)


@pytest.mark.gpu
def test_hip_config4_full_size_and_idempotence():
    """B=32 x 256 tokens x 8 codebooks of [4096, 4] (config 4): bit-exact on one codebook
    against the oracle, and idempotence on all (quantised codes map to themselves)."""
    g = torch.Generator().manual_seed(9)
    f = torch.randn(32 * 256, 32, generator=g)
    books = [torch.rand(4096, 4, generator=g) * 2 - 1 for _ in range(8)]
    fc = f.cuda()
    for i, w in enumerate(books):
        got = _hip(fc[:, 4 * i:4 * i + 4], w.cuda())
        if i == 0:
            assert np.array_equal(got, ops_oracle.codebook_argmax(f[:, :4].numpy(), w.numpy()))
        again = _hip(w[got].cuda(), w.cuda())      # a code's nearest code is itself
        same = again == got
        # a different answer is only allowed for a (near-)parallel earlier/later code
        wn = w.numpy() / np.linalg.norm(w.numpy(), axis=1, keepdims=True)
        assert np.all(np.abs((wn[again[~same]] * wn[got[~same]]).sum(1) - 1) < 1e-6)
        assert same.mean() > 0.999
