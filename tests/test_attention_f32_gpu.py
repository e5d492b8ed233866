"""fp32 attention forward + backward (csrc/attention_f32.hip, 3-term bf16 split on MFMA)
against an fp64 torch restatement of softmax(Q K^T / sqrt(d)) V on the same inputs: the
fusion adapter's packed-qkv layout (reference networks/utils/ldm_utils.py:55-87) and the
decoder's null-key/value self-attention (reference networks/utils/gigagan_utils.py:53-91),
plus ragged token counts (tiles partially filled on both the query and key side).

Tolerance: 5e-5 of max |ref| on O, 2e-4 of max |ref| on dQ/dK/dV (the split products carry
~2^-16 relative error each, accumulated in fp32 over up to 1025 keys)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(q, k, v, do):
    q, k, v = (t.detach().double().requires_grad_(True) for t in (q, k, v))
    s = torch.einsum("bhqd,bhkd->bhqk", q, k) * q.shape[-1] ** -0.5
    o = torch.einsum("bhqk,bhkd->bhqd", s.softmax(-1), v)
    o.backward(do.double())
    return o, q.grad, k.grad, v.grad


def _rel(a, b):
    return float((a.double() - b).abs().max() / b.abs().max())


def _check(q, k, v, seed=0):
    from torch_utils.ops import attn_hip
    g = torch.Generator(device=DEV).manual_seed(seed)
    do = torch.randn(q.shape, generator=g, device=DEV)
    ro, rq, rk, rv = _ref(q, k, v, do)
    qq, kk, vv = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
    assert attn_hip.supported_f32(qq, kk, vv)
    o = attn_hip.sdpa_f32(qq, kk, vv)
    o.backward(do)
    assert _rel(o, ro) < 5e-5
    assert _rel(qq.grad, rq) < 2e-4
    assert _rel(kk.grad, rk) < 2e-4
    assert _rel(vv.grad, rv) < 2e-4


@pytest.mark.parametrize("B,H,Nq,Nk", [(2, 3, 200, 200), (1, 2, 64, 64), (2, 1, 37, 5), (1, 2, 130, 257),
                                       (2, 2, 1024, 1025)])
def test_attention_f32_contiguous(B, H, Nq, Nk):
    g = torch.Generator(device=DEV).manual_seed(Nq * 7 + Nk)
    q = torch.randn(B, H, Nq, 64, generator=g, device=DEV)
    k = torch.randn(B, H, Nk, 64, generator=g, device=DEV)
    v = torch.randn(B, H, Nk, 64, generator=g, device=DEV)
    _check(q, k, v)


def test_attention_f32_packed_qkv_large_scores():
    """Adapter layout: qkv [B, N, 3, H, d] permuted in place; scores of O(30) stress the softmax."""
    B, N, H = 2, 1024, 16
    g = torch.Generator(device=DEV).manual_seed(3)
    qkv = torch.randn(B, N, 3 * H * 64, generator=g, device=DEV) * 2.5
    q, k, v = qkv.reshape(B, N, 3, H, 64).permute(2, 0, 3, 1, 4).unbind(0)
    _check(q, k, v, seed=1)


def test_attention_f32_null_kv_cat():
    """Decoder layout: q contiguous [B, h, P, d], k/v = cat(null, k) along tokens (P + 1 keys)."""
    B, h, P = 2, 8, 256
    g = torch.Generator(device=DEV).manual_seed(5)
    q = torch.randn(B, h, P, 64, generator=g, device=DEV)
    nk = torch.randn(1, h, 1, 64, generator=g, device=DEV).expand(B, h, 1, 64)
    k = torch.cat([nk, torch.randn(B, h, P, 64, generator=g, device=DEV)], 2)
    v = torch.cat([nk * 0.5, torch.randn(B, h, P, 64, generator=g, device=DEV)], 2)
    _check(q, k, v)
