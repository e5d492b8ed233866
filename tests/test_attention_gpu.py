"""Fused attention forward of the frozen ViT towers (csrc/attention.hip) against the
plain PyTorch fp32 reference of the same op, softmax(q k^T / sqrt(d)) v, evaluated on the
same bf16 inputs.

Tolerance: the kernel rounds P to bf16 before P.V and writes bf16 output (2^-8 relative),
so max |err| <= 1.5e-2 * max|ref| and mean |err| <= 2e-3 * max|ref|; an indexing or
layout error gives O(1) errors. Cases cover the SigLIP2-L shape (packed qkv, 1024 tokens,
16 heads), ragged token counts (DINO ViT-S 197, DINOv2 257/577/1025, N=1 and N=65),
strided [B, H, N, d] operands, and large-magnitude scores whose running max moves across
key tiles (exercises the online-softmax rescale)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(q, k, v):
    """q, k, v: [B, N, H, d] -> [B, N, H, d] fp32."""
    qf, kf, vf = (t.float().permute(0, 2, 1, 3) for t in (q, k, v))
    s = qf @ kf.transpose(-1, -2) * qf.shape[-1] ** -0.5
    return (s.softmax(-1) @ vf).permute(0, 2, 1, 3)


def _check(out, ref):
    err = (out.float() - ref).abs()
    m = float(ref.abs().max())
    assert float(err.max()) <= 1.5e-2 * m, (float(err.max()), m)
    assert float(err.mean()) <= 2e-3 * m, (float(err.mean()), m)


@pytest.mark.parametrize("B,N,H,qscale", [(2, 1024, 16, 1.0), (3, 197, 6, 1.0), (2, 257, 16, 1.0),
                                          (1, 577, 4, 1.0), (1, 1025, 2, 1.0), (2, 1, 3, 1.0),
                                          (2, 65, 2, 1.0), (2, 300, 2, 8.0)])
def test_attention_packed_qkv(B, N, H, qscale):
    from torch_utils.ops import attn_hip, kernel_timer
    g = torch.Generator().manual_seed(N * 7 + H)
    D = H * 64
    qkv = torch.randn(B, N, 3 * D, generator=g)
    qkv[..., :D] *= qscale
    if qscale > 1:            # a drifting key bias: the row max rises tile after tile
        qkv[..., D:2 * D] += torch.linspace(0, 3, N)[None, :, None]
    qkv = qkv.to(torch.bfloat16).to(DEV)
    kernel_timer.enable(True)
    out = attn_hip.attention_packed(qkv, H)
    torch.cuda.synchronize()
    assert any(k.startswith("attention_fwd") for k in kernel_timer.summary())
    kernel_timer.enable(False)
    v5 = qkv.view(B, N, 3, H, 64)
    ref = _ref(v5[:, :, 0], v5[:, :, 1], v5[:, :, 2]).reshape(B, N, D)
    assert out.shape == (B, N, D) and out.dtype == torch.bfloat16
    _check(out, ref)


def test_attention_strided_bhnd_operands():
    """[B, H, N, d]-contiguous q, k, v (head stride N*d) and a preallocated output view."""
    from torch_utils.ops import attn_hip
    g = torch.Generator().manual_seed(11)
    B, H, N = 2, 4, 130
    q, k, v = (torch.randn(B, H, N, 64, generator=g).to(torch.bfloat16).to(DEV) for _ in range(3))
    qv, kv, vv = (t.transpose(1, 2) for t in (q, k, v))          # [B, N, H, d] views
    out = torch.empty(B, N, H, 64, dtype=torch.bfloat16, device=DEV)
    attn_hip.attention(qv, kv, vv, out=out)
    _check(out, _ref(qv, kv, vv))


def test_attention_matches_sdpa_in_siglip_layer():
    """The SigLIP2 attention module (fused path) against F.scaled_dot_product_attention on the
    same bf16 projections."""
    import torch.nn.functional as F
    from networks.utils.vfms.siglip2_utils import SiglipAttention
    cfg = dict(hidden_size=1024, num_attention_heads=16)
    torch.manual_seed(0)
    m = SiglipAttention(cfg).to(DEV)
    x = torch.randn(2, 1024, 1024, device=DEV).to(torch.bfloat16)
    with torch.no_grad():
        got = m(x)
        w, b = m.fused_qkv(x.dtype)
        qkv = torch.addmm(b.to(x.dtype), x.reshape(-1, 1024), w.t()).reshape(2, 1024, 3, 16, 64)
        q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)
        o = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(2, 1024, 1024)
        ref = torch.addmm(m.out_proj.bias.to(x.dtype), o.reshape(-1, 1024), m.out_proj.weight.to(x.dtype).t())
    err = (got.float().reshape(-1, 1024) - ref.float()).abs()
    assert float(err.max()) <= 2e-2 * float(ref.float().abs().max())


def test_attention_rejects_bad_args():
    from torch_utils import custom_ops
    from torch_utils.ops import attn_hip
    x = torch.zeros(1, 8, 2, 32, dtype=torch.bfloat16, device=DEV)      # head dim 32: no kernel
    with pytest.raises(custom_ops.NativeError):
        attn_hip.attention(x, x, x)
