"""The decoder's self-attention with the learned null key / value (reference
networks/utils/gigagan_utils.py:53-91) on the fused Function (torch_utils/ops/gigaattn_hip.py: projections
written into a packed token-major buffer whose row 0 is the null key / value, attention read in place,
one packed gradient) against the unfused chain of the same module (VFM_GIGA_ATTN off: pointwise GEMMs,
torch.cat of the null key / value, the same attention kernels) and against an fp64 torch restatement.
The GEMMs see transposed operand orientations, so the two HIP paths agree to fp32 rounding: outputs
within 1e-5 of max |ref|, every gradient within 1e-4 (fp64: 2e-5 / 2e-4)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / (b.double().abs().max() + 1e-30))


def _ref64(mod, fmap):
    B, C, H, W = fmap.shape
    h, d = mod.heads, mod.dim_head
    x = F.normalize(fmap, dim=1) * mod.norm.scale * mod.norm.gamma
    x = x.reshape(B, C, H * W)
    wq, wk, wv = (m.weight.reshape(h * d, C) for m in (mod.to_q, mod.to_k, mod.to_v))
    q, k, v = (torch.matmul(w, x).reshape(B, h, d, H * W).transpose(2, 3) for w in (wq, wk, wv))
    nk, nv = (t[None, :, None, :].expand(B, h, 1, d) for t in mod.null_kv.unbind(0))
    k, v = torch.cat([nk, k], 2), torch.cat([nv, v], 2)
    o = F.scaled_dot_product_attention(q, k, v)
    o = o.transpose(2, 3).reshape(B, h * d, H * W)
    return torch.matmul(mod.to_out.weight.reshape(C, h * d), o).reshape(B, C, H, W)


@pytest.mark.parametrize("B,C,HW,heads", [(3, 512, 8, 8), (2, 512, 16, 8), (2, 256, 12, 4)])
def test_null_kv_self_attention_fused_matches_unfused(B, C, HW, heads):
    from networks.utils.gigagan_utils import SelfAttention
    torch.manual_seed(C + HW)
    mod = SelfAttention(C, dim_head=64, heads=heads).cuda()
    with torch.no_grad():
        mod.to_out.weight.normal_(0, 0.02)          # zero-initialised in the reference
        mod.norm.gamma.uniform_(0.5, 1.5)
    fmap = torch.randn(B, C, HW, HW, device="cuda")
    gy = torch.randn(B, C, HW, HW, device="cuda")
    params = [mod.to_q.weight, mod.to_k.weight, mod.to_v.weight, mod.to_out.weight, mod.null_kv, mod.norm.gamma]

    def run(fused):
        mod.fused = fused
        x = fmap.clone().requires_grad_(True)
        y = mod(x)
        grads = torch.autograd.grad(y, [x] + params, gy)
        return y.detach(), grads

    y1, g1 = run(True)
    y0, g0 = run(False)
    assert _rel(y1, y0) < 1e-5
    for a, b in zip(g1, g0):
        assert _rel(a, b) < 1e-4
    mod64 = mod.double()
    x64 = fmap.double().requires_grad_(True)
    y64 = _ref64(mod64, x64)
    g64 = torch.autograd.grad(y64, [x64] + [p for p in (mod64.to_q.weight, mod64.to_k.weight, mod64.to_v.weight,
                                                           mod64.to_out.weight, mod64.null_kv, mod64.norm.gamma)],
                              gy.double())
    assert _rel(y1, y64) < 2e-5
    for a, b in zip(g1, g64):
        assert _rel(a, b) < 2e-4
