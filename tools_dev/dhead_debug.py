"""Diagnostics: the golden D case with decoder_hip's GEMM on vs off; prints every pointwise GEMM
call (shapes, strides, dtype) and the worst gradient differences."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch

import net_cases
from det_init import det_init
from test_networks_parity import _arr
from torch_utils.ops import decoder_hip, gemm_hip
from networks.discriminator import ProjectedDiscriminator

calls = []
orig = gemm_hip.try_gemm


MODE = os.environ.get("SPY_MODE", "check")   # check | torch_out


def spy(A, B, **kw):
    a0, b0 = A.clone(), B.clone()
    out = orig(A, B, **kw)
    err = None
    if out is not None:
        torch.cuda.synchronize()
        changed = (not torch.equal(a0, A)) or (not torch.equal(b0, B))
        ref = a0.double() @ b0.double()
        if kw.get("reduce_batch"):
            ref = ref.sum(0)
        err = (float((out.double() - ref).abs().max() / (ref.abs().max() + 1e-30)), "INPUT CHANGED" if changed else "")
        if MODE == "torch_out":
            out.copy_(ref.to(out.dtype))
    calls.append((tuple(A.shape), A.stride(), tuple(B.shape), B.stride(), str(A.dtype), {k: v for k, v in kw.items()
                                                                                         if k in ("reduce_batch", "splits")},
                  out is not None, err))
    return out


gemm_hip.try_gemm = spy
res = {}
for use in (False, True):
    decoder_hip._USE_HIP_GEMM = use
    calls.clear()
    D = ProjectedDiscriminator(c_dim=0, **net_cases.D_KWARGS).train()
    det_init(D)
    D = D.cuda()
    x = torch.from_numpy(_arr("D/x")).cuda().requires_grad_(True)
    out = D(x, None)
    R = torch.from_numpy(_arr("D/R")).cuda()
    dl = (out.stylegan_t_logits * R).sum() + sum(s[-1].square().mean() for s in out.patchgan_logits)
    dl.backward()
    res[use] = (x.grad.clone(), {n: p.grad.clone() for n, p in D.named_parameters() if p.grad is not None},
                out.stylegan_t_logits.detach().clone())
    if use:
        for c in calls:
            print("call", c)
gx0, g0, l0 = res[False]
gx1, g1, l1 = res[True]
rel = lambda a, b: float((a - b).abs().max() / (b.abs().max() + 1e-30))
print("logits rel", rel(l1, l0), "dx rel", rel(gx1, gx0))
worst = sorted(((rel(g1[n], g0[n]), n) for n in g0), reverse=True)[:8]
for w in worst:
    print("grad", w)
