"""Probe: fp32 (f32x6) split-K products of the D heads' folded 1-D conv weight gradients at ragged
reduction depths vs fp64, and whether a split-K launch disturbs neighbouring allocations."""
import sys, torch
sys.path.insert(0, "vfm-vae_amd")
from torch_utils.ops import gemm_hip


def rel(a, b):
    return float((a.double() - b).norm() / b.norm())


torch.manual_seed(0)
for (O, Ck, N) in [(384, 3456, 3136), (384, 3456, 4096), (384, 384, 3136), (384, 3456, 3152), (384, 384, 394)]:
    cols = torch.randn(Ck, N, device="cuda")
    gy = torch.randn(O, N, device="cuda")
    ref_w = gy.double() @ cols.double().t()
    for splits in (1, 2, 3, 5, 6, 8):
        guard = [torch.randn(1 << 20, device="cuda") for _ in range(4)]
        copies = [g.clone() for g in guard]
        out = gemm_hip.try_gemm(gy, cols.t(), out_dtype=torch.float32, splits=splits)
        torch.cuda.synchronize()
        ok = all(torch.equal(g, c) for g, c in zip(guard, copies))
        print(O, Ck, N, "splits", splits, None if out is None else f"{rel(out, ref_w):.2e}", "guards intact" if ok else "GUARDS CHANGED",
              flush=True)
