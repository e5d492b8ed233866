"""The full-size backward checker (tests/fullsize_case.py grad_errors / full_grad_error, used by
tests/test_fullsize_bwd_gpu.py) sees layout errors: the reference's own gradient of a square weight passes,
the same gradient transposed keeps its norm and sum but fails the projection and the stored-tensor check.
CPU only: the stored gradients come from the golden (tests/golden/make_golden_fullsize_bwd.py)."""
import json
import os

import numpy as np
import torch

import fullsize_case as fc

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "fullsize_bwd_golden.npz")


def _case(name_part):
    z = np.load(GOLDEN)
    meta = json.loads(str(z["meta"]))
    i = next(i for i, (n, step) in enumerate(meta["full_grads"]) if name_part in n and step == 1)
    n = meta["full_grads"][i][0]
    j = meta["grad_names"].index(n)
    floor = 1e-4 * float(np.max(z["grad_norm"]))
    return n, torch.from_numpy(z[f"full_grad{i}"]).double(), z["grad_norm"][j], z["grad_sum"][j], z["grad_proj"][j], floor


def test_checker_passes_the_reference_gradient():
    for part in ("final_quant.blocks.0.attn.proj", "patch_quants.0.0.blocks.0.attn.proj", "z_convs.2.1.0"):
        n, g, nm, sm, pj, floor = _case(part)
        e_norm, e_proj = fc.grad_errors(n, g, nm, pj, floor)
        assert e_norm < 1e-6 and e_proj < 1e-6, (n, e_norm, e_proj)          # fp32 storage of the fp64 values
        assert abs(float(g.sum()) - sm) <= 1e-5 * max(nm, floor)
        assert fc.full_grad_error(g, g.float().numpy(), 1) == 0.0


def test_checker_fails_a_transposed_gradient():
    for part in ("final_quant.blocks.0.attn.proj", "patch_quants.0.0.blocks.0.attn.proj", "z_convs.2.1.0"):
        n, g, nm, sm, pj, floor = _case(part)
        gt = g.transpose(0, 1).contiguous()                # square weight: same shape, norm and sum
        assert gt.shape == g.shape
        e_norm, e_proj = fc.grad_errors(n, gt, nm, pj, floor)
        assert e_norm < 1e-6                               # what the round-4 checker compared: blind
        assert abs(float(gt.sum()) - sm) <= 1e-5 * max(nm, floor)
        assert e_proj > 0.5, (n, e_proj)                   # ~|g^T - g| / |g| (1.3-1.4 here)
        assert fc.full_grad_error(gt, g.float().numpy(), 1) > 0.25


def test_checker_fails_a_permuted_bucket():
    n, g, nm, sm, pj, floor = _case("final_quant.blocks.0.attn.proj")
    perm = g.flatten()[torch.randperm(g.numel(), generator=torch.Generator().manual_seed(0))].view_as(g)
    e_norm, e_proj = fc.grad_errors(n, perm, nm, pj, floor)
    assert e_norm < 1e-6 and e_proj > 0.5, (e_norm, e_proj)
