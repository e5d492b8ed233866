"""Full-size parity of the TRAINING backward on cuda:0 against vectors generated from the reference
itself (tests/golden/make_golden_fullsize_bwd.py): the f16d32 stage-0 Generator on the full SigLIP2-L
tower at 256^2, batch 1, KL / VF losses on, posterior noise from the CPU generator as the reference
draws it, and loss = sum(gen_img R) + sum_i sum(ms_i R_i) + 3 vf + 1e-3 kl back-propagated into the
groups the G phase trains (synthesis, mapping, ldm_adapter; reference networks/generator.py:1152-1206,
training/loss.py:721-1001). The reference side is fp32 (CPU).

Every parameter gradient is checked by its norm, its sum and its projection <g, P> on a seeded random P
(tests/fullsize_case.py grad_probe), and the weights of fullsize_case.FULL_GRADS element-wise (one 1x1 per
decoder block, a square latent-stem 1x1, the adapter's projections): norm and sum alone cannot see a
transposed or permuted gradient, the projection and the stored tensors can (tests/test_fullsize_checker.py
proves it on CPU with a deliberately transposed gradient).

Stated tolerances (the matched-precision bf16 test at the end has its own):
  fp32 -- the product path at reference precision (decoder num_fp16_res 0, fp32 tower; our kernels
  with fp32-equivalent f32x6 products): loss terms 1e-5 relative; every parameter's gradient norm and
  projection within FP32_TOL = 2e-4 (relative to the gradient's norm, floor 1e-4 of the largest norm for
  gradients that are ~0 in exact math), sum within 1e-3 scaled; stored gradients within 2e-4; group
  norms 1e-3;
  bf16 -- the bench's precision (decoder blocks 3-5 and the SigLIP2 tower in bf16, BASELINE config 1)
  against the same fp32 numbers: loss within 3e-2, group gradient norms within 5e-2, every parameter's
  gradient norm within BF16_NORM_TOL and projection within BF16_PROJ_TOL of its own size (floor 1e-3 of
  the largest), stored gradients within BF16_PROJ_TOL: bf16 rounding noise (2^-8 per op over ~60 ops of
  depth), set at about 1.5x the worst case measured on MI355X (below), while a layout / indexing error
  moves the projection by O(1).
"""
import json
import os

import numpy as np
import pytest
import torch

import fullsize_case as fc
from det_init import det_init

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "fullsize_bwd_golden.npz")


@pytest.fixture(scope="module")
def golden():
    z = np.load(GOLDEN)
    return z, json.loads(str(z["meta"]))


@pytest.fixture(scope="module")
def vfm_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("vfmfullbwd") / fc.VFM_DIRNAME
    d.mkdir()
    json.dump(fc.SIGLIP_L_CFG, open(d / "config.json", "w"))
    return str(d)


def _run(vfm_dir, meta, precision):
    from networks.generator import Generator
    kw = dict(meta["g_kwargs"], vfm_name=vfm_dir)
    if precision == "bf16":
        kw["num_fp16_res"] = 3              # the stage-0 YAML's value: blocks 3-5 in bf16 (amp_dtype)
    G = Generator(label_dim=0, **kw)
    det_init(G)
    G = G.train().requires_grad_(False).to(DEV)
    for name in fc.TRAIN_GROUPS:
        getattr(G, name).requires_grad_(True)
    G.vfm_encoder.encoder.amp_enabled = precision == "bf16"
    img = fc.image()
    assert abs(float(img.double().sum()) - meta["img_sum"]) < 1e-6
    torch.manual_seed(fc.EPS_SEED)
    out = G(img.to(DEV), ["x"], validation=True)
    R, Rs = fc.loss_weights(out.gen_img.shape, [m.shape for m in out.gen_multiscale_imgs])
    loss = (out.gen_img * R.to(DEV)).sum() + sum((m * r.to(DEV)).sum() for m, r in zip(out.gen_multiscale_imgs, Rs)) \
        + fc.VF_W * out.vf_loss + fc.KL_W * out.kl_loss
    loss.backward()
    torch.cuda.synchronize()
    return G, out, loss


# measured worst cases on MI355X (r5p): fp32 norm 4.8e-5, projection 4.6e-5, stored tensors 6.3e-6; bf16
# norm 8.9e-2 (synthesis.blocks.5.convs1.0.noise_strength), projection 1.05e-1
# (ldm_adapter.post_quant.blocks.0.norm3.weight), stored tensors 5.8e-2. Bounds: fp32 2e-4 (4x), bf16 1.5x.
MEASURED_BF16 = dict(norm=8.91e-2, proj=1.05e-1, full=5.79e-2)
FP32_TOL = 2e-4
BF16_NORM_TOL = 1.35e-1
BF16_PROJ_TOL = 1.6e-1


def _rel(a, b):
    return abs(float(a) - float(b)) / max(abs(float(b)), 1e-30)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_generator_training_backward_full_size(vfm_dir, golden, precision):
    z, meta = golden
    G, out, loss = _run(vfm_dir, meta, precision)
    e_loss = _rel(loss, meta["loss"])
    e_vf, e_kl = _rel(out.vf_loss, meta["vf_loss"]), _rel(out.kl_loss, meta["kl_loss"])
    e_img = _rel(out.gen_img.double().norm(), meta["gen_img_norm"])
    e_px = float((out.gen_img.detach().double().cpu() - torch.from_numpy(z["gen_img"]).double()).abs().max())
    print(f"{precision}: loss rel {e_loss:.2e} (vf {e_vf:.2e}, kl {e_kl:.2e}), gen_img norm rel {e_img:.2e}, "
          f"max |pixel err| {e_px:.2e}")
    names, norms, sums, projs = meta["grad_names"], z["grad_norm"], z["grad_sum"], z["grad_proj"]
    params = dict(G.named_parameters())
    got = {n for n, p in params.items() if p.grad is not None}
    assert got == set(names), got ^ set(names)
    floor = (1e-4 if precision == "fp32" else 1e-3) * float(np.max(norms))
    tol_norm = FP32_TOL if precision == "fp32" else BF16_NORM_TOL
    tol_proj = FP32_TOL if precision == "fp32" else BF16_PROJ_TOL
    worst = {"norm": (0.0, None), "proj": (0.0, None), "full": (0.0, None)}
    bad = []
    group_sq = {g: 0.0 for g in fc.TRAIN_GROUPS}
    for n, nm, sm, pj in zip(names, norms, sums, projs):
        gd = params[n].grad.detach().double().cpu()
        group_sq[n.split(".")[0]] += float(gd.square().sum())
        e_norm, e_proj = fc.grad_errors(n, gd, nm, pj, floor)
        for key, e in (("norm", e_norm), ("proj", e_proj)):
            if e > worst[key][0]:
                worst[key] = (e, n)
        scale = max(float(nm), floor, 1e-30)
        e_sum_bad = precision == "fp32" and abs(float(gd.sum()) - float(sm)) > 1e-3 * scale * max(1.0, gd.numel() ** 0.5)
        if e_norm >= tol_norm or e_proj >= tol_proj or e_sum_bad:
            bad.append((n, e_norm, e_proj, float(gd.norm()), float(nm), float(gd.sum()), float(sm)))
    for i, (n, step) in enumerate(meta["full_grads"]):
        e = fc.full_grad_error(params[n].grad, z[f"full_grad{i}"], step)
        if e > worst["full"][0]:
            worst["full"] = (e, f"{n}[::{step}]")
        if e >= tol_proj:
            bad.append((f"{n}[::{step}] (stored tensor)", e, e, 0.0, 0.0, 0.0, 0.0))
    for b in sorted(bad, key=lambda t: -max(t[1], t[2]))[:12]:
        print("  out of tolerance: %s norm err %.2e proj err %.2e (norm %.4e vs %.4e, sum %.4e vs %.4e)" % b)
    g_err = {g: _rel(v ** 0.5, meta["group_norms"][g]) for g, v in group_sq.items()}
    print(f"{precision}: worst gradient errors " + ", ".join(f"{k} {v[0]:.2e} ({v[1]})" for k, v in worst.items())
          + "; group norm rel err " + ", ".join(f"{g} {e:.2e}" for g, e in g_err.items()))
    assert not bad, f"{len(bad)} parameter gradients out of tolerance"
    if precision == "fp32":
        assert e_loss < 1e-5 and e_vf < 1e-5 and e_kl < 1e-5, (e_loss, e_vf, e_kl)
        assert e_px <= 2e-3, e_px
        assert all(e < 1e-3 for e in g_err.values()), g_err
    else:
        assert e_loss < 3e-2, e_loss
        assert all(e < 5e-2 for e in g_err.values()), g_err


# matched precision (bf16 HIP kernels vs the reference's op sequence in torch at the same bf16 schedule), measured
# on MI355X (r6bf): loss 4.4e-3; tensor gradients: difference median 2.0e-2, worst 3.2e-2, norm error median
# 9.5e-4, worst 1.0e-2; the 38 scalar gradients (noise strengths: sums of many cancelling products, and the torch
# side's reductions are not run-to-run deterministic) 1.0e-1 worst over two runs. Bounds ~2x.
MATCHED_BF16 = dict(loss=4.4e-3, diff=3.19e-2, diff_median=1.97e-2, norm=1.00e-2, scalar=1.00e-1)
MATCHED_LOSS_TOL = 1e-2
MATCHED_DIFF_TOL = 6e-2
MATCHED_DIFF_MEDIAN_TOL = 3e-2
MATCHED_NORM_TOL = 2e-2
MATCHED_SCALAR_TOL = 2e-1


def test_generator_backward_bf16_matched_precision(vfm_dir, golden):
    """The bench's precision pinned at matched precision: the bf16 Generator's training backward with the
    decoder's HIP kernels against the same network, same init and same noise draws with every decoder op
    on its torch restatement of the reference (decoder_ops.set_force_ref(True): torch's bf16 convolutions,
    GroupNorm, GELU ... in the dtypes the reference's autocast gives them). Both runs share everything
    else (tower, adapter), so the difference is the decoder kernels' own rounding: each parameter gradient
    compared as a whole tensor, |g_hip - g_torch| / max(|g_torch|, 1e-3 max norm). A systematic error of a
    few percent in one bf16 kernel exceeds the bound, which the fp32-golden comparison above (bf16 noise
    against fp32 numbers: 13.5 %) cannot resolve: tensor gradients within MATCHED_DIFF_TOL = 6e-2 as a
    difference, MATCHED_NORM_TOL = 2e-2 in norm (a systematic scale error of a few percent moves the norm
    by as much, rounding noise moves it by ~1e-3), median difference below 3e-2; scalars within 2e-1."""
    from torch_utils.ops import decoder_ops
    _, meta = golden
    G_hip, out_hip, loss_hip = _run(vfm_dir, meta, "bf16")
    decoder_ops.set_force_ref(True)
    try:
        G_ref, out_ref, loss_ref = _run(vfm_dir, meta, "bf16")
    finally:
        decoder_ops.set_force_ref(False)
    e_loss = _rel(loss_hip, loss_ref)
    ph, pr = dict(G_hip.named_parameters()), dict(G_ref.named_parameters())
    names = [n for n, p in pr.items() if p.grad is not None]
    assert names and {n for n, p in ph.items() if p.grad is not None} == set(names)
    floor = 1e-3 * max(float(pr[n].grad.double().norm()) for n in names)
    rows = []            # (difference error, norm error, name, numel)
    for n in names:
        gh, gr = ph[n].grad.double(), pr[n].grad.double()
        scale = max(float(gr.norm()), floor)
        rows.append((float((gh - gr).norm()) / scale, abs(float(gh.norm()) - float(gr.norm())) / scale, n, gr.numel()))
    e_px = float((out_hip.gen_img.double() - out_ref.gen_img.double()).abs().max())
    print(f"matched bf16: loss rel {e_loss:.2e}, max |pixel diff| {e_px:.2e}")
    for label, sel in (("tensors", [r for r in rows if r[3] > 1]), ("scalars", [r for r in rows if r[3] == 1])):
        if not sel:
            continue
        by_diff = sorted(sel, reverse=True)
        by_norm = sorted(sel, key=lambda r: -r[1])
        print(f"matched bf16 {label} ({len(sel)}): difference median {by_diff[len(sel) // 2][0]:.2e}, worst "
              + ", ".join(f"{r[2]} {r[0]:.2e}" for r in by_diff[:5]))
        print(f"matched bf16 {label}: norm error median {by_norm[len(sel) // 2][1]:.2e}, worst "
              + ", ".join(f"{r[2]} {r[1]:.2e}" for r in by_norm[:5]))
    assert e_loss < MATCHED_LOSS_TOL, e_loss
    tens = [r for r in rows if r[3] > 1]
    bad = [(n, e, en) for e, en, n, k in rows
           if (k > 1 and (e >= MATCHED_DIFF_TOL or en >= MATCHED_NORM_TOL)) or (k == 1 and e >= MATCHED_SCALAR_TOL)]
    assert not bad, bad[:10]
    assert sorted(r[0] for r in tens)[len(tens) // 2] < MATCHED_DIFF_MEDIAN_TOL
