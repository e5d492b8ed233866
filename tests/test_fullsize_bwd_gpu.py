"""Full-size parity of the TRAINING backward on cuda:0 against vectors generated from the reference
itself (tests/golden/make_golden_fullsize_bwd.py): the f16d32 stage-0 Generator on the full SigLIP2-L
tower at 256^2, batch 1, KL / VF losses on, posterior noise from the CPU generator as the reference
draws it, and loss = sum(gen_img R) + sum_i sum(ms_i R_i) + 3 vf + 1e-3 kl back-propagated into the
groups the G phase trains (synthesis, mapping, ldm_adapter; reference networks/generator.py:1152-1206,
training/loss.py:721-1001). The reference side is fp32 (CPU).

Stated tolerances:
  fp32 -- the product path at reference precision (decoder num_fp16_res 0, fp32 tower; our kernels
  with fp32-equivalent f32x6 products): the 64-px golden's tolerances -- loss terms 1e-5 relative,
  every parameter's gradient norm within 1e-3 and sum within 1e-3 (scaled, with a floor at 1e-4 of
  the largest norm for gradients that are ~0 in exact math), group norms within 1e-3;
  bf16 -- the bench's precision (decoder blocks 3-5 and the SigLIP2 tower in bf16, BASELINE config 1)
  against the same fp32 numbers: loss within 3e-2, group gradient norms within 5e-2, every
  parameter's gradient norm within 2e-1 of its own size (floor 1e-3 of the largest), i.e. bf16
  rounding noise (2^-8 per op over ~60 ops of depth) but no layout / indexing error, which shows up
  as O(1).
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
    names, norms, sums = meta["grad_names"], z["grad_norm"], z["grad_sum"]
    params = dict(G.named_parameters())
    got = {n for n, p in params.items() if p.grad is not None}
    assert got == set(names), got ^ set(names)
    floor = (1e-4 if precision == "fp32" else 1e-3) * float(np.max(norms))
    worst, worst_name, bad = 0.0, None, []
    group_sq = {g: 0.0 for g in fc.TRAIN_GROUPS}
    for n, nm, sm in zip(names, norms, sums):
        gd = params[n].grad.detach().double()
        group_sq[n.split(".")[0]] += float(gd.square().sum())
        scale = max(float(nm), floor, 1e-30)
        err = abs(float(gd.norm()) - float(nm)) / scale
        if err > worst:
            worst, worst_name = err, n
        if precision == "fp32":
            if err >= 1e-3 or abs(float(gd.sum()) - float(sm)) > 1e-3 * scale * max(1.0, gd.numel() ** 0.5):
                bad.append((n, err, float(gd.norm()), float(nm), float(gd.sum()), float(sm)))
        elif err >= 2e-1:
            bad.append((n, err, float(gd.norm()), float(nm), float(gd.sum()), float(sm)))
    for b in sorted(bad, key=lambda t: -t[1])[:12]:
        print("  out of tolerance: %s norm rel err %.2e (norm %.4e vs %.4e, sum %.4e vs %.4e)" % b)
    assert not bad, f"{len(bad)} parameter gradients out of tolerance"
    g_err = {g: _rel(v ** 0.5, meta["group_norms"][g]) for g, v in group_sq.items()}
    print(f"{precision}: worst parameter gradient norm rel err {worst:.2e} ({worst_name}); group norm rel err "
          + ", ".join(f"{g} {e:.2e}" for g, e in g_err.items()))
    if precision == "fp32":
        assert e_loss < 1e-5 and e_vf < 1e-5 and e_kl < 1e-5, (e_loss, e_vf, e_kl)
        assert e_px <= 2e-3, e_px
        assert all(e < 1e-3 for e in g_err.values()), g_err
    else:
        assert e_loss < 3e-2, e_loss
        assert all(e < 5e-2 for e in g_err.values()), g_err
