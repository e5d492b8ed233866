"""Full-size golden vectors for the TRAINING backward, generated FROM THE REFERENCE ITSELF.

Runs only in the build container (CPU, fp32): imports /root/reference with the stand-ins of
tests/golden/ref_stubs (as make_golden_fullsize.py), builds the full f16d32 stage-0 Generator
(configs/vfm_vae_f16d32_siglip2_stage_0_strong_alignment.yaml G_kwargs plus the use_* flags reference
train.py:76-96 derives from loss_kwargs -- KL and VF losses on -- img_resolution 256, unconditional) on the full SigLIP2-L tower, overwrites every
weight with tests/det_init.py, and runs one 256^2 image through Generator.forward(validation=True)
in train mode (reference networks/generator.py:1152-1206; the equivariance draw is off under
validation) with the posterior noise drawn from the CPU generator seeded 123. The scalar

    loss = sum(gen_img * R) + sum_i sum(ms_i * R_i) + 3 vf_loss + 1e-3 kl_loss

(R, R_i: standard normal from a seeded CPU generator, regenerated on the GPU side; the same form as
tests/golden/make_golden_networks.py's 64-px case, with a KL weight that keeps the three terms of similar size) is back-propagated into the trainable groups the
reference's G phase updates -- synthesis, mapping, ldm_adapter (the VFM tower is frozen; reference
training/loss.py:721-1001 accumulate_gradients and networks/generator.py set_train_mode). Stored:
the loss terms, the per-parameter gradient norms, sums and NPROJ projections <g, P_k> on seeded
random P_k (tests/fullsize_case.py grad_probe: sensitive to a transposed or permuted gradient, which keeps norm
and sum), whole (or row-subsampled) gradients of the weights in fullsize_case.FULL_GRADS, per-group
gradient norms, and per-image sums / norms of the outputs. The decoder runs in fp32 here (num_fp16_res 0: the CPU reference has no
fp16 path); the GPU test compares both its fp32 product path and the bench's precision (bf16 blocks
3-5, bf16 tower) against these fp32 numbers with stated tolerances.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_fullsize_bwd.py
"""
import json
import os
import sys
import tempfile

import numpy as np
import torch
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("VFM_REFERENCE", "/root/reference")
import transformers  # noqa: E402,F401  (import before the stubs: keeps its torchvision probe negative)
from transformers import SiglipVisionConfig, SiglipVisionModel  # noqa: E402

sys.path.insert(0, os.path.dirname(HERE))           # tests/ (det_init, fullsize_case)
sys.path.insert(0, os.path.join(HERE, "ref_stubs"))
sys.path.insert(0, REF)

from det_init import det_init  # noqa: E402
import fullsize_case as fc  # noqa: E402

OUT = os.path.join(HERE, "fullsize_bwd_golden.npz")
torch.set_num_threads(int(os.environ.get("THREADS", "8")))
arrays, meta = {}, {}

work = tempfile.mkdtemp(prefix="vfm_golden_fullbwd_")
vfm_dir = os.path.join(work, fc.VFM_DIRNAME)
torch.manual_seed(0)
SiglipVisionModel(SiglipVisionConfig(**fc.SIGLIP_L_CFG)).save_pretrained(vfm_dir)

cfg = yaml.safe_load(open(os.path.join(REF, "configs", fc.REF_YAML)))
g_kwargs, loss_kwargs = cfg["G_kwargs"], cfg["loss_kwargs"]
g_kwargs.pop("class_name")
# the G_kwargs reference train.py:76-96 derives from loss_kwargs for training (KL / VF losses on, adaptive
# VF weight, equivariance regulariser, multiscale outputs)
g_kwargs.setdefault("use_kl_loss", loss_kwargs.get("kl_loss_weight", 0.0) > 0.0)
g_kwargs.setdefault("use_vf_loss", loss_kwargs.get("vf_loss_weight", 0.0) > 0.0)
g_kwargs.setdefault("use_adaptive_vf_loss", loss_kwargs.get("use_adaptive_vf_loss", False))
g_kwargs.setdefault("use_equivariance_regularization", loss_kwargs.get("use_equivariance_regularization", False))
g_kwargs.setdefault("use_multiscale_output", len(loss_kwargs.get("multiscale_block_indices", [])) > 0)
g_kwargs.update(fc.TRAIN_OVERRIDES, vfm_name=vfm_dir)

from networks.generator import Generator  # noqa: E402

G = Generator(label_dim=0, **g_kwargs)
det_init(G)
G.train().requires_grad_(False)
for name in fc.TRAIN_GROUPS:
    getattr(G, name).requires_grad_(True)
img = fc.image()
meta["img_sum"] = float(img.double().sum())
torch.manual_seed(fc.EPS_SEED)
out = G(img, ["x"], validation=True)
R, Rs = fc.loss_weights(out.gen_img.shape, [m.shape for m in out.gen_multiscale_imgs])
loss = (out.gen_img * R).sum() + sum((m * r).sum() for m, r in zip(out.gen_multiscale_imgs, Rs)) \
    + fc.VF_W * out.vf_loss + fc.KL_W * out.kl_loss
assert float(out.vf_loss) != 0.0 and float(out.kl_loss) != 0.0, "KL / VF losses are off"
meta["loss"] = float(loss)
meta["vf_loss"] = float(out.vf_loss)
meta["kl_loss"] = float(out.kl_loss)
meta["gen_img_sum"] = float(out.gen_img.double().sum())
meta["gen_img_norm"] = float(out.gen_img.double().norm())
meta["ms_sums"] = [float(m.double().sum()) for m in out.gen_multiscale_imgs]
meta["ms_norms"] = [float(m.double().norm()) for m in out.gen_multiscale_imgs]
arrays["gen_img"] = out.gen_img.detach().float().numpy()
loss.backward()
names, norms, sums, projs = [], [], [], []
group_sq = {g: 0.0 for g in fc.TRAIN_GROUPS}
for n, p in G.named_parameters():
    if p.grad is None:
        continue
    gd = p.grad.detach().double()
    names.append(n)
    norms.append(float(gd.norm()))
    sums.append(float(gd.sum()))
    projs.append(fc.projections(n, gd).numpy())
    group_sq[n.split(".")[0]] += float(gd.square().sum())
meta["grad_names"] = names
meta["group_norms"] = {g: v ** 0.5 for g, v in group_sq.items()}
arrays["grad_norm"] = np.asarray(norms, np.float64)
arrays["grad_sum"] = np.asarray(sums, np.float64)
arrays["grad_proj"] = np.stack(projs).astype(np.float64)          # [n_params, NPROJ]
params = dict(G.named_parameters())
meta["full_grads"] = []
for i, (n, step) in enumerate(fc.FULL_GRADS):
    arrays[f"full_grad{i}"] = params[n].grad.detach()[::step].float().numpy()
    meta["full_grads"].append([n, step])
meta["g_kwargs"] = {k: v for k, v in g_kwargs.items() if k != "vfm_name"}
arrays["meta"] = np.array(json.dumps(meta))
np.savez_compressed(OUT, **arrays)
print(f"wrote {OUT}: {len(names)} parameter gradients, loss {meta['loss']:.6e}, group norms {meta['group_norms']}, "
      f"{os.path.getsize(OUT) / 1024:.1f} KiB")
