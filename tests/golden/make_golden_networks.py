"""Golden vectors for the network/loss layers, generated FROM THE REFERENCE ITSELF.

Runs only in the build container: imports /root/reference (with the small
third-party stand-ins of tests/golden/ref_stubs) on CPU in fp32, builds a tiny
but complete configuration (random SigLIP2 tower 2 x 128, full 6-block
ConvNeXt decoder at 64 px, StyleGAN-T D + PatchGAN, LPIPS, stage-0 loss mix),
overwrites every weight with tests/det_init.py, runs forward/backward and one
D + G `accumulate_gradients`, and writes tests/golden/networks_golden.npz.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_networks.py
"""
import json
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("VFM_REFERENCE", "/root/reference")
import transformers  # noqa: E402,F401  (import before the stubs: keeps its torchvision probe negative)
from transformers import SiglipVisionConfig, SiglipVisionModel  # noqa: E402

sys.path.insert(0, os.path.dirname(HERE))           # tests/ (det_init, net_cases)
sys.path.insert(0, os.path.join(HERE, "ref_stubs"))
sys.path.insert(0, REF)

from det_init import det_init  # noqa: E402
import net_cases  # noqa: E402

OUT = os.path.join(HERE, "networks_golden.npz")
torch.set_grad_enabled(True)
arrays = {}
meta = {}


def put(k, v):
    arrays[k] = v.detach().cpu().float().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)


def grad_stats(prefix, module):
    names, sums, norms = [], [], []
    for n, p in module.named_parameters():
        if p.grad is None:
            continue
        names.append(n)
        sums.append(float(p.grad.double().sum()))
        norms.append(float(p.grad.double().norm()))
        if p.numel() <= 1024:
            put(f"{prefix}/grad/{n}", p.grad)
    arrays[f"{prefix}/grad_sum"] = np.array(sums)
    arrays[f"{prefix}/grad_norm"] = np.array(norms)
    meta[f"{prefix}/grad_names"] = names


work = tempfile.mkdtemp(prefix="vfm_golden_")
vfm_dir = os.path.join(work, net_cases.VFM_DIRNAME)
cfg = SiglipVisionConfig(**net_cases.SIGLIP_CFG)
torch.manual_seed(0)
SiglipVisionModel(cfg).save_pretrained(vfm_dir)

# LPIPS loads `taming/modules/autoencoder/lpips/vgg.pth` relative to cwd (lpips.py:80-82).
os.chdir(work)
os.makedirs("taming/modules/autoencoder/lpips", exist_ok=True)
torch.save({f"lin{i}.model.1.weight": torch.rand(1, c, 1, 1) for i, c in enumerate([64, 128, 256, 512, 512])},
           "taming/modules/autoencoder/lpips/vgg.pth")

from networks.generator import Generator  # noqa: E402
from networks.discriminator import ProjectedDiscriminator  # noqa: E402
from training.lpips import LPIPS  # noqa: E402
from training.loss import TotalLoss  # noqa: E402

# ------------------------------------------------------------ Generator fwd/bwd
G = Generator(label_dim=0, **net_cases.g_kwargs(vfm_dir)).train()
det_init(G)
meta["G_state_keys"] = sorted(G.state_dict().keys())
g = torch.Generator().manual_seed(11)
img = torch.rand(2, 3, 64, 64, generator=g)
put("G/img", img)
G.requires_grad_(False)
G.synthesis.requires_grad_(True)
G.mapping.requires_grad_(True)
G.ldm_adapter.requires_grad_(True)
torch.manual_seed(123)                   # epsilon of DiagonalGaussianDistribution.sample (CPU randn)
out = G(img, ['x'] * 2, validation=True)
put("G/gen_img", out.gen_img)
for i, m in enumerate(out.gen_multiscale_imgs):
    put(f"G/ms{i}", m)
put("G/vf_loss", out.vf_loss)
put("G/kl_loss", out.kl_loss)
R = torch.randn(out.gen_img.shape, generator=g)
Rs = [torch.randn(m.shape, generator=g) for m in out.gen_multiscale_imgs]
put("G/R", R)
for i, r in enumerate(Rs):
    put(f"G/R{i}", r)
loss = (out.gen_img * R).sum() + sum((m * r).sum() for m, r in zip(out.gen_multiscale_imgs, Rs)) \
    + 3.0 * out.vf_loss + 1e3 * out.kl_loss
loss.backward()
grad_stats("G", G)
meta["G_num_ws"] = G.num_ws

# ------------------------------------------------------------ Discriminator
D = ProjectedDiscriminator(c_dim=0, **net_cases.D_KWARGS).train()
det_init(D)
meta["D_state_keys"] = sorted(D.state_dict().keys())
xd = (torch.rand(2, 3, 64, 64, generator=g) * 2 - 1).requires_grad_(True)
put("D/x", xd)
dout = D(xd, None)
put("D/logits", dout.stylegan_t_logits)
for s, scale in enumerate(dout.patchgan_logits):
    put(f"D/patch{s}", scale[-1])
    meta[f"D/patch{s}_feat_sums"] = [float(t.double().sum()) for t in scale]
Rd = torch.randn(dout.stylegan_t_logits.shape, generator=g)
put("D/R", Rd)
dl = (dout.stylegan_t_logits * Rd).sum() + sum(s[-1].square().mean() for s in dout.patchgan_logits)
dl.backward()
put("D/dx", xd.grad)
grad_stats("D", D)
for n, b in D.named_buffers():
    if n.endswith("weight_u"):
        put(f"D/buf/{n}", b)        # power-iteration state after one train-mode forward

# ------------------------------------------------------------ LPIPS
L = LPIPS().eval()
det_init(L)
a = torch.rand(2, 3, 64, 64, generator=g) * 2 - 1
b = (torch.rand(2, 3, 64, 64, generator=g) * 2 - 1).requires_grad_(True)
put("L/a", a)
put("L/b", b)
v = L(a, b)
put("L/val", v)
v.sum().backward()
put("L/db", b.grad)

# ------------------------------------------------------------ TotalLoss: one D + one G step
torch.manual_seed(5)
G2 = Generator(label_dim=0, **net_cases.g_kwargs(vfm_dir)).train().requires_grad_(False)
D2 = ProjectedDiscriminator(c_dim=0, **net_cases.D_KWARGS).train().requires_grad_(False)
det_init(G2)
det_init(D2)
loss_obj = TotalLoss(device=torch.device('cpu'), G=G2, D=D2, **net_cases.loss_kwargs(vfm_dir))
det_init(loss_obj.perceptual_module)
real = torch.rand(2, 3, 64, 64, generator=g)
put("T/real", real)
cur_nimg = 0
D2.requires_grad_(True)
D2.dino.requires_grad_(False)
torch.manual_seed(321)
loss_obj.accumulate_gradients(phase='D', real_img=real, real_c=['x'] * 2, cur_nimg=cur_nimg)
D2.requires_grad_(False)
grad_stats("T/D", D2)
G2.requires_grad_(False)
for name, layer in G2.named_modules():
    layer.requires_grad_(any(t in name for t in G2.trainable_layers))
torch.manual_seed(654)
loss_obj.accumulate_gradients(phase='G', real_img=real, real_c=['x'] * 2, cur_nimg=cur_nimg)
grad_stats("T/G", G2)
meta["T/prev_loss_dict"] = loss_obj.prev_loss_dict

arrays["meta"] = np.array(json.dumps(meta))
np.savez_compressed(OUT, **arrays)
print(f"wrote {OUT}: {len(arrays)} arrays, {os.path.getsize(OUT) / 1024:.1f} KiB")
