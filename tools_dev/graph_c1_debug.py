"""Diagnostics: D-phase graph replay vs eager generator forward at the full C1 config,
at each stage of one training iteration (fresh, after D phase, after G phase, after step)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch

from test_configs_gpu import _build, _images

reuse = os.environ.get("REUSE", "1") == "1"
B = int(os.environ.get("B", "32"))
c, step = _build("vfm_vae_f16d32_siglip2_stage_0_synthetic.yaml", batch=B, graphs=True)
G = step.G
G.vfm_encoder.reuse_features = reuse
eqt = G.equivariance_transform
forced = (1.0, 0, False)
eqt.forced = forced
eqt.outcomes = lambda: [forced]
img, labels = _images(B, 256), ['a photo'] * B
gr = step.loss.graphed_nograd


def compare(tag):
    with torch.no_grad():
        torch.manual_seed(7)
        rep = gr(img, labels).gen_img.float().clone()
        torch.manual_seed(7)
        eag = G(img, labels).gen_img.float().clone()
        torch.manual_seed(7)
        eag2 = G(img, labels).gen_img.float().clone()
    e = float((rep - eag).abs().max() / eag.abs().max())
    e2 = float((eag2 - eag).abs().max() / eag.abs().max())
    print(f"[{tag}] replay-vs-eager {e:.3e}  eager-vs-eager {e2:.3e}  max rep {float(rep.abs().max()):.3f} "
          f"eag {float(eag.abs().max()):.3f} nan rep {int(rep.isnan().sum())} eag {int(eag.isnan().sum())}", flush=True)


compare("fresh")
dph, gph = step.phases
step._apply_freeze(dph)
dph.sync.prepare()
step.loss.accumulate_gradients(phase='D', real_img=img, real_c=labels, cur_nimg=0)
dph.module.requires_grad_(False)
dph.sync.finish(gain=1)
compare("after D accumulate")
dph.opt.step()
dph.opt.zero_grad(set_to_none=True)
step._apply_freeze(gph)
gph.sync.prepare()
step.loss.accumulate_gradients(phase='G', real_img=img, real_c=labels, cur_nimg=0)
gph.module.requires_grad_(False)
gph.sync.finish(gain=1)
print("reuse hits", getattr(G.vfm_encoder, "reuse_hits", 0))
compare("after G accumulate")
gph.opt.step()
gph.opt.zero_grad(set_to_none=True)
compare("after G step")
