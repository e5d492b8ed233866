"""Diagnostics 4: replay, eager, in-place weight change, replay -> where does it break?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch

from test_configs_gpu import _build, _images

B = int(os.environ.get("B", "4"))
HOOKS = os.environ.get("HOOKS", "1") == "1"
c, step = _build("vfm_vae_f16d32_siglip2_stage_0_synthetic.yaml", batch=B, graphs=True)
G = step.G
G.vfm_encoder.reuse_features = False
eqt = G.equivariance_transform
forced = (1.0, 0, False)
eqt.forced = forced
eqt.outcomes = lambda: [forced]
img, labels = _images(B, 256), ['a photo'] * B
gr = step.loss.graphed_nograd
order, acts = [], {}


def hook(name):
    def fn(mod, inp, out):
        if not torch.cuda.is_current_stream_capturing():
            return
        t = out if isinstance(out, torch.Tensor) else (out[0] if isinstance(out, (tuple, list)) and out and
                                                      isinstance(out[0], torch.Tensor) else None)
        if t is not None:
            order.append(name)
            acts[name] = t
    return fn


if HOOKS:
    for n, m in G.named_modules():
        if n and not n.startswith("vfm_encoder"):
            m.register_forward_hook(hook(n))


def rep():
    with torch.no_grad():
        torch.manual_seed(7)
        o = gr(img, labels).gen_img.float().clone()
    torch.cuda.synchronize()
    bad = [n for n in order if not torch.isfinite(acts[n].float()).all()]
    return o, bad


def eag():
    with torch.no_grad():
        torch.manual_seed(7)
        return G(img, labels).gen_img.float().clone()


o, bad = rep()
e = eag()
print(f"HOOKS={HOOKS} fresh: rep-eag {float((o - e).abs().max()):.3e} bad {bad[:3]}", flush=True)
o, bad = rep()
print(f"replay after eager: finite {bool(torch.isfinite(o).all())} bad {bad[:3]}", flush=True)
for tag, mods in [("synthesis", G.synthesis), ("mapping", G.mapping), ("ldm_adapter", G.ldm_adapter)]:
    e = eag()
    with torch.no_grad():
        for p in mods.parameters():
            p.add_(1e-3 * torch.randn_like(p))
    o, bad = rep()
    e2 = eag()
    print(f"perturb {tag}: replay finite {bool(torch.isfinite(o).all())} first bad {bad[:4]} | rep-eag "
          f"{float((o - e2).abs().max()):.3e}", flush=True)
    o, bad = rep()
    print(f"   second replay finite {bool(torch.isfinite(o).all())} rep-eag {float((o - e2).abs().max()):.3e}",
          flush=True)
