"""Diagnostics 3: which module of the captured D-phase generator forward first produces NaN
after an in-place parameter update."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch

from test_configs_gpu import _build, _images

B = int(os.environ.get("B", "4"))
c, step = _build("vfm_vae_f16d32_siglip2_stage_0_synthetic.yaml", batch=B, graphs=True)
G = step.G
G.vfm_encoder.reuse_features = False
eqt = G.equivariance_transform
forced = (1.0, 0, False)
eqt.forced = forced
eqt.outcomes = lambda: [forced]
img, labels = _images(B, 256), ['a photo'] * B
gr = step.loss.graphed_nograd

order = []
acts = {}
capturing = {"on": False}


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


for n, m in G.named_modules():
    if n and not n.startswith("vfm_encoder"):
        m.register_forward_hook(hook(n))

with torch.no_grad():
    torch.manual_seed(7)
    gr(img, labels)
print("captured activations:", len(order), flush=True)


def scan(tag):
    with torch.no_grad():
        torch.manual_seed(7)
        gr(img, labels)
    torch.cuda.synchronize()
    bad = [n for n in order if not torch.isfinite(acts[n].float()).all()]
    print(f"[{tag}] non-finite activations: {len(bad)}; first: {bad[:5]}", flush=True)


scan("fresh")
for name, p in G.synthesis.named_parameters():
    with torch.no_grad():
        p.add_(1e-3 * torch.randn_like(p))
    with torch.no_grad():
        torch.manual_seed(7)
        gr(img, labels)
    torch.cuda.synchronize()
    bad = [n for n in order if not torch.isfinite(acts[n].float()).all()]
    if bad:
        print(f"perturbing synthesis.{name} -> first non-finite: {bad[:3]}", flush=True)
        break
else:
    print("no parameter broke the replay", flush=True)
