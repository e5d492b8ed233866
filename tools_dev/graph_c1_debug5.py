"""Diagnostics 5: does a library scratch buffer leak between eager calls and the captured graph?
Toggle candidate libraries off and check replay == eager after an in-place weight change."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch

if os.environ.get("NO_CUDNN") == "1":
    torch.backends.cudnn.enabled = False
if os.environ.get("SDPA_MATH") == "1":
    torch.backends.cuda.enable_flash_sdp(False)
    torch.backends.cuda.enable_mem_efficient_sdp(False)
from test_configs_gpu import _build, _images

B = int(os.environ.get("B", "4"))
PART = os.environ.get("PART", "synthesis")
c, step = _build("vfm_vae_f16d32_siglip2_stage_0_synthetic.yaml", batch=B, graphs=True)
G = step.G
G.vfm_encoder.reuse_features = False
eqt = G.equivariance_transform
forced = (1.0, 0, False)
eqt.forced = forced
eqt.outcomes = lambda: [forced]
img, labels = _images(B, 256), ['a photo'] * B
gr = step.loss.graphed_nograd


def rep():
    with torch.no_grad():
        torch.manual_seed(7)
        return gr(img, labels).gen_img.float().clone()


def eag():
    with torch.no_grad():
        torch.manual_seed(7)
        return G(img, labels).gen_img.float().clone()


o = rep()
e = eag()
mod = dict(G.named_children())[PART] if PART != "synthesis.b0" else G.synthesis.blocks[0]
with torch.no_grad():
    for p in mod.parameters():
        p.add_(1e-3 * torch.randn_like(p))
o1 = rep()
e2 = eag()
o2 = rep()
print(f"flags CAST_CACHE_OFF={os.environ.get('VFM_NO_CAST_CACHE')} NO_CUDNN={os.environ.get('NO_CUDNN')} SDPA_MATH={os.environ.get('SDPA_MATH')} PART={PART}: "
      f"rep1-eag {float((o1 - e2).abs().max()):.3e} rep2-eag {float((o2 - e2).abs().max()):.3e} "
      f"finite {bool(torch.isfinite(o1).all())} {bool(torch.isfinite(o2).all())}", flush=True)
