"""Diagnostics 2: is the D-phase graph replay reading memory it does not own, or stale weights?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT, os.path.join(ROOT, "tests")]
import torch

from test_configs_gpu import _build, _images
from torch_utils.ops import decoder_hip

B = int(os.environ.get("B", "8"))
c, step = _build("vfm_vae_f16d32_siglip2_stage_0_synthetic.yaml", batch=B, graphs=True)
G = step.G
G.vfm_encoder.reuse_features = os.environ.get("REUSE", "0") == "1"
eqt = G.equivariance_transform
forced = (1.0, 0, False)
eqt.forced = forced
eqt.outcomes = lambda: [forced]
img, labels = _images(B, 256), ['a photo'] * B
gr = step.loss.graphed_nograd

hits = {"capture_hit": 0, "capture_calls": 0}
orig = decoder_hip._cast_cached


def spy(w, dtype):
    if torch.cuda.is_current_stream_capturing():
        hits["capture_calls"] += 1
    return orig(w, dtype)


decoder_hip._cast_cached = spy


def compare(tag):
    with torch.no_grad():
        torch.manual_seed(7)
        rep = gr(img, labels).gen_img.float().clone()
        torch.manual_seed(7)
        eag = G(img, labels).gen_img.float().clone()
    e = float((rep - eag).abs().max() / eag.abs().max())
    print(f"[{tag}] replay-vs-eager {e:.3e} max rep {float(rep.abs().max()):.3f} eag {float(eag.abs().max()):.3f} "
          f"nan rep {int(rep.isnan().sum())}", flush=True)


compare("fresh")
print("casts under capture:", hits, flush=True)
junk = [torch.full((64 << 20,), float("nan"), device="cuda") for _ in range(16)]
del junk
torch.cuda.synchronize()
compare("after NaN fill of freed memory")
torch.cuda.empty_cache()
junk = [torch.full((64 << 20,), float("nan"), device="cuda") for _ in range(16)]
del junk
compare("after empty_cache + NaN fill")
with torch.no_grad():
    for p in G.synthesis.parameters():
        p.add_(1e-3 * torch.randn_like(p))
compare("after in-place param perturbation (synthesis)")
with torch.no_grad():
    for p in G.ldm_adapter.parameters():
        p.add_(1e-3 * torch.randn_like(p))
compare("after in-place param perturbation (adapter)")
with torch.no_grad():
    for p in G.mapping.parameters():
        p.add_(1e-3 * torch.randn_like(p))
compare("after in-place param perturbation (mapping)")
params = [p for p in G.parameters() if p.dtype == torch.float32 and p.requires_grad is False]
opt = torch.optim.Adam([p for n, p in G.named_parameters() if not n.startswith("vfm_encoder")], lr=1e-4,
                       betas=(0.0, 0.99), fused=True)
for n, p in G.named_parameters():
    if not n.startswith("vfm_encoder"):
        p.grad = torch.randn_like(p)
opt.step()
compare("after fused Adam step")
