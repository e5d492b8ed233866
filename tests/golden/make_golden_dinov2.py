"""DINOv2-L golden vectors (BASELINE config 3's encoder), generated FROM THE REFERENCE ITSELF.

Runs only in the build container (CPU, fp32): imports /root/reference with the small third-party stand-ins of
tests/golden/ref_stubs (torchvision's `normalize` only), saves a random-init HF `transformers.Dinov2Model` of the
DINOv2-L architecture (24 x 1024, 16 heads, patch 14, 518^2 position grid) to a local directory, builds the
reference's `networks.utils.vfms.dinov2_utils.DINOv2Encoder` on it (AutoModel.from_pretrained of that directory),
overwrites every weight with tests/det_init.py (values depend only on the state-dict name and shape, so the GPU
test rebuilds the same tower without shipping 1.2 GB of weights) and runs `encode_image` with the C3 YAML's
settings (scale_factor 0.875, patch_from_layers [0, 12, -1]) on
  * 256^2, 384^2 and 512^2 inputs (16 / 24 / 32 patches a side: the dynamic-resolution stream), and
  * a 256^2 input with the equivariance prior's bicubic downscale (eq_scale_factor 0.5, is_eq_prior=True).
Stored per case and hidden state: every 16th patch token (all 1024 channels), the per-token L2 norms over all
tokens, and the pooled CLS output. The inputs are regenerated from their seeds on both sides.

The reference pins transformers 4.50.1 (requirements.txt:25); this container has 5.15.0, whose Dinov2Layer /
interpolate_pos_encoding are what the vectors come from (parity is pinned to that version).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_dinov2.py
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
from transformers import Dinov2Config, Dinov2Model  # noqa: E402

sys.path.insert(0, os.path.dirname(HERE))           # tests/ (det_init, dinov2_case)
sys.path.insert(0, os.path.join(HERE, "ref_stubs"))
sys.path.insert(0, REF)

from det_init import det_init  # noqa: E402
import dinov2_case as dc  # noqa: E402

OUT = os.path.join(HERE, "dinov2_golden.npz")
torch.set_num_threads(int(os.environ.get("THREADS", "8")))
arrays, meta = {}, {"cases": [], "transformers": transformers.__version__}


def put(k, v):
    arrays[k] = v.detach().cpu().float().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)


work = tempfile.mkdtemp(prefix="vfm_golden_dinov2_")
vfm_dir = os.path.join(work, dc.VFM_DIRNAME)
torch.manual_seed(0)
Dinov2Model(Dinov2Config(**dc.DINOV2_L_CFG)).save_pretrained(vfm_dir)

from networks.utils.vfms.dinov2_utils import DINOv2Encoder  # noqa: E402

enc = DINOv2Encoder(model_name=vfm_dir, scale_factor=dc.SCALE_FACTOR, patch_from_layers=list(dc.LAYERS),
                    amp_enabled=False)
touched = det_init(enc.vision_model)
meta["det_init_tensors"] = len(touched)
enc.eval()
with torch.no_grad():
    for case in dc.CASES:
        name, res, eqs, prior = case["name"], case["res"], case["eq_scale"], case["prior"]
        img = dc.image(res, case["seed"])
        meta[f"{name}/img_sum"] = float(img.double().sum())
        feats, pooled = enc.encode_image(img, eqs, prior)
        for hname, f in zip(dc.HIDDEN_NAMES, feats):
            put(f"{name}/{hname}/rows", f[0, ::dc.ROW_STRIDE])
            put(f"{name}/{hname}/norms", f[0].double().norm(dim=-1))
            meta[f"{name}/{hname}/shape"] = list(f.shape)
        put(f"{name}/pooled", pooled[0])
        meta["cases"].append(name)
        print(name, [tuple(f.shape) for f in feats], flush=True)
np.savez_compressed(OUT, meta=json.dumps(meta), **arrays)
print("wrote", OUT, os.path.getsize(OUT), "bytes")
