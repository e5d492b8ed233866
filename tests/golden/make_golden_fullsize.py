"""Full-size golden vectors for the continuous path, generated FROM THE REFERENCE ITSELF.

Runs only in the build container (CPU, fp32): imports /root/reference with the small
third-party stand-ins of tests/golden/ref_stubs, builds
  * the full SigLIP2-L tower (24 x 1024, 16 heads, patch 16, 512^2 input) as
    transformers.SiglipVisionModel, and
  * the full f16d32 stage-0 Generator on top of it (configs/vfm_vae_f16d32_siglip2_stage_0_
    strong_alignment.yaml G_kwargs) with the settings tools/reconstruct/reconstruct.py:106-113
    uses for reconstructions (img_resolution 256, unconditional, num_fp16_res 0, no KL / VF loss),
overwrites every weight with tests/det_init.py (values depend only on the state-dict name and
shape, so the GPU tests rebuild the same network without shipping 1.3 GB of weights), and runs
one 256^2 image through
  * SigLIP2Encoder.encode_image (reference networks/utils/vfms/siglip2_utils.py:94-137): the
    patch features hidden_states[0], hidden_states[12] and last_hidden_state, and
  * Generator.forward(validation=True) (reference networks/generator.py:1152-1206) with the
    posterior noise drawn from the CPU generator seeded 123 (the reference's own draw).
The input image is regenerated from its seed on both sides (its checksum is stored). Stored:
every 16th token (64 x 1024) of each hidden state plus per-token L2 norms over all 1024 tokens,
the latent moments (mean || logvar) and the full reconstructed image.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_fullsize.py
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

OUT = os.path.join(HERE, "fullsize_golden.npz")
torch.set_num_threads(int(os.environ.get("THREADS", "8")))
arrays, meta = {}, {}


def put(k, v):
    arrays[k] = v.detach().cpu().float().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)


work = tempfile.mkdtemp(prefix="vfm_golden_full_")
vfm_dir = os.path.join(work, fc.VFM_DIRNAME)
torch.manual_seed(0)
SiglipVisionModel(SiglipVisionConfig(**fc.SIGLIP_L_CFG)).save_pretrained(vfm_dir)

g_kwargs = yaml.safe_load(open(os.path.join(REF, "configs", fc.REF_YAML)))["G_kwargs"]
g_kwargs.pop("class_name")
g_kwargs.update(fc.RECON_OVERRIDES, vfm_name=vfm_dir)

from networks.generator import Generator  # noqa: E402

G = Generator(label_dim=0, **g_kwargs)
det_init(G)
G.eval().requires_grad_(False)
img = fc.image()
meta["img_sum"] = float(img.double().sum())
with torch.no_grad():
    feats, _ = G.vfm_encoder.encode_image(img)
    for name, f in zip(fc.HIDDEN_NAMES, feats):
        put(f"S/{name}/rows", f[0, ::fc.ROW_STRIDE])
        put(f"S/{name}/norms", f[0].double().norm(dim=-1))
        meta[f"S/{name}/sum"] = float(f.double().sum())
    moments = G.encode(img, return_z_before_quantize=True)
    put("F/moments", moments)
    torch.manual_seed(fc.EPS_SEED)
    out = G(img, ["x"], validation=True)
    put("F/gen_img", out.gen_img)
meta["g_kwargs"] = {k: v for k, v in g_kwargs.items() if k != "vfm_name"}
arrays["meta"] = np.array(json.dumps(meta))
np.savez_compressed(OUT, **arrays)
print(f"wrote {OUT}: {len(arrays)} arrays, {os.path.getsize(OUT) / 1024:.1f} KiB")
