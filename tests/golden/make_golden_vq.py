"""Golden vectors for the discrete-latent codebook lookup, generated FROM THE REFERENCE.

Runs only in the build container: imports /root/reference's
networks/utils/quant_utils.py on CPU (fp32) and records, for config 4's quantiser
(vocab 32768, width 32, 8 codebooks -> 8 x [4096, 4]) and a few edge cases:
  * inputs (features, codebook weights),
  * the reference's indices from VectorQuantizerM.f_to_idx and forward()'s f_hat /
    vq_loss / vocab_usage,
  * the reference's top-1 / top-2 score margin per token (so a test can tell a genuine
    mismatch from a last-ulp near-tie that depends on the GEMM's summation order).
Writes tests/golden/vq_golden.npz.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_vq.py
"""
import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("VFM_REFERENCE", "/root/reference")
sys.path.insert(0, os.path.join(HERE, "ref_stubs"))
sys.path.insert(0, REF)

from networks.utils.quant_utils import VectorQuantizerM, VectorQuantizer  # noqa: E402

OUT = os.path.join(HERE, "vq_golden.npz")
arrays, meta = {}, {"cases": []}


def margins(feat, weight):
    f = F.normalize(feat.reshape(-1, feat.shape[-1]), dim=-1).float()
    s = f @ F.normalize(weight, dim=1).float().T
    top = torch.topk(s, 2, dim=1).values
    return (top[:, 0] - top[:, 1]).numpy()


def put(k, v):
    arrays[k] = v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)


# ---- config 4 quantiser: VectorQuantizerM(32768, 32, num_codebooks=8), B=2 x 256 tokens
torch.manual_seed(0)
vq = VectorQuantizerM(vocab_size=32768, vocab_width=32, beta=0.25, num_codebooks=8)
vq.init_vocab(-1)                          # uniform init of the reference's config path
feats = torch.randn(2, 256, 32)
with torch.no_grad():
    idx = vq.f_to_idx(feats)               # [B, 8, L]
vq.train()
fin = feats.clone().requires_grad_(True)
f_hat, vq_loss, ent, usage = vq(fin)
put("m/features", feats)
for i, cb in enumerate(vq.codebooks):
    put(f"m/codebook{i}", cb.codebook.weight)
    put(f"m/margin{i}", margins(feats[..., 4 * i:4 * i + 4], cb.codebook.weight.detach()))
put("m/indices", idx)
put("m/f_hat", f_hat)
put("m/vq_loss", vq_loss)
put("m/vocab_usage", usage)
meta["m"] = {"vocab_size": 32768, "vocab_width": 32, "num_codebooks": 8}

# ---- single wide codebook (VectorQuantizer, width 32), trunc-normal init
torch.manual_seed(1)
q = VectorQuantizer(vocab_size=1000, vocab_width=32)
q.init_vocab(0.02)
f32 = torch.randn(3, 100, 32)
with torch.no_grad():
    put("w/indices", q.f_to_idx(f32))
put("w/features", f32)
put("w/codebook", q.codebook.weight)
put("w/margin", margins(f32, q.codebook.weight.detach()))

# ---- exact ties: duplicated codebook rows and scaled copies -> the first index must win
torch.manual_seed(2)
w = torch.randn(64, 4)
w[40] = w[7]
w[41] = 3.0 * w[7]
w[50] = w[3]
ft = torch.cat([w[7:8] * 0.5, w[3:4], torch.randn(6, 4)], 0)
q2 = VectorQuantizer(vocab_size=64, vocab_width=4)
with torch.no_grad():
    q2.codebook.weight.copy_(w)
    put("t/indices", q2.f_to_idx(ft[None]))
put("t/features", ft)
put("t/codebook", w)

# ---- zero feature vector (normalize eps path): all scores 0 -> index 0
q3 = VectorQuantizer(vocab_size=16, vocab_width=4)
torch.manual_seed(3)
z = torch.zeros(1, 2, 4)
z[0, 1] = torch.randn(4)
with torch.no_grad():
    put("z/indices", q3.f_to_idx(z))
put("z/features", z)
put("z/codebook", q3.codebook.weight)

arrays["meta"] = np.array(json.dumps(meta))
np.savez_compressed(OUT, **arrays)
print(f"wrote {OUT}: {len(arrays)} arrays, {os.path.getsize(OUT) / 1024:.1f} KiB")
