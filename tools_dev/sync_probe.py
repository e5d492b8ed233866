"""Host<->device synchronisations inside one training iteration of the bench workload: torch's CUDA sync debug
mode ("warn") reports every synchronising call (blocking H2D / D2H copies such as torch.tensor(..., device=cuda),
.item(), .tolist(), stream synchronisation); each is printed once per call site with the innermost repo frames.

  python tools_dev/sync_probe.py"""
import collections
import os
import sys
import traceback
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vfm-vae_amd")]
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
c, step = bench.build(bench.CONFIG, 32, dev, 1)
from training.data_synthetic import SyntheticDataset  # noqa: E402
pool = SyntheticDataset(resolution=c.training_set_kwargs.resolution, seed=0).make_pool(32, dev)
labels = ['a photo'] * 32
eqt = step.G.equivariance_transform
for v in eqt.variants():
    eqt.forced = v
    step([pool[0].float() / 255.], [labels], 0)
eqt.forced = None
for i in range(3):
    step([pool[i % len(pool)].float() / 255.], [labels], (i + 1) * 32)
torch.cuda.synchronize()

sites = collections.Counter()


def hook(message, category, filename, lineno, file=None, line=None):
    frames = [f for f in traceback.extract_stack() if ROOT in f.filename and "sync_probe" not in f.filename]
    key = " < ".join(f"{os.path.relpath(f.filename, ROOT)}:{f.lineno}" for f in frames[-3:][::-1])
    sites[(str(message)[:60], key)] += 1


warnings.showwarning = hook
warnings.simplefilter("always")
n = 4
torch.cuda.set_sync_debug_mode("warn")
for i in range(n):
    step([pool[i % len(pool)].float() / 255.], [labels], (10 + i) * 32)
torch.cuda.set_sync_debug_mode("default")
torch.cuda.synchronize()
print(f"synchronising calls over {n} iterations: {sum(sites.values())}")
for (msg, key), k in sites.most_common():
    print(f"{k:5d}  {msg:60s}  {key}")
