"""Why the fused optimizer step rebuilds its device tables: a few bench iterations with VFM_ADAM_DEBUG=1 (the
reason printed per rebuild) and the rebuild count per phase."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vfm-vae_amd")]
os.environ["VFM_ADAM_DEBUG"] = "1"
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
c, step = bench.build(bench.CONFIG, 32, dev, 1)
from training.data_synthetic import SyntheticDataset  # noqa: E402
pool = SyntheticDataset(resolution=c.training_set_kwargs.resolution, seed=0).make_pool(32, dev)
for i in range(6):
    print(f"--- step {i}", flush=True)
    step([pool[i % len(pool)].float() / 255.], [['a photo'] * 32], i * 32)
torch.cuda.synchronize()
for ph in step.phases:
    print(ph.name, "rebuilds", ph.get("adam_rebuilds"), flush=True)
