"""Which ops launch the large copies of one training iteration: for every aten::copy_ with
more than 4M elements, its chain of parent ops (torch.profiler event tree) and shapes."""
import os
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vfm-vae_amd"))
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    c, step = bench.build(bench.CONFIG, 32, dev, 1)
    from training.data_synthetic import SyntheticDataset
    pool = SyntheticDataset(resolution=c.training_set_kwargs.resolution, seed=0).make_pool(32, dev)
    labels = ['a photo'] * 32
    for i in range(3):
        step([pool[i % len(pool)].float() / 255.], [labels], i * 32)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, record_shapes=True) as prof:
        step([pool[0].float() / 255.], [labels], 3 * 32)
        torch.cuda.synchronize()
    chains = Counter()
    for e in prof.events():
        if e.name != "aten::copy_" or not e.input_shapes or not e.input_shapes[0]:
            continue
        n = 1
        for d in e.input_shapes[0]:
            n *= d
        if n < 4_000_000:
            continue
        names, p = [], e.cpu_parent
        while p is not None and len(names) < 6:
            names.append(p.name)
            p = p.cpu_parent
        dts = ",".join(str(x) for x in (e.input_shapes[0], e.input_shapes[1] if len(e.input_shapes) > 1 else ""))
        chains[(" <- ".join(names), dts)] += 1
    for (ch, sh), k in chains.most_common(40):
        print(f"{k:4d}  {sh}  <- {ch}")


if __name__ == "__main__":
    main()
