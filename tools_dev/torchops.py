"""Where the small torch kernels of one training iteration come from: every aten op that launches
GPU work outside our kernel library, grouped by (op, nearest non-aten parent chain), ranked by GPU
time (torch.profiler, record_shapes). One warm step first."""
import os
import sys
from collections import defaultdict

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
    with torch.profiler.profile(activities=acts, record_shapes=True, with_stack=True) as prof:
        step([pool[0].float() / 255.], [labels], 3 * 32)
        torch.cuda.synchronize()
    agg = defaultdict(lambda: [0, 0.0])
    for e in prof.events():
        if not e.name.startswith("aten::") or e.cpu_parent is None:
            continue
        if e.cpu_parent.name.startswith("aten::"):      # count the outermost aten op only
            continue
        dt = getattr(e, "device_time_total", 0.0) or getattr(e, "cuda_time_total", 0.0)
        if dt <= 0:
            continue
        frames = [f for f in (e.stack or []) if "vfm-vae_amd" in f or "bench.py" in f]
        where = " | ".join(f.split("vfm-vae_amd/")[-1] for f in frames[:3])
        agg[(e.name, where)][0] += 1
        agg[(e.name, where)][1] += dt
    tot_n = sum(v[0] for v in agg.values())
    tot_t = sum(v[1] for v in agg.values())
    print(f"torch ops with GPU work: {tot_n} calls, {tot_t / 1e3:.1f} ms GPU per step", flush=True)
    for (name, where), (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:60]:
        print(f"{t / 1e3:7.2f} ms {n:5d}x  {name:28s} {where}", flush=True)


if __name__ == "__main__":
    main()
