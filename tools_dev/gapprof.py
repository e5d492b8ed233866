"""Where the GPU waits for the host: torch.profiler (kineto) over N bench iterations with Python stacks,
then every idle stretch between kernels (>= MIN_GAP us) is sampled every 5 us and attributed to the
innermost repo Python frame running at that moment on each host thread (the main thread and the
autograd engine's device thread). Prints inclusive / exclusive idle time per frame.

  python tools_dev/gapprof.py [steps=2]
"""
import collections
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vfm-vae_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

MIN_GAP = 20.0      # us
DT = 5.0            # us


def run(steps):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    c, step = bench.build(bench.CONFIG, 32, dev, 1)
    from training.data_synthetic import SyntheticDataset
    pool = SyntheticDataset(resolution=c.training_set_kwargs.resolution, seed=0).make_pool(32, dev)
    labels = ['a photo'] * 32
    for i in range(4):
        step([pool[i % len(pool)].float() / 255.], [labels], i * 32)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True) as prof:
        for i in range(steps):
            step([pool[i % len(pool)].float() / 255.], [labels], (4 + i) * 32)
        torch.cuda.synchronize()
    path = os.path.join(tempfile.mkdtemp(), "trace.json")
    prof.export_chrome_trace(path)
    return path


def analyse(path, steps):
    tr = json.load(open(path))
    evs = tr["traceEvents"] if isinstance(tr, dict) else tr
    gpu, py = [], collections.defaultdict(list)
    cats = collections.Counter(e.get("cat", "") for e in evs if e.get("ph") == "X")
    print("event categories:", dict(cats.most_common(12)), flush=True)
    for e in evs:
        if e.get("ph") != "X":
            continue
        cat = e.get("cat", "")
        ts, dur = float(e.get("ts", 0)), float(e.get("dur", 0))
        if cat in ("kernel", "gpu_memcpy", "gpu_memset"):
            gpu.append((ts, ts + dur))
        elif cat in ("python_function", "cpu_op", "user_annotation"):
            name = e.get("name", "")
            py[e.get("tid")].append((ts, ts + dur, name if cat == "python_function" else f"[{cat}] {name}"))
    gpu.sort()
    busy, merged = 0.0, []
    for s, t in gpu:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], t)
        else:
            merged.append([s, t])
    for s, t in merged:
        busy += t - s
    gaps = [(a[1], b[0]) for a, b in zip(merged, merged[1:]) if b[0] - a[1] >= MIN_GAP]
    idle = sum(b - a for a, b in gaps)
    span = merged[-1][1] - merged[0][0]
    print(f"{steps} steps: GPU busy {busy / steps / 1e3:.1f} ms/step, idle (gaps >= {MIN_GAP:.0f} us) "
          f"{idle / steps / 1e3:.1f} ms/step, span {span / steps / 1e3:.1f} ms/step, {len(gaps)} gaps", flush=True)
    samples = []
    for a, b in gaps:
        t = a + DT / 2
        while t < b:
            samples.append(t)
            t += DT
    keys = ("vfm-vae_amd", "bench.py", "training/", "torch_utils/", "networks/")
    repo = lambda n: any(k in n for k in keys) and "tools_dev" not in n and "site-packages" not in n  # noqa: E731
    print("host events per thread:", {t: len(v) for t, v in py.items()}, flush=True)
    names = collections.Counter(e[2] for v in py.values() for e in v if not e[2].startswith("["))
    print("sample python frames:", [n for n, _ in names.most_common(8)], flush=True)
    for tid, lst in py.items():
        lst.sort(key=lambda x: (x[0], -x[1]))
        incl, excl = collections.Counter(), collections.Counter()
        stack, i = [], 0
        hit = 0
        for t in samples:
            while i < len(lst) and lst[i][0] <= t:
                while stack and stack[-1][1] < lst[i][0]:
                    stack.pop()
                stack.append(lst[i])
                i += 1
            while stack and stack[-1][1] < t:
                stack.pop()
            live = [e[2] for e in stack if e[1] >= t]
            frames = [f for f in live if repo(f)]
            if live and live[-1].startswith("["):       # the innermost event is an op: keep it as the leaf
                frames.append(live[-1])
            if not frames:
                continue
            hit += 1
            excl[frames[-1]] += DT
            for f in set(frames):
                incl[f] += DT
        if hit * DT < 0.02 * idle:
            continue
        print(f"\nthread {tid}: {hit * DT / steps / 1e3:.1f} ms/step of GPU idle inside repo frames", flush=True)
        print("  inclusive:")
        for f, v in incl.most_common(40):
            print(f"  {v / steps / 1e3:7.2f} ms/step  {f}")
        print("  exclusive (innermost repo frame):")
        for f, v in excl.most_common(40):
            print(f"  {v / steps / 1e3:7.2f} ms/step  {f}")


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    analyse(run(n), n)
