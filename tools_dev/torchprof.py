"""Attribute GPU time of one training iteration to torch ops (torch.profiler).

  python tools_dev/torchprof.py [--batch 32] [--out gpurun_out/tp]

Prints the top ops by self device time and the top kernels with the op and
input shapes that launched them (record_shapes), to find unfused copies etc.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "vfm-vae_amd"))
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")

import torch  # noqa: E402

import bench  # noqa: E402


def _ours(stack):
    """This package's frames of a profiler stack (relative paths; torch / builtin frames dropped)."""
    return [f.split("vfm-vae_amd/")[-1] for f in stack
            if not f.startswith(("torch/", "<built-in", "nn.Module", "contextlib")) and "kernel_timer" not in f
            and "/torch/" not in f]


def idle_by_stack(prof, path, min_gap_us=5.0):
    """GPU idle gaps attributed to the Python call site that launched the kernel after each
    gap (kernel -> runtime launch event by correlation id -> innermost op with a stack)."""
    import bisect
    from collections import defaultdict
    kin = prof.profiler.kineto_results
    t0 = kin.trace_start_ns()
    kernels, cpu_by_corr = [], {}
    for e in kin.events():
        if e.device_type() == torch.autograd.DeviceType.CUDA:
            if e.duration_ns() > 0:
                kernels.append((e.start_ns(), e.start_ns() + e.duration_ns(), e.linked_correlation_id(), e.name()))
        else:
            cpu_by_corr[e.correlation_id()] = e.start_ns()
    kernels.sort()
    ops = [fe for fe in prof.events() if fe.stack and fe.device_type == torch.autograd.DeviceType.CPU]
    ops.sort(key=lambda fe: fe.time_range.start)
    starts = [t0 + fe.time_range.start * 1000 for fe in ops]

    def site(t):
        i = bisect.bisect_right(starts, t) - 1
        best = None
        while i >= 0 and i > bisect.bisect_right(starts, t) - 400:
            fe = ops[i]
            if t0 + fe.time_range.end * 1000 >= t:
                if best is None or fe.time_range.start > best.time_range.start:
                    best = fe
                    break
            i -= 1
        if best is None:
            return "(no op)"
        return best.name + " <- " + " <- ".join(_ours(best.stack)[:4])

    idle = defaultdict(float)
    cnt = defaultdict(int)
    total = 0.0
    for (s0, e0, _, _), (s1, e1, corr, name) in zip(kernels, kernels[1:]):
        gap = (s1 - max(e0, s0)) / 1e3
        if gap < min_gap_us:
            continue
        t = cpu_by_corr.get(corr)
        key = site(t) if t is not None else "(no launch event) " + name[:60]
        idle[key] += gap
        cnt[key] += 1
        total += gap
    with open(path, "w") as f:
        f.write(f"GPU idle in gaps >= {min_gap_us} us: {total / 1e3:.2f} ms over {len(kernels)} kernels\n")
        for k, v in sorted(idle.items(), key=lambda kv: -kv[1])[:80]:
            f.write(f"{v / 1e3:8.2f} ms  {cnt[k]:6d} gaps  {k}\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--out", default="gpurun_out/tp")
    ap.add_argument("--rows", type=int, default=60)
    ap.add_argument("--eq-scale", type=float, default=1.0, help="force the equivariance scale of the profiled step")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    c, step = bench.build(bench.CONFIG, args.batch, dev, 1)
    from training.data_synthetic import SyntheticDataset
    pool = SyntheticDataset(resolution=c.training_set_kwargs.resolution, seed=0).make_pool(args.batch, dev)
    labels = ['a photo'] * args.batch
    for i in range(2):
        step([pool[i % len(pool)].float() / 255.], [labels], i * args.batch)
    step.G.equivariance_transform.forced = (args.eq_scale, 0, False)
    step([pool[1].float() / 255.], [labels], 2 * args.batch)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    cfg = torch._C._profiler._ExperimentalConfig(verbose=True)      # Python stacks need verbose on this torch
    with torch.profiler.profile(activities=acts, record_shapes=True, with_stack=True, experimental_config=cfg) as prof:
        step([pool[0].float() / 255.], [labels], 2 * args.batch)
        torch.cuda.synchronize()
    sort = "self_cuda_time_total"
    t1 = prof.key_averages().table(sort_by=sort, row_limit=args.rows, max_name_column_width=60)
    t2 = prof.key_averages(group_by_input_shape=True).table(sort_by=sort, row_limit=args.rows,
                                                            max_name_column_width=50, max_shapes_column_width=90)
    t3 = prof.key_averages(group_by_stack_n=8).table(sort_by=sort, row_limit=args.rows, max_name_column_width=40)
    open(os.path.join(args.out, "ops_stack.txt"), "w").write(t3)
    # copies only, with their stacks
    evs = [e for e in prof.key_averages(group_by_input_shape=True, group_by_stack_n=10) if e.key in ("aten::copy_", "aten::clone", "aten::contiguous")]
    evs.sort(key=lambda e: -e.self_device_time_total)
    with open(os.path.join(args.out, "copies.txt"), "w") as f:
        for e in evs[:40]:
            f.write(f"{e.key} calls={e.count} self_dev_ms={e.self_device_time_total / 1e3:.2f} shapes={e.input_shapes}\n")
            for fr in e.stack:
                f.write(f"    {fr}\n")
    # every non-GEMM op group (op + input shapes + stack), by self device time
    skip = ("aten::mm", "aten::bmm", "aten::addmm", "aten::convolution", "aten::cudnn_convolution",
            "aten::miopen_convolution", "aten::_scaled_dot_product", "aten::_efficient_attention",
            "aten::_flash_attention", "aten::matmul", "aten::linear", "aten::baddbmm")
    evs = [e for e in prof.key_averages(group_by_input_shape=True, group_by_stack_n=12)
           if e.key.startswith("aten::") and not e.key.startswith(skip) and e.self_device_time_total > 0]
    evs.sort(key=lambda e: -e.self_device_time_total)
    with open(os.path.join(args.out, "small_ops.txt"), "w") as f:
        for e in evs[:120]:
            f.write(f"{e.key} calls={e.count} self_dev_ms={e.self_device_time_total / 1e3:.2f} shapes={e.input_shapes}\n")
            for fr in e.stack:
                f.write(f"    {fr}\n")
    idle_by_stack(prof, os.path.join(args.out, "idle_by_stack.txt"))
    open(os.path.join(args.out, "ops_count.txt"), "w").write(
        prof.key_averages().table(sort_by="count", row_limit=80, max_name_column_width=60))
    # launch sites: (op, our call stack) groups with device work, by number of calls
    evs = [e for e in prof.key_averages(group_by_stack_n=25)
           if e.key.startswith("aten::") and e.self_device_time_total > 0]
    evs.sort(key=lambda e: -e.count)
    with open(os.path.join(args.out, "launch_sites.txt"), "w") as f:
        for e in evs[:150]:
            fr = _ours(e.stack)[:5]
            f.write(f"{e.count:6d} calls {e.self_device_time_total / 1e3:8.2f} ms  {e.key}  <- {' <- '.join(fr)}\n")
    open(os.path.join(args.out, "ops.txt"), "w").write(t1)
    open(os.path.join(args.out, "ops_shapes.txt"), "w").write(t2)
    print(t1[:12000])


if __name__ == "__main__":
    main()
