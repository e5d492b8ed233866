"""Call sites of the torch (aten) ops one training iteration runs on the GPU, by count: a
TorchDispatchMode sees every aten call; forward calls are attributed to the innermost repo frames
of the Python stack, backward calls to the autograd node being run and the forward stack that made
it (anomaly mode keeps it). Ops from our own kernel library are not aten calls and do not show.
With OPSITES_TIME=1 each aten call is also timed on the GPU (the stream synchronised before the
call, HIP events around it: kernel time plus ~10 us of launch latency per call) and the call sites
are ranked by that time."""
import collections
import re
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vfm-vae_amd")]
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

import bench  # noqa: E402

SKIP = {"aten.detach.default", "aten.view.default", "aten._unsafe_view.default", "aten.t.default",
        "aten.as_strided.default", "aten.expand.default", "aten.permute.default", "aten.transpose.int",
        "aten.unsqueeze.default", "aten.squeeze.dim", "aten.slice.Tensor", "aten.select.int",
        "aten.alias.default", "aten.empty.memory_format", "aten.empty_strided.default",
        "aten.is_same_size.default", "aten._to_copy.default_noop", "aten.split.Tensor",
        "aten.lift_fresh.default", "aten._local_scalar_dense.default", "aten.empty_like.default",
        "aten.reshape.default", "aten.unbind.int", "aten.chunk.default", "aten.split_with_sizes.default",
        "aten.squeeze.default", "aten.view_as_real.default", "aten.new_empty.default",
        "aten.new_empty_strided.default", "aten.set_.source_Storage_storage_offset"}


def _repo_frames(frames, n=3):
    out = [f"{os.path.relpath(f.filename, ROOT)}:{f.lineno}" for f in frames
           if ROOT in f.filename and "tools_dev" not in f.filename and "_python_dispatch" not in f.filename]
    return " < ".join(reversed(out[-n:]))


# OPSITES_OPS=mm,bmm,addmm,convolution: only aten ops whose name contains one of these (the library GEMM /
# convolution call sites), printed with their shapes
ONLY = [o for o in os.environ.get("OPSITES_OPS", "").split(",") if o]


class Sites(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.count = collections.Counter()
        self.timed = os.environ.get("OPSITES_TIME") == "1"
        self.events = collections.defaultdict(list)

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        ev = None
        if self.timed and name not in SKIP:
            torch.cuda.synchronize()
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        out = func(*args, **(kwargs or {}))
        if ev is not None:
            ev[1].record()
        if name in SKIP or (ONLY and not any(o in name for o in ONLY)):
            return out
        t = out[0] if isinstance(out, (tuple, list)) and out else out
        if not (isinstance(t, torch.Tensor) and (t.is_cuda or os.environ.get("OPSITES_CPU"))):
            return out
        node = torch._C._current_autograd_node()
        if node is not None:
            tb = node.metadata.get("traceback_", []) if hasattr(node, "metadata") else []
            sites = []
            for ent in tb if isinstance(tb, list) else []:
                m = re.search(r'File "([^"]+)", line (\d+)', ent)
                if m and ROOT in m.group(1) and "tools_dev" not in m.group(1):
                    sites.append(f"{os.path.relpath(m.group(1), ROOT)}:{m.group(2)}")
            here = _repo_frames(traceback.extract_stack(), 1)
            where = f"bwd {node.name()}{' @ ' + here if here else ''} < " + " < ".join(reversed(sites[-2:]))
        else:
            where = "fwd " + _repo_frames(traceback.extract_stack())
        if ONLY:
            where += "  " + " ".join(str(tuple(a.shape)) + ("" if a.is_contiguous() else "nc")
                                     for a in args if isinstance(a, torch.Tensor)) + f" {t.dtype}"
        self.count[(name, where)] += 1
        if ev is not None:
            self.events[(name, where)].append(ev)
        return out


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
    mode = Sites()
    with torch.autograd.set_detect_anomaly(True, check_nan=False), mode:
        step([pool[0].float() / 255.], [labels], 3 * 32)
    torch.cuda.synchronize()
    tot = sum(mode.count.values())
    per_op = collections.Counter()
    for (name, _), n in mode.count.items():
        per_op[name] += n
    print(f"aten calls on the GPU in one iteration: {tot}", flush=True)
    for name, n in per_op.most_common(30):
        print(f"  {n:5d}  {name}", flush=True)
    print("by call site:", flush=True)
    for (name, where), n in mode.count.most_common(120):
        print(f"{n:5d}  {name:36s} {where}", flush=True)
    if mode.timed:
        ms = {k: sum(a.elapsed_time(b) for a, b in evs) for k, evs in mode.events.items()}
        per_op_ms = collections.Counter()
        for (name, _), t in ms.items():
            per_op_ms[name] += t
        print(f"GPU time of the timed aten calls: {sum(ms.values()):.2f} ms", flush=True)
        for name, t in per_op_ms.most_common(30):
            print(f"  {t:8.3f} ms  {name}", flush=True)
        print("by call site (GPU ms, calls):", flush=True)
        for (name, where), t in sorted(ms.items(), key=lambda kv: -kv[1])[:150]:
            print(f"{t:8.3f} ms {mode.count[(name, where)]:5d}  {name:36s} {where}", flush=True)


if __name__ == "__main__":
    main()
