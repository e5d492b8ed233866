"""Which fp32 operands the f32x6 products split into bf16 pieces per training iteration (csrc/gemm8.hip
split_planar_kernel / split_f32_kernel launches): every split that misses the per-tensor cache is recorded
with the operand's shape, whether it is a parameter, and the repo call site (forward stack, or the autograd
node in the backward)."""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vfm-vae_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from torch_utils.ops import gemm_hip  # noqa: E402


def _where():
    fr = [f"{os.path.relpath(f.filename, ROOT)}:{f.lineno}" for f in traceback.extract_stack()
          if ROOT in f.filename and "tools_dev" not in f.filename and "gemm_hip.py" not in f.filename]
    node = torch._C._current_autograd_node()
    pre = f"bwd {node.name()} " if node is not None else "fwd "
    return pre + " < ".join(reversed(fr[-3:]))


REC = collections.Counter()
BYTES = collections.Counter()
ON = [False]
REPL = []
SEQ = []


def _wrap(name, fn, hit_attr):
    def w(t3, *a, **k):
        if ON[0]:
            base = t3._base if t3._base is not None else t3
            before = getattr(base, hit_attr, None)
            out = fn(t3, *a, **k)
            after = getattr(base, hit_attr, None)
            if tuple(base.shape) == (32, 2048, 1024) and len(SEQ) < 40:
                SEQ.append((f"{id(base):x}", base._version, before is None, after is before, _where()))
            if after is not before or after is None:
                if before is not None and len(REPL) < 12:
                    REPL.append((tuple(base.shape), before[0], after[0] if after is not None else None, _where()))
                key = (name, tuple(base.shape), isinstance(base, torch.nn.Parameter), _where())
                REC[key] += 1
                BYTES[key] += base.numel() * 4
            return out
        return fn(t3, *a, **k)
    return w


gemm_hip._planar = _wrap("planar", gemm_hip._planar, "_vfm_planar")
gemm_hip._split_f32 = _wrap("stacked", gemm_hip._split_f32, "_vfm_split_f32")


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
    ON[0] = True
    n = 4
    for i in range(n):
        step([pool[(3 + i) % len(pool)].float() / 255.], [labels], (3 + i) * 32)
    torch.cuda.synchronize()
    ON[0] = False
    tot = sum(REC.values()) / n
    params = sum(v for k, v in REC.items() if k[2]) / n
    print(f"splits per iteration: {tot:.1f} (parameters {params:.1f}); "
          f"fp32 bytes split per iteration {sum(BYTES.values()) / n / 1e6:.1f} MB", flush=True)
    print("cache entries replaced (old key -> new key):", flush=True)
    for r in REPL:
        print("   ", r, flush=True)
    print("(32, 2048, 1024) operand events (base id, version, no entry before, hit, site):", flush=True)
    for r in SEQ:
        print("   ", r, flush=True)
    for (kind, shape, isp, where), cnt in sorted(REC.items(), key=lambda kv: -BYTES[kv[0]])[:80]:
        print(f"{cnt / n:6.1f}/it {BYTES[(kind, shape, isp, where)] / n / 1e6:8.2f} MB  {kind:7s} "
              f"{'param' if isp else 'act  '} {str(shape):24s} {where}", flush=True)


if __name__ == "__main__":
    main()
