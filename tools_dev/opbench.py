"""Micro-benchmark of the StyleGAN-lineage HIP ops (algorithmic GB/s vs 8 TB/s)."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch
from torch_utils.ops import upfirdn2d, bias_act, filtered_lrelu

dev = "cuda"
def timeit(fn, iters=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / iters / 1e3

res = {}
for dt in (torch.float32, torch.bfloat16):
    x = torch.randn(32, 128, 256, 256, device=dev, dtype=dt)
    f = upfirdn2d.setup_filter([1, 4, 6, 4, 1], device=dev)
    t = timeit(lambda: upfirdn2d.filter2d(x, f))
    byt = 2 * x.numel() * x.element_size()
    res[f"filter2d_5x5_{dt}"] = dict(ms=t * 1e3, GBs=byt / t / 1e9)
    f4 = upfirdn2d.setup_filter([1, 3, 3, 1], device=dev)
    xs = x[:, :, :128, :128].contiguous()
    t = timeit(lambda: upfirdn2d.upsample2d(xs, f4))
    byt = 5 * xs.numel() * xs.element_size()
    res[f"upsample2d_{dt}"] = dict(ms=t * 1e3, GBs=byt / t / 1e9)
    b = torch.randn(128, device=dev, dtype=dt)
    t = timeit(lambda: bias_act.bias_act(x, b, act='lrelu'))
    byt = 2 * x.numel() * x.element_size()
    res[f"bias_act_lrelu_{dt}"] = dict(ms=t * 1e3, GBs=byt / t / 1e9)
x = torch.randn(32, 128, 128, 128, device=dev, dtype=torch.float16)
f12 = upfirdn2d.setup_filter(torch.rand(12) + .2, separable=True, device=dev)
t = timeit(lambda: filtered_lrelu.filtered_lrelu(x, f12, f12, up=2, down=2, padding=10))
res["filtered_lrelu_fp16_u2d2_12tap"] = dict(ms=t * 1e3, GBs=2 * x.numel() * 2 / t / 1e9)
print(json.dumps(res, indent=1))
