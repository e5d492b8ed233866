"""Micro-benchmark of the channel RMS norm (decoder attention blocks, fp32 [B, C, H, W]) forward and
backward at batch 32: average us and algorithmic GB/s (fwd x + y, bwd x + dy + dx).
  python tools_dev/crmsbench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch  # noqa: E402

from torch_utils.ops import decoder_hip  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


for C, R in [(512, 8), (512, 16), (512, 32), (256, 32), (256, 64)]:
    x = torch.randn(32, C, R, R, device="cuda", requires_grad=True)
    g = torch.rand(C, device="cuda", requires_grad=True)
    n = x.numel() * 4
    us = timeit(lambda: decoder_hip.channel_rms_norm(x.detach(), g.detach(), C ** 0.5))
    print(f"C={C} {R}x{R} fwd {us:8.1f} us {2 * n / us / 1e3:8.1f} GB/s", flush=True)
    y = decoder_hip.channel_rms_norm(x, g, C ** 0.5)
    dy = torch.randn_like(y)
    us = timeit(lambda: torch.autograd.grad(y, (x, g), dy, retain_graph=True))
    print(f"C={C} {R}x{R} bwd {us:8.1f} us {3 * n / us / 1e3:8.1f} GB/s", flush=True)
