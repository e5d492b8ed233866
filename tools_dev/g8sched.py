"""Microbench: gemm8 (both K-tile staging schedules, vfm_gemm8_set_schedule) against hipBLASLt on the bf16 square and SigLIP2 shapes and the f32x6
decoder / adapter shapes (times include the activation split for fp32; weights cached)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch

from torch_utils import custom_ops
from torch_utils.ops import gemm_hip

lib = custom_ops.get_native()


def bench(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def rnd(*shape, dt=torch.bfloat16):
    return (torch.rand(*shape, device="cuda") * 2 - 1).to(dt)       # uniform [-1, 1) (not zero-filled)


def row(name, fl, ours, blas):
    res = []
    for sched in (1, 0):
        lib.vfm_gemm8_set_schedule(sched)
        res.append(bench(ours))
    lib.vfm_gemm8_set_schedule(1)
    tb = bench(blas)
    print(f"{name:34s} deep {res[0] * 1e3:8.1f}us {fl / res[0] / 1e9:7.1f} | one-ahead {res[1] * 1e3:8.1f}us "
          f"{fl / res[1] / 1e9:7.1f} | blas {tb * 1e3:8.1f}us {fl / tb / 1e9:7.1f}  TF/s", flush=True)


torch.backends.cuda.matmul.allow_tf32 = False
for name, M, N, K in [("bf16 8192^3", 8192, 8192, 8192), ("bf16 4096^3", 4096, 4096, 4096),
                      ("siglip qkv 32768x3072x1024", 32768, 3072, 1024), ("siglip fc1 32768x4096x1024", 32768, 4096, 1024),
                      ("siglip fc2 32768x1024x4096", 32768, 1024, 4096), ("siglip o 32768x1024x1024", 32768, 1024, 1024)]:
    A, W = rnd(M, K), rnd(N, K)
    row(name, 2.0 * M * N * K, lambda: gemm_hip.gemm(A, W.t(), route=("g8", 0)), lambda: A @ W.t())

for name, M, N, K in [("f32x6 adapter qkv 32768x3072x1024", 32768, 3072, 1024), ("f32x6 dino fc1 6304x1536x384", 6304, 1536, 384)]:
    A, W = rnd(M, K, dt=torch.float32), rnd(N, K, dt=torch.float32)
    row(name, 2.0 * M * N * K, lambda: gemm_hip.gemm(A, W.t(), cache_b=True, route=("g8", 0)), lambda: A @ W.t())

for name, O, I, P in [("f32x6 b2 W1 2048x1024x512x32", 2048, 512, 1024), ("f32x6 b2 W2 512x1024x2048x32", 512, 2048, 1024)]:
    Bn = 32
    W, x = rnd(O, I, dt=torch.float32), rnd(Bn, I, P, dt=torch.float32)
    row(name, 2.0 * Bn * O * I * P, lambda: gemm_hip.gemm(W, x, cache_a=True, route=("g8", 0)),
        lambda: torch.bmm(W.expand(Bn, O, I), x))
