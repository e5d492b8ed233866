"""Microbench: gemm8 (bf16) time vs K at fixed M x N against hipBLASLt, to separate the per-tile
fixed cost (prologue, epilogue, block dispatch) from the per-K-tile cost of the main loop."""
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
    return s.elapsed_time(e) / iters * 1e3


def rnd(*shape):
    return (torch.rand(*shape, device="cuda") * 2 - 1).to(torch.bfloat16)


lib.vfm_gemm8_set_schedule(int(os.environ.get("G8_DEEP", "1")))
for M, N in [(32768, 1024), (32768, 3072), (8192, 8192)]:
    tiles = (M // 256) * (N // 256)
    for K in (64, 128, 256, 512, 1024, 2048, 4096):
        A, W = rnd(M, K), rnd(N, K)
        out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        t8 = bench(lambda: gemm_hip.try_gemm(A, W.t(), out=out, route=("g8", 0)))
        tb = bench(lambda: torch.matmul(A, W.t(), out=out))
        fl = 2.0 * M * N * K
        per = t8 * 256 / tiles
        print(f"M={M} N={N} K={K:5d} tiles={tiles:5d} | gemm8 {t8:8.1f}us {fl / t8 / 1e6:7.1f} TF/s "
              f"({per:6.2f} us/tile/CU) | blas {tb:8.1f}us {fl / tb / 1e6:7.1f} TF/s", flush=True)
