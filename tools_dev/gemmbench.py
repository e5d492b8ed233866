"""Microbench: MFMA GEMM (csrc/gemm.hip) vs hipBLASLt (torch) on the hot path's shapes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch

from torch_utils.ops import gemm_hip


def bench(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


cases = [
    # (name, dtype, M, N, K, a_t, b_t)   a_t: A stored [K][M]; b_t: B stored [N][K]
    ("siglip qkv", torch.bfloat16, 32768, 3072, 1024, False, True),
    ("siglip fc1", torch.bfloat16, 32768, 4096, 1024, False, True),
    ("siglip fc2", torch.bfloat16, 32768, 1024, 4096, False, True),
    ("siglip o", torch.bfloat16, 32768, 1024, 1024, False, True),
    ("dec b2 mlp W1.x (fp32)", torch.float32, 2048, 1024, 512, False, False),
    ("adapter qkv (fp32)", torch.float32, 32768, 3072, 1024, False, True),
    ("dec b5 1x1 W.x (bf16)", torch.bfloat16, 512, 65536, 128, False, False),
]
for name, dt, M, N, K, a_t, b_t in cases:
    A = torch.randn(K, M, device="cuda").to(dt).t() if a_t else torch.randn(M, K, device="cuda").to(dt)
    B = torch.randn(N, K, device="cuda").to(dt).t() if b_t else torch.randn(K, N, device="cuda").to(dt)
    fl = 2.0 * M * N * K
    th = bench(lambda: gemm_hip.gemm(A, B))
    tt = bench(lambda: A @ B)
    print(f"{name:28s} M={M} N={N} K={K}: hip {th:.3f} ms {fl / th / 1e9:7.1f} TF/s | torch {tt:.3f} ms "
          f"{fl / tt / 1e9:7.1f} TF/s", flush=True)
