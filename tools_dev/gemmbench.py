"""Microbench: MFMA GEMM (csrc/gemm.hip, csrc/gemm_fast.hip) vs hipBLASLt (torch) on the hot
path's shapes, including the decoder's fp32 1x1 convolutions at batch 32 (forward, data
gradient, batch-reduced weight gradient) and the adapter projections."""
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


def row(name, fl, fh, ft):
    gemm_hip.GEMM8 = True
    th8 = bench(fh)
    gemm_hip.GEMM8 = False
    th = bench(fh)
    gemm_hip.GEMM8 = True
    tt = bench(ft)
    print(f"{name:34s} gemm8 {th8:7.3f} ms {fl / th8 / 1e9:7.1f} TF/s | fast {th:7.3f} ms {fl / th / 1e9:7.1f} TF/s"
          f" | torch {tt:7.3f} ms {fl / tt / 1e9:7.1f} TF/s", flush=True)


dev = "cuda"
for name, dt, M, N, K in [("siglip qkv bf16", torch.bfloat16, 32768, 3072, 1024),
                          ("siglip fc1 bf16", torch.bfloat16, 32768, 4096, 1024),
                          ("siglip fc2 bf16", torch.bfloat16, 32768, 1024, 4096),
                          ("square 8192 bf16", torch.bfloat16, 8192, 8192, 8192),
                          ("adapter qkv fp32", torch.float32, 32768, 3072, 1024)]:
    A = torch.randn(M, K, device=dev).to(dt)
    W = torch.randn(N, K, device=dev).to(dt)
    row(name, 2.0 * M * N * K, lambda: gemm_hip.gemm(A, W.t(), cache_b=True), lambda: A @ W.t())

# decoder fp32 1x1 convs at batch 32: (O, I, P) per block
for name, O, I, P in [("b2 W1 (512->2048 @32^2)", 2048, 512, 1024), ("b2 W2 (2048->512 @32^2)", 512, 2048, 1024),
                      ("b1 W1 (512->2048 @16^2)", 2048, 512, 256), ("b0 W1 (512->2048 @8^2)", 2048, 512, 64)]:
    Bn = 32
    W = torch.randn(O, I, device=dev)
    x = torch.randn(Bn, I, P, device=dev)
    dy = torch.randn(Bn, O, P, device=dev)
    fl = 2.0 * Bn * O * I * P
    row(f"fwd  {name}", fl, lambda: gemm_hip.gemm(W, x, cache_a=True), lambda: torch.bmm(W.expand(Bn, O, I), x))
    row(f"dx   {name}", fl, lambda: gemm_hip.gemm(W.t(), dy, cache_a=True),
        lambda: torch.bmm(W.t().expand(Bn, I, O), dy))
    sp = max(1, min(-(-1024 // (-(-O // 128) * -(-I // 128) * Bn)), P // 512, 64))
    row(f"dW   {name} (splits {sp})", fl,
        lambda: gemm_hip.gemm(dy, x.transpose(1, 2), out_dtype=torch.float32, reduce_batch=True, splits=sp),
        lambda: torch.bmm(dy, x.transpose(1, 2)).sum(0))
