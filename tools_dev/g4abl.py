"""gemm4 K-loop ablations on the SigLIP qkv shape: full, no operand loads (LDS stage reused), no MFMAs,
neither -- where a K-tile's time goes (vfm_gemm4_set_debug)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch

from torch_utils import custom_ops
from torch_utils.ops import gemm_hip

lib = custom_ops.get_native()


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


for M, N, K in [(32768, 3072, 1024), (32768, 3072, 64), (32768, 3072, 4096)][:0]:
    A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    W = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    fl = 2.0 * M * N * K
    res = []
    for dbg in (0, 1, 2, 3):
        lib.vfm_gemm4_set_debug(dbg)
        t = timeit(lambda: gemm_hip.try_gemm(A, W.t(), route=("g4", 0)))
        res.append(f"dbg{dbg} {t:8.1f}us ({t / 6 / (K // 64):5.2f} us/K-tile)")
    lib.vfm_gemm4_set_debug(0)
    t8 = timeit(lambda: gemm_hip.try_gemm(A, W.t(), route=("g8", 0)))
    tb = timeit(lambda: A @ W.t())
    print(f"{M}x{N}x{K}: " + " | ".join(res) + f" | g8 {t8:8.1f}us | blas {tb:8.1f}us", flush=True)
