"""Microbench of the f32x6 products whose route the gemm9 planner (gemm_hip.G9F_PLAN) would change: the adapter's
token-major weight gradients (M x N outputs over K = 32 x 1024 tokens, A = dy^T M-contiguous, B = x N-contiguous)
and the DINO tower's few-tile products, on the default route (128-tile kernel split-K / gemm9 unsplit) against
gemm9 with the planner's K split."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch  # noqa: E402

from torch_utils.ops import gemm_hip  # noqa: E402


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
    return s.elapsed_time(e) / iters * 1e3


g = torch.Generator().manual_seed(0)
cases = [("adapter dW qkv", 3072, 1024, 32768, "ff"), ("adapter dW w0/w1", 4096, 1024, 32768, "ff"),
         ("adapter dW w2", 1024, 4096, 32768, "ff"), ("adapter dW proj", 1024, 1024, 32768, "ff"),
         ("dino fc2/proj", 6304, 384, 1536, "tt"), ("dino fc2 dx", 6304, 384, 1536, "tf"),
         ("dino qkv", 6304, 1152, 384, "tt"), ("dino proj", 6304, 384, 384, "tt")]
ZB = 32
bcases = [("b1 pwconv2", 512, 256, 2048, "tf"), ("b1 pwconv1 dx", 512, 256, 2048, "tf"), ("b2 small", 512, 1024, 2048, "tf")]
for name, M, N, K, lay in cases:
    A = (torch.rand(K, M, generator=g) * 2 - 1).cuda().t() if lay[0] == "f" else (torch.rand(M, K, generator=g) * 2 - 1).cuda()
    B = (torch.rand(K, N, generator=g) * 2 - 1).cuda() if lay[1] == "f" else (torch.rand(N, K, generator=g) * 2 - 1).cuda().t()
    res = []
    for plan in (False, True):
        gemm_hip.G9F_PLAN = plan
        t = bench(lambda: gemm_hip.try_gemm(A, B, out_dtype=torch.float32, auto=True))
        res.append(f"{'g9 split' if plan else 'default '} {t:8.1f}us {2.0 * M * N * K / t / 1e6:6.1f} TF/s")
    print(f"{name:18s} {M}x{N}x{K} {lay} S={gemm_hip._splits9f(M, N, K, 1, False)} | " + " | ".join(res), flush=True)
for name, M, N, K, lay in bcases:
    A = (torch.rand(M, K, generator=g) * 2 - 1).cuda()
    B = (torch.rand(ZB, K, N, generator=g) * 2 - 1).cuda()
    res = []
    for deep in (False, True):
        gemm_hip.G9F_PLAN, gemm_hip.DEEP9F = False, deep
        t = bench(lambda: gemm_hip.try_gemm(A, B, out_dtype=torch.float32, auto=True))
        res.append(f"{'g9 bsplit' if deep else 'default  '} {t:8.1f}us {2.0 * M * N * K * ZB / t / 1e6:6.1f} TF/s")
    ref = torch.matmul(A.double(), B.double())
    out = gemm_hip.try_gemm(A, B, out_dtype=torch.float32, auto=True)
    e = float((out.double() - ref).abs().max() / ref.abs().max())
    print(f"{name:18s} {M}x{N}x{K}x{ZB} {lay} S={gemm_hip._deep9f(M, N, K, ZB, False)} err {e:.1e} | " + " | ".join(res), flush=True)
