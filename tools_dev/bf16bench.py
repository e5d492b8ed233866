"""Microbench of the decoder's bf16 1x1 convolutions at batch 32 (blocks 3-4, the ConvNeXt MLP widths):
forward W . x[b], data gradient W^T . dy[b] and the batch-reduced weight gradient sum_b dy[b] x[b]^T,
on hipBLASLt (torch.bmm; the weight gradient as bmm + sum(0) in fp32, what decoder_hip does) and on our
kernels (gemm8 batched / batch-reduced split-K)."""
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
    return s.elapsed_time(e) / iters


def line(name, fl, variants):
    parts = []
    for tag, fn in variants:
        try:
            t = bench(fn)
            parts.append(f"{tag} {t * 1e3:7.1f}us {fl / t / 1e9:6.1f}")
        except Exception as ex:  # noqa: BLE001
            parts.append(f"{tag} ERR {type(ex).__name__}: {ex}"[:80])
    print(f"{name:34s} | " + " | ".join(parts), flush=True)


dev = "cuda"
bf = torch.bfloat16
Bn = 32
print("TF/s = FLOPs / time", flush=True)
SHAPES = [("b3 W1 512->2048 @64^2", 2048, 512, 4096), ("b3 W2 2048->512 @64^2", 512, 2048, 4096),
          ("b4 W1 256->1024 @128^2", 1024, 256, 16384), ("b4 W2 1024->256 @128^2", 256, 1024, 16384),
          ("b5 W1 128->512 @256^2", 512, 128, 65536), ("b5 W2 512->128 @256^2", 128, 512, 65536)]
only_dw = os.environ.get("BF16BENCH_DW_ONLY") == "1"
for name, O, I, P in SHAPES:
    W = (torch.randn(O, I, device=dev) * 0.05).to(bf)
    x = torch.randn(Bn, I, P, device=dev).to(bf)
    dy = torch.randn(Bn, O, P, device=dev).to(bf)
    fl = 2.0 * Bn * O * I * P
    if only_dw:
        V = Bn * (P // 64)
        vs = [("blas", lambda: torch.bmm(dy, x.transpose(1, 2), out_dtype=torch.float32).sum(0))]
        for S in (16, 32, 64, 128, 256):
            vs.append((f"g8r{S}", (lambda S=S: gemm_hip.try_gemm(dy, x.transpose(1, 2), out_dtype=torch.float32,
                                                                  reduce_batch=True, route=("g8", -(-V // S))))))
        line(f"dW  {name}", fl, vs)
        continue
    line(f"fwd {name}", fl, [("blas", lambda: torch.bmm(W.expand(Bn, O, I), x)),
                             ("g8", lambda: gemm_hip.try_gemm(W, x, route=("g8", 0)))])
    line(f"dx  {name}", fl, [("blas", lambda: torch.bmm(W.t().expand(Bn, I, O), dy)),
                             ("g8", lambda: gemm_hip.try_gemm(W.t(), dy, route=("g8", 0)))])
    V = Bn * (P // 64)
    vs = [("blas", lambda: torch.bmm(dy, x.transpose(1, 2), out_dtype=torch.float32).sum(0))]
    for S in (8, 16, 32, 64):
        vs.append((f"g8r{S}", (lambda S=S: gemm_hip.try_gemm(dy, x.transpose(1, 2), out_dtype=torch.float32,
                                                              reduce_batch=True, route=("g8", -(-V // S))))))
    vs.append(("g128r", lambda: gemm_hip.try_gemm(dy, x.transpose(1, 2), out_dtype=torch.float32,
                                                  reduce_batch=True, splits=1, route=("g128", 1))))
    line(f"dW  {name}", fl, vs)
