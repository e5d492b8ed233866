"""Microbench of the fp32-equivalent (f32x6) GEMM routes on the training step's fp32 shapes
(from the VFM_TIMER_SHAPES=1 bench breakdown): the 256-tile kernel direct / split-K, the 128-tile
kernel (split in registers), and hipBLASLt's exact fp32 GEMM for reference. Times include the
operand split of the activation (weights cached, as in the step)."""
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


def line(name, fl, variants):
    parts = []
    for tag, fn in variants:
        try:
            t = bench(fn)
            parts.append(f"{tag} {t * 1e3:7.1f}us {fl / t / 1e9:6.1f}")
        except Exception as ex:  # noqa: BLE001
            parts.append(f"{tag} ERR {type(ex).__name__}")
    print(f"{name:40s} | " + " | ".join(parts), flush=True)


dev = "cuda"
torch.backends.cuda.matmul.allow_tf32 = False
gemm_hip.SPLIT8 = True
print("TF/s = fp32 FLOPs / time", flush=True)

# token-major linears: x [M, K] @ W^T (W [N, K], cached split), DINO ViT-S (M = 32 * 197) and adapter
for name, M, N, K in [("dino fc2 fwd", 6304, 384, 1536), ("dino qkv fwd", 6304, 1152, 384),
                      ("dino proj fwd", 6304, 384, 384), ("dino fc1 fwd", 6304, 1536, 384),
                      ("dino fc2 dx (dy W)", 6304, 1536, 384), ("adapter qkv fwd", 32768, 3072, 1024)]:
    x = torch.randn(M, K, device=dev)
    W = torch.randn(N, K, device=dev)
    fl = 2.0 * M * N * K
    V = 6 * (K // 64)
    vs = [("auto", lambda: gemm_hip.gemm(x, W.t(), cache_b=True, auto=True)),
          ("g8", lambda: gemm_hip.gemm(x, W.t(), cache_b=True, route=("g8", 0)))]
    for S in (2, 3, 4, 6, 8):
        if V // S >= 4:
            vs.append((f"g8s{S}", (lambda S=S: gemm_hip.gemm(x, W.t(), cache_b=True, route=("g8", -(-V // S))))))
    vs += [("g128", lambda: gemm_hip.gemm(x, W.t(), cache_b=True, route=("g128", 1))),
           ("blas", lambda: x @ W.t())]
    line(name, fl, vs)

# decoder fp32 1x1 convs at batch 32: W [O, I] . x[b] [I, P]; dW = sum_b dy[b] x[b]^T
for name, O, I, P in [("b2 W1 512->2048 @32^2", 2048, 512, 1024), ("b2 W2 2048->512 @32^2", 512, 2048, 1024),
                      ("b1 W1 512->2048 @16^2", 2048, 512, 256), ("b0 W1 512->2048 @8^2", 2048, 512, 64),
                      ("b1 up 512->2048 @16^2", 2048, 512, 144)]:
    Bn = 32
    W = torch.randn(O, I, device=dev)
    x = torch.randn(Bn, I, P, device=dev)
    dy = torch.randn(Bn, O, P, device=dev)
    fl = 2.0 * Bn * O * I * P
    line(f"fwd {name}", fl, [("auto", lambda: gemm_hip.gemm(W, x, cache_a=True, auto=True)),
                             ("g8", lambda: gemm_hip.gemm(W, x, cache_a=True, route=("g8", 0))),
                             ("g128", lambda: gemm_hip.gemm(W, x, cache_a=True, route=("g128", 1))),
                             ("blas", lambda: torch.bmm(W.expand(Bn, O, I), x))])
    Vr = 6 * Bn * (P // 64) if P % 64 == 0 else 0
    vs = [("g128r", lambda: gemm_hip.gemm(dy, x.transpose(1, 2), out_dtype=torch.float32, reduce_batch=True,
                                          splits=1, route=("g128", 1)))]
    for S in (8, 16, 32):
        if Vr:
            vs.append((f"g8r{S}", (lambda S=S: gemm_hip.gemm(dy, x.transpose(1, 2), out_dtype=torch.float32,
                                                              reduce_batch=True, route=("g8", -(-Vr // S))))))
    vs.append(("blas", lambda: torch.bmm(dy, x.transpose(1, 2)).sum(0)))
    line(f"dW  {name}", fl, vs)

# adapter weight gradient: dW [3072, 1024] = dy^T [3072, 32768] x [32768, 1024]
M, N, K = 3072, 1024, 32768
dy = torch.randn(K, M, device=dev)
x = torch.randn(K, N, device=dev)
fl = 2.0 * M * N * K
vs = []
for sp in (4, 6, 8, 16):
    vs.append((f"g128s{sp}", (lambda sp=sp: gemm_hip.gemm(dy.t(), x, out_dtype=torch.float32, route=("g128", sp)))))
for S in (2, 4, 8):
    vs.append((f"g8s{S}", (lambda S=S: gemm_hip.gemm(dy.t(), x, out_dtype=torch.float32,
                                                      route=("g8", -(-6 * (K // 64) // S))))))
vs.append(("blas", lambda: dy.t() @ x))
line("adapter qkv dW", fl, vs)
