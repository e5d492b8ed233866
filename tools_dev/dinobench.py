"""Microbench of the DINO ViT-S tower's fp32 linears (token-major, M = 32 images x 197 tokens = 6304)
on the f32x6 routes: the 256-tile kernel direct / split-K, the 128-tile kernel direct / split-K, and
hipBLASLt's exact fp32 GEMM. Calls cycle over 4 distinct activation tensors so the 256-tile kernel's
planar piece split of the activation is re-done each time (as in the step: its cached pieces are dropped
before each call); weights are cached."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch  # noqa: E402

from torch_utils.ops import gemm_hip  # noqa: E402


def bench(fn, iters=20):
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


torch.backends.cuda.matmul.allow_tf32 = False
print("TF/s = fp32 FLOPs / time", flush=True)
M = 6304
for name, N, K in [("qkv fwd / proj-in", 1152, 384), ("proj fwd / dx", 384, 384), ("fc1 fwd / fc2 dx", 1536, 384),
                   ("fc2 fwd / fc1 dx", 384, 1536), ("qkv dx", 384, 1152)]:
    xs = [torch.randn(M, K, device="cuda") for _ in range(4)]
    x = xs[0]
    W = torch.randn(N, K, device="cuda")
    fl = 2.0 * M * N * K
    it = [0]

    def call(route):
        it[0] += 1
        xi = xs[it[0] % 4]
        xi.__dict__.pop("_vfm_planar", None)
        return gemm_hip.gemm(xi, W.t(), cache_b=True, auto=route is None, route=route)

    parts = []
    variants = [("auto", None), ("g8", ("g8", 0))]
    V = 6 * (K // 64)
    for S in (2, 3, 4):
        variants.append((f"g8s{S}", ("g8", -(-V // S))))
    for S in (1, 2, 3, 4):
        variants.append((f"g128s{S}", ("g128", S)))
    for tag, route in variants:
        try:
            t = bench(lambda: call(route))
            parts.append(f"{tag} {t * 1e3:6.1f}us {fl / t / 1e9:5.1f}")
        except Exception as ex:  # noqa: BLE001
            parts.append(f"{tag} ERR {type(ex).__name__}")
    t = bench(lambda: x @ W.t())
    parts.append(f"blas {t * 1e3:6.1f}us {fl / t / 1e9:5.1f}")
    print(f"{name:18s} [{M}x{N}x{K}] | " + " | ".join(parts), flush=True)
