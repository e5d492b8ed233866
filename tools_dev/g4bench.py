"""Microbench: the one-wave-per-SIMD bf16 GEMM (csrc/gemm4.hip) vs gemm8 (csrc/gemm8.hip) vs hipBLASLt
(torch) on the hot path's bf16 shapes: the SigLIP2-L tower's linears at 32 x 1024 tokens and the decoder's
bf16 1x1 convolutions at batch 32 (forward and data gradient). Interleaved rounds in one process, random
[-1, 1) operands; every shape is first checked against an fp32 product of the same bf16 operands."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch

from torch_utils.ops import gemm_hip

ROUNDS = int(os.environ.get("G4_ROUNDS", "3"))
ONLY = os.environ.get("G4_ONLY", "")


def rnd(*shape):
    return (torch.rand(*shape, device="cuda") * 2 - 1).to(torch.bfloat16)


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


KINDS = tuple(os.environ.get("G4_KINDS", "g9,g8").split(","))


def case(name, A, B, ref_fn, torch_fn, flops, kinds=KINDS):
    if ONLY and ONLY not in name:
        return
    ref = ref_fn()
    def run(k):
        if k == "g9np":                     # gemm9, one workgroup per tile
            prev = gemm_hip._lib.vfm_gemm9_set_mode(0)
            try:
                return gemm_hip.try_gemm(A, B, route=("g9", 0))
            finally:
                gemm_hip._lib.vfm_gemm9_set_mode(prev)
        return gemm_hip.try_gemm(A, B, route=(k, 0))
    fns = {k: (lambda k=k: run(k)) for k in kinds}
    fns["blas"] = torch_fn
    errs = {}
    for k in kinds:
        out = fns[k]()
        if out is None:
            print(f"{name}: {k} returned None", flush=True)
            return
        errs[k] = float((out.float() - ref).abs().max() / ref.abs().max())
    ts = {k: [] for k in fns}
    for _ in range(ROUNDS):
        for k, f in fns.items():
            ts[k].append(timeit(f))
    parts = []
    for k in fns:
        t = sorted(ts[k])[len(ts[k]) // 2]
        e = f" err {errs[k]:.1e}" if k in errs else ""
        parts.append(f"{k} {t:8.1f}us {flops / t / 1e6:7.1f} TF/s{e}")
    print(f"{name:36s} " + " | ".join(parts), flush=True)


torch.manual_seed(0)
for name, M, N, K in [("siglip qkv 32768x3072x1024", 32768, 3072, 1024),
                      ("siglip o 32768x1024x1024", 32768, 1024, 1024),
                      ("siglip fc1 32768x4096x1024", 32768, 4096, 1024),
                      ("siglip fc2 32768x1024x4096", 32768, 1024, 4096),
                      ("square 8192^3", 8192, 8192, 8192)]:
    A, W = rnd(M, K), rnd(N, K)
    case(name, A, W.t(), lambda: A.float() @ W.float().t(), lambda: A @ W.t(), 2.0 * M * N * K)
    del A, W

# decoder bf16 1x1 convs at batch 32: (tag, O, I, P): y[b] = W x[b] (W [O, I], x [I, P]); dx[b] = W^T dy[b]
for tag, O, I, P in [("b3 W1 512->2048 @64^2", 2048, 512, 4096), ("b3 W2 2048->512 @64^2", 512, 2048, 4096),
                     ("b4 W1 256->1024 @128^2", 1024, 256, 16384), ("b4 W2 1024->256 @128^2", 256, 1024, 16384)]:
    Bn = 32
    W = rnd(O, I)
    x, dy = rnd(Bn, I, P), rnd(Bn, O, P)
    fl = 2.0 * Bn * O * I * P
    case(f"fwd {tag}", W, x, lambda: torch.matmul(W.float(), x.float()), lambda: torch.bmm(W.expand(Bn, O, I), x), fl)
    case(f"dx  {tag}", W.t(), dy, lambda: torch.matmul(W.t().float(), dy.float()),
         lambda: torch.bmm(W.t().expand(Bn, I, O), dy), fl)
    del W, x, dy
    torch.cuda.empty_cache()

# ragged edges and a single K-tile (correctness only, small)
for M, N, K in [(300, 200, 64), (257, 520, 128), (1000, 136, 192)]:
    A, W = rnd(M, K), rnd(N, K)
    ref = A.float() @ W.float().t()
    out = gemm_hip.try_gemm(A, W.t(), route=(KINDS[0], 0))
    err = float((out.float() - ref).abs().max() / ref.abs().max())
    print(f"ragged {M}x{N}x{K}: err {err:.1e}", flush=True)
