"""Per-shape bf16 GEMM microbench of the step's largest products: the SigLIP2-L tower linears
(M = 32 images x 1024 tokens; QKV / O / fc1 (+tanh-GELU) / fc2 with bias) and the decoder's bf16 1x1
data gradients, on gemm9 (csrc/gemm9.hip) against hipBLASLt (torch addmm / _addmm_activation / bmm).
Also fc1 without its epilogue on gemm9, which prices the GELU epilogue. TF/s = FLOPs / time."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch  # noqa: E402

from torch_utils.ops import gemm_hip  # noqa: E402


def bench(fn, iters=int(os.environ.get("TB_ITERS", 20))):
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


def line(name, fl, variants):
    parts = []
    for tag, fn in variants:
        t = bench(fn)
        parts.append(f"{tag} {t * 1e3:7.1f}us {fl / t / 1e9:6.1f}")
    print(f"{name:30s} | " + " | ".join(parts), flush=True)


bf = torch.bfloat16
dev = "cuda"
M = 32768
only = os.environ.get("TB_ONLY", "")
for name, N, K, act in [("qkv", 3072, 1024, None), ("o", 1024, 1024, None), ("fc1", 4096, 1024, "gelu_tanh"),
                        ("fc2", 1024, 4096, None)]:
    if only and name not in only.split(","):
        continue
    x = (torch.randn(M, K, device=dev) * 0.5).to(bf)
    w = (torch.randn(N, K, device=dev) * 0.03).to(bf)
    b = (torch.randn(N, device=dev) * 0.1).to(bf)
    bf32 = b.float()
    fl = 2.0 * M * N * K
    v = [("g9", lambda: gemm_hip.try_gemm(x, w.t(), bias=bf32, bias_dim=1, act=act, route=("g9", 0)))]
    if act is not None:
        v.append(("g9plain", lambda: gemm_hip.try_gemm(x, w.t(), route=("g9", 0))))
        v.append(("blas", lambda: torch._addmm_activation(b, x, w.t(), use_gelu=True)))
    else:
        v.append(("blas", lambda: torch.addmm(b, x, w.t())))
    line(f"tower {name} {M}x{N}x{K}", fl, v)

Bn = 32
for name, O, I, P in [("b3 dx W1", 2048, 512, 4096), ("b3 dx W2", 512, 2048, 4096), ("b4 dx W1", 1024, 256, 16384),
                      ("b4 dx W2", 256, 1024, 16384), ("b5 dx", 512, 128, 65536), ("b5 dx2", 128, 512, 65536)]:
    if only and "dec" not in only.split(","):
        continue
    W = (torch.randn(O, I, device=dev) * 0.05).to(bf)
    dy = torch.randn(Bn, O, P, device=dev).to(bf)
    fl = 2.0 * Bn * O * I * P
    Wt = W.t()
    line(f"{name} {I}x{P}x{O}x{Bn}", fl,
         [("g9", lambda: gemm_hip.try_gemm(Wt, dy, route=("g9", 0))),
          ("blas", lambda: torch.bmm(Wt.unsqueeze(0).expand(Bn, I, O), dy))])
