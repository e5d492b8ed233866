"""One gemm8 bf16 TN shape (env G8_M/G8_N/G8_K, default 8192 x 8192 x 4096), 10 timed calls: the
target of the rocprofv3 --pmc passes of tools_dev/gpu_run.sh g8pmc1."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch

from torch_utils.ops import gemm_hip

M, N, K = (int(os.environ.get(k, d)) for k, d in (("G8_M", 8192), ("G8_N", 8192), ("G8_K", 4096)))
Z = int(os.environ.get("G8_Z", 1))
KIND = os.environ.get("G8_KIND", "g8")          # g8 / g9 / g9f (f32x6 on gemm9) / blas (hipBLASLt through torch)
if KIND == "g9f":
    gemm_hip.G9_F32, KIND = True, "g8"
dt = torch.float32 if os.environ.get("G8_DT", "bf16") == "f32" else torch.bfloat16   # f32: the f32x6 products
if Z > 1:   # the decoder's 1x1 conv form: shared weight [M, K] times per-sample planes [Z, K, N]
    A = (torch.rand(M, K, device="cuda") * 2 - 1).to(dt)
    X = (torch.rand(Z, K, N, device="cuda") * 2 - 1).to(dt)
    fn = lambda: gemm_hip.try_gemm(A, X, route=(KIND, 0))
else:
    A = (torch.rand(M, K, device="cuda") * 2 - 1).to(dt)
    W = (torch.rand(N, K, device="cuda") * 2 - 1).to(dt)
    fn = (lambda: gemm_hip.try_gemm(A, W.t(), route=(KIND, 0))) if KIND != "blas" else (lambda: A @ W.t())
M = M * Z
for _ in range(3):
    fn()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(10):
    fn()
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / 10
print(f"{KIND} {dt} {M}x{N}x{K}: {ms * 1e3:.1f} us, {2.0 * M * N * K / ms / 1e9:.1f} TF/s", flush=True)
