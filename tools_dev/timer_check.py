"""Check: kernel_timer's dispatch-bound events (vfm_timer_arm / hipExtLaunchKernelGGL) against rocprofv3's
kernel trace for the same launches. Run under `rocprofv3 --kernel-trace --stats` and compare the printed
per-launch averages with the stats CSV."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch

from torch_utils.ops import gemm_hip, kernel_timer

A = torch.randn(32768, 1024, device="cuda")
W = torch.randn(3072, 1024, device="cuda")
Ab, Wb = A.bfloat16(), W.bfloat16()
for _ in range(3):
    gemm_hip.try_gemm(A, W.t(), route=("g8", 0), cache_b=True)
    gemm_hip.try_gemm(Ab, Wb.t(), route=("g9", 0))
torch.cuda.synchronize()
kernel_timer.enable(True, 1)
for i in range(20):
    gemm_hip.try_gemm(A, W.t(), route=("g8", 0), cache_b=True)
    gemm_hip.try_gemm(Ab, Wb.t(), route=("g9", 0))
    if i % 5 == 0:
        torch.cuda.synchronize()          # idle gaps in front of some launches: the events must not see them
kernel_timer.enable(False)
for k, v in kernel_timer.summary().items():
    print(f"{k:40s} launches {v['launches']:3d} avg {v['total_ms'] * 1e3 / v['launches']:9.2f} us", flush=True)
