"""gemm8 f32x3 on the decoder's largest fp32 1x1-conv shape (b2 W1: 512 -> 2048 channels at
32^2 pixels, batch 32, stride-0 weights), timed with events; run under rocprofv3 --pmc for the
counter passes (tools_dev/gpu_run.sh g8pmc)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch

from torch_utils.ops import gemm_hip

dev = "cuda"
O, I, P, B = 2048, 512, 1024, 32
W = torch.randn(O, I, device=dev)
x = torch.randn(B, I, P, device=dev)
fn = lambda: gemm_hip.gemm(W, x, cache_a=True)
for _ in range(3):
    fn()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(20):
    fn()
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / 20
fl = 2.0 * B * O * I * P
print(f"gemm8 f32x3 {O}x{P}x{I} x{B}: {ms:.3f} ms per call (incl. split3 of x), {fl / ms / 1e9:.1f} TF/s fp32", flush=True)
