"""Microbench: LPIPS VGG16 taps forward (64 images) and forward+backward (32 images) at 256^2,
HIP implicit-GEMM stack (torch_utils/ops/vgg_hip.py) vs MIOpen (VFM_LPIPS_VGG=torch path)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch

from training.lpips import vgg16
from torch_utils.ops import kernel_timer

os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")


def bench(fn, iters=5):
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


net = vgg16(pretrained=False).cuda()
x64 = torch.randn(64, 3, 256, 256, device="cuda")
x32 = torch.randn(32, 3, 256, 256, device="cuda", requires_grad=True)
GF = 2 * 20.1e9 * 1.0          # conv flops per image forward (sum over the 13 layers)
for impl in ("hip", "torch"):
    type(net).impl = impl
    with torch.no_grad():
        tf = bench(lambda: net(x64))

    def fb():
        outs = net(x32)
        torch.autograd.backward(list(outs), [torch.ones_like(o) for o in outs])

    tb = bench(fb)
    print(f"{impl:6s} fwd 64 img {tf:7.2f} ms ({64 * GF / tf / 1e9:6.1f} TF/s)   fwd+bwd 32 img {tb:7.2f} ms", flush=True)
type(net).impl = "hip"
kernel_timer.enable(True)
with torch.no_grad():
    net(x64)
for k, v in sorted(kernel_timer.summary().items(), key=lambda kv: -kv[1]["total_ms"]):
    print(f"  {k:40s} {v['total_ms']:7.3f} ms  {v['flops'] / v['total_ms'] / 1e9:7.1f} TF/s")

# kernel breakdown of one HIP forward + backward (32 images)
from torch.profiler import profile, ProfilerActivity
type(net).impl = "hip"
fb()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CUDA]) as prof:
    fb()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=25, max_name_column_width=70))
