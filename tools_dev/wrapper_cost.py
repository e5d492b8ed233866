"""Host time per call of the op wrappers on the training path (no synchronisation inside the loop: the launches
queue, the GPU runs behind; the numbers are the Python + launch cost the host pays per op), against a bare
ctypes launch of the same kernel. Small tensors so the GPU never throttles the host queue.

  python tools_dev/wrapper_cost.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vfm-vae_amd")]
import torch  # noqa: E402

from torch_utils import custom_ops  # noqa: E402
from torch_utils.ops import gemm_hip, decoder_ops  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)


def cost(label, fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    us = (time.perf_counter() - t) / n * 1e6
    torch.cuda.synchronize()
    print(f"{label:60s} {us:7.2f} us/call", flush=True)


g = torch.Generator().manual_seed(0)
a16 = torch.randn(256, 256, generator=g).bfloat16().to(dev)
b16 = torch.randn(256, 256, generator=g).bfloat16().to(dev)
a32 = torch.randn(4, 256, 256, generator=g).to(dev)
w32 = torch.randn(256, 256, generator=g).to(dev)
x32n = torch.randn(4, 64, 64, generator=g).to(dev)
w32n = torch.randn(64, 64, generator=g).to(dev)
out16 = torch.empty(256, 256, dtype=torch.bfloat16, device=dev)
lib = custom_ops.get_native()
st = custom_ops.stream_ptr(dev)

cost("try_gemm bf16 256^3 (gemm9)", lambda: gemm_hip.try_gemm(a16, b16.t(), auto=True))
cost("vfm_gemm9 bare ctypes", lambda: lib.vfm_gemm9(a16.data_ptr(), b16.data_ptr(), out16.data_ptr(), None, 1, 256, 256,
                                                   256, 1, 1, 256, 0, 1, 256, 0, 256, 0, 1.0, 0.0, 0, 0, st))
cost("try_gemm fp32 W[256,256] x[4,256,256] (f32x6)", lambda: gemm_hip.try_gemm(w32, a32, auto=True))
cost("try_gemm fp32 W[64,64] x[4,64,64] (sgemm)", lambda: gemm_hip.try_gemm(w32n, x32n, auto=True))
cost("torch.empty(256,256)", lambda: torch.empty(256, 256, device=dev))
cost("custom_ops.stream_ptr", lambda: custom_ops.stream_ptr(dev))
xg = torch.randn(4, 64, 32, 32, generator=g).to(dev)
wg = torch.randn(64, generator=g).to(dev)
bg = torch.randn(64, generator=g).to(dev)
cost("decoder_ops.group_norm fp32 [4,64,32,32]", lambda: decoder_ops.group_norm(xg, 32, wg, bg))
cost("torch group_norm fp32 [4,64,32,32]", lambda: torch.nn.functional.group_norm(xg, 32, wg, bg))
cost("decoder_ops.scale_bias_gelu fp32", lambda: decoder_ops.scale_bias_gelu(xg.view(4, 64, -1), None, bg))
cost("torch x + y", lambda: xg + xg)
