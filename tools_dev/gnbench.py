"""GroupNorm backward (csrc/decoder.hip gn_bwd) on the ConvNeXt layers' bf16 shapes: time per launch and the
fraction of 8 TB/s at its algorithmic bytes (x, dy read once, dx written once), for the workgroup cap given by
VFM_GN_BWD_WGS (0: one workgroup per (sample, group)). Run once per cap value (the cap is read at first use).

  VFM_GN_BWD_WGS=256 python tools_dev/gnbench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vfm-vae_amd")]
import torch  # noqa: E402

from torch_utils import custom_ops  # noqa: E402

lib = custom_ops.get_native()
dev = torch.device("cuda", 0)
BF16 = custom_ops.DTYPE_CODES[torch.bfloat16]
for C, H in ((128, 256), (256, 128), (512, 64)):
    B, G = 32, 32
    x = torch.randn(B, C, H, H, device=dev).bfloat16()
    dy = torch.randn(B, C, H, H, device=dev).bfloat16()
    dx = torch.empty_like(x)
    mean = torch.randn(B * G, device=dev)
    rstd = torch.rand(B * G, device=dev) + 0.5
    w = torch.randn(C, device=dev)
    b = torch.randn(C, device=dev)
    s = torch.randn(B, C, device=dev)
    dwp, dbp, ds = (torch.empty(B, C, device=dev) for _ in range(3))
    st = torch.cuda.current_stream().cuda_stream

    def run():
        custom_ops.check(lib.vfm_group_norm_bwd(x.data_ptr(), dy.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                                                w.data_ptr(), b.data_ptr(), s.data_ptr(), dx.data_ptr(), dwp.data_ptr(),
                                                dbp.data_ptr(), ds.data_ptr(), BF16, BF16, B, C, G, H * H, st),
                         "vfm_group_norm_bwd")
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    e0.record()
    for _ in range(n):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / n
    nbytes = 3 * x.numel() * 2
    print(f"C={C:4d} {H}x{H} cap={os.environ.get('VFM_GN_BWD_WGS', '0'):>5s}: {us:8.1f} us  "
          f"{nbytes / us / 1e3:7.0f} GB/s  {nbytes / us / 1e3 / 8000:.2f} of 8 TB/s", flush=True)
