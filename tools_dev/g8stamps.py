"""Microbench: where a gemm8 tile's time goes (s_memrealtime stamps (100 MHz) written by the kernel when a stamp
buffer is set, vfm_gemm8_set_stamps): prologue (first K-tile landed), main loop, epilogue, and the
share of the launch's wall time the blocks are resident (block dispatch gaps)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch

from torch_utils import custom_ops
from torch_utils.ops import gemm_hip

lib = custom_ops.get_native()


def rnd(*shape):
    return (torch.rand(*shape, device="cuda") * 2 - 1).to(torch.bfloat16)


def run(M, N, K, sched, out_dtype):
    A, W = rnd(M, K), rnd(N, K)
    tiles = -(-M // 256) * -(-N // 256)
    nblk = tiles
    st = torch.zeros(nblk * 16, dtype=torch.int64, device="cuda")
    f = lambda: gemm_hip.try_gemm(A, W.t(), out_dtype=out_dtype, route=("g8", 0))
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        f()
    e.record()
    torch.cuda.synchronize()
    wall_us = s.elapsed_time(e) / 5 * 1e3
    lib.vfm_gemm8_set_stamps(st.data_ptr())
    f()
    torch.cuda.synchronize()
    lib.vfm_gemm8_set_stamps(None)
    x = st.view(nblk, 16).cpu()
    t0 = x[:, 0]
    span = float(x[x > 0].max() - t0.min())
    pro = (x[:, 1] - x[:, 0]).double().mean()
    loops, epis, drains = [], [], []
    for b in range(nblk):
        loops.append(float(x[b, 2] - x[b, 1]))
        epis.append(float(x[b, 3] - x[b, 2]))
        drains.append(float(x[b, 4] - x[b, 3]))
    loop = sum(loops) / len(loops)
    epi = sum(epis) / len(epis)
    drain = sum(drains) / len(drains)
    busy = float(((x.max(1).values - x[:, 0]).double()).sum())
    clk = 100.0                 # s_memrealtime: 100 MHz
    print(f"{M}x{N}x{K} {str(out_dtype)[6:]:8s} wall {wall_us:8.1f}us "
          f"span {span / clk:8.1f}us | per tile: prologue {pro / clk:6.2f}us loop {loop / clk:7.2f}us "
          f"epilogue {epi / clk:6.2f}us + drain {drain / clk:6.2f}us | resident {busy / (span * min(nblk, 256)):.2f}", flush=True)


if os.environ.get("G8ST_SCALE"):
    # main-loop time per K-tile vs the number of tiles running at once (L2 / fabric contention)
    for M, N in [(512, 512), (1024, 1024), (2048, 2048), (4096, 4096), (8192, 8192)]:
        run(M, N, 4096, 1, torch.float32)
else:
    for M, N, K in [(8192, 8192, 64), (8192, 8192, 1024), (8192, 8192, 4096), (32768, 3072, 1024),
                    (32768, 1024, 4096)]:
        for odt in (torch.bfloat16, torch.float32):
            run(M, N, K, 1, odt)
