"""Exact-fp32 GEMM (csrc/sgemm.hip) against hipBLASLt's exact fp32 (torch, TF32 off) on the training step's
library-routed fp32 shapes (tools_dev/opsites.py with OPSITES_OPS, gpurun_out/r6a): the D heads' batch-folded
1-D convs, the 8^2 / 4^2 decoder 1x1s, the adapter's 64-wide linears. Prints us and TF/s for both."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vfm-vae_amd")]
import torch  # noqa: E402

from torch_utils.ops import gemm_hip  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False
DEV = "cuda:0"


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def case(name, A, B, reduce=False, **kw):
    z = max(A.shape[0] if A.dim() == 3 else 1, B.shape[0] if B.dim() == 3 else 1)
    M, K, N = A.shape[-2], A.shape[-1], B.shape[-1]
    fl = 2.0 * z * M * N * K
    if reduce:
        t_lib = timeit(lambda: torch.bmm(A, B).sum(0))
    elif A.dim() == 3 or B.dim() == 3:
        t_lib = timeit(lambda: torch.matmul(A, B))
    else:
        t_lib = timeit(lambda: torch.mm(A, B))
    out = gemm_hip.sgemm(A, B, reduce_batch=reduce, **kw)
    assert out is not None, name
    t_own = timeit(lambda: gemm_hip.sgemm(A, B, reduce_batch=reduce, **kw))
    ref = torch.bmm(A, B).sum(0) if reduce else torch.matmul(A, B)
    err = float((out - ref).abs().max() / ref.abs().max())
    print(f"{name:34s} {M:6d}x{N:6d}x{K:6d}x{z:3d}  sgemm {t_own:8.1f} us {fl / t_own / 1e6:7.1f} TF/s   "
          f"hipBLASLt {t_lib:8.1f} us {fl / t_lib / 1e6:7.1f} TF/s   ratio {t_lib / t_own:5.2f}  err {err:.1e}",
          flush=True)


def sweep(name, A, B, reduce=False):
    """every tile x split for one shape: the best configuration and the heuristic's pick"""
    z = max(A.shape[0] if A.dim() == 3 else 1, B.shape[0] if B.dim() == 3 else 1)
    M, K, N = A.shape[-2], A.shape[-1], B.shape[-1]
    fl = 2.0 * z * M * N * K
    res = []
    for tile in range(8):
        for sp in (1, 2, 3, 4, 6, 8, 12):
            try:
                t = timeit(lambda: gemm_hip.sgemm(A, B, reduce_batch=reduce, tile=tile, splits=sp), iters=10)
            except Exception as e:  # noqa: BLE001
                continue
            res.append((t, tile, sp))
    res.sort()
    auto = timeit(lambda: gemm_hip.sgemm(A, B, reduce_batch=reduce))
    print(f"  sweep {name:28s} best " + "  ".join(f"t{c}s{sp} {t:.1f}us {fl / t / 1e6:.0f}TF" for t, c, sp in res[:4])
          + f"   auto {auto:.1f}us {fl / auto / 1e6:.0f}TF", flush=True)


def main():
    g = torch.Generator(device=DEV).manual_seed(0)
    r = lambda *s: torch.randn(*s, device=DEV, generator=g)
    B, C, L = 32, 384, 196
    cols1, cols9 = r(C, B * L), r(9 * C, B * L)
    w1, w9 = r(C, C), r(C, 9 * C)
    gy = r(C, B * L)
    case("dhead fwd k1", w1, cols1)
    case("dhead fwd k9", w9, cols9)
    case("dhead dx k1", w1.t(), gy)
    case("dhead dx k9", w9.t(), gy)
    case("dhead dW k1", gy, cols1.t())
    case("dhead dW k9", gy, cols9.t())
    case("dhead fwd cls", r(1, C), cols1)
    x64 = r(32, 512, 64)
    case("dec 8^2 1x1 512->2048", r(2048, 512), x64)
    case("dec 8^2 1x1 2048->512", r(512, 2048), r(32, 2048, 64))
    case("dec 8^2 1x1 dx 2048->512", r(2048, 512).t(), r(32, 2048, 64))
    case("dec 4^2 1x1 512->2048", r(2048, 512), r(32, 512, 16))
    case("dec 4^2 1x1 512->8192", r(8192, 512), r(32, 512, 16))
    case("dec 8^2 dW 2048x512", r(32, 2048, 64), r(32, 64, 512), reduce=True)
    case("adapter lin 1024->64", r(32768, 1024), r(64, 1024).t())
    case("adapter lin 128->64", r(32768, 128), r(64, 128).t())
    case("adapter lin dW 64x1024", r(32768, 64).t(), r(32768, 1024))
    case("adapter lin dx 64->1024", r(32768, 64), r(64, 1024))
    case("style fc 512->1536", r(32, 512), r(1536, 512).t())
    case("gram 256x256x1024", r(32, 256, 1024), r(32, 1024, 256))
    case("dino patch 768->384", r(6272, 768), r(384, 768).t())
    N = 4096
    case("square 4096", r(N, N), r(N, N))
    case("square 4096 tn", r(N, N), r(N, N).t())
    case("square 4096 nt", r(N, N).t(), r(N, N))
    if os.environ.get("SWEEP", "1") == "1":
        sweep("dhead fwd k9", w9, cols9)
        sweep("dhead fwd k1", w1, cols1)
        sweep("dhead dx k9", w9.t(), gy)
        sweep("dhead dW k9", gy, cols9.t())
        sweep("dhead dW k1", gy, cols1.t())
        sweep("dec 8^2 1x1 2048->512", r(512, 2048), r(32, 2048, 64))
        sweep("dec 8^2 1x1 512->2048", r(2048, 512), x64)
        sweep("adapter lin 1024->64", r(32768, 1024), r(64, 1024).t())
        sweep("adapter lin dx 64->1024", r(32768, 64), r(64, 1024))
        sweep("gram 256x256x1024", r(32, 256, 1024), r(32, 1024, 256))


if __name__ == "__main__":
    main()
