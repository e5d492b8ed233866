"""Driver for rocprofv3 PMC passes over csrc/sgemm.hip: a few step shapes, fixed (tile, split), 20 launches each."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vfm-vae_amd")]
import torch  # noqa: E402

from torch_utils.ops import gemm_hip  # noqa: E402

DEV = "cuda:0"
g = torch.Generator(device=DEV).manual_seed(0)
r = lambda *s: torch.randn(*s, device=DEV, generator=g)
which = os.environ.get("SGP", "dec512to2048")
cases = {"square_nt": (r(4096, 4096).t(), r(4096, 4096), 0, 1),
         "dec2048to512": (r(512, 2048), r(32, 2048, 64), 3, 1),
         "dec512to2048": (r(2048, 512), r(32, 512, 64), 3, 1),
         "dheadk9": (r(384, 3456), r(3456, 6272), 1, 5)}
for name in which.split(","):
    A, B, tile, sp = cases[name]
    for _ in range(20):
        gemm_hip.sgemm(A, B, tile=tile, splits=sp)
    torch.cuda.synchronize()
    print(name, "done", flush=True)
