"""Cache behaviour of the planar piece splits (gemm_hip._planar) over one fp32 pointwise conv forward + backward
(decoder_hip.pointwise): every call printed with the operand's base tensor identity, version and hit / miss."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vfm-vae_amd")]
import torch  # noqa: E402

from torch_utils.ops import decoder_hip, gemm_hip  # noqa: E402

_orig = gemm_hip._planar


def _planar(t3, stream):
    base = t3._base if t3._base is not None else t3
    before = getattr(base, "_vfm_planar", None)
    out = _orig(t3, stream)
    after = getattr(base, "_vfm_planar", None)
    node = torch._C._current_autograd_node()
    print(f"  planar view {tuple(t3.shape)} base id {id(base):x} {tuple(base.shape)} ptr {base.data_ptr():x} "
          f"v{base._version} {'HIT' if after is before and after is not None else 'MISS'} "
          f"{'(' + node.name() + ')' if node is not None else '(fwd)'}", flush=True)
    return out


gemm_hip._planar = _planar

dev = torch.device("cuda", 0)
w = torch.randn(512, 2048, device=dev, requires_grad=True)
x = torch.randn(4, 2048, 32, 32, device=dev, requires_grad=True)
for it in range(2):
    print(f"iteration {it}", flush=True)
    y = decoder_hip.pointwise(w, x.view(4, 2048, 1024)).view(4, 512, 32, 32)
    (y * 1.5).sum().backward()
torch.cuda.synchronize()
