"""Microbench: a ConvNeXt layer's style affine + demodulation (csrc/style.hip) forward and forward +
backward against the torch formulation (decoder_ops.style_and_demod with VFM_STYLE_HIP off), B = 32,
w_dim = 512, at the decoder's widths."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch  # noqa: E402

from networks.utils.shared import StyleSplit  # noqa: E402
from torch_utils.ops import decoder_ops  # noqa: E402


def bench(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


for C in (512, 256, 128):
    aff = StyleSplit(512, C, bias_init=1).cuda()
    w1 = (torch.randn(4 * C, C, device="cuda") * 0.02).requires_grad_(True)
    ws = torch.randn(32, 20, 512, device="cuda", requires_grad=True)
    gs, gd = torch.randn(32, C, device="cuda"), torch.randn(32, 4 * C, device="cuda")
    res = []
    for hip in (True, False):
        decoder_ops.STYLE_HIP = hip

        def fwd():
            with torch.no_grad():
                decoder_ops.style_and_demod(aff, ws[:, 3], w1)

        def fb():
            s, d = decoder_ops.style_and_demod(aff, ws[:, 3], w1)
            torch.autograd.backward([s, d], [gs, gd])

        res.append((bench(fwd), bench(fb)))
    print(f"C={C}: hip fwd {res[0][0]:7.1f} us  fwd+bwd {res[0][1]:7.1f} us | torch fwd {res[1][0]:7.1f} us  "
          f"fwd+bwd {res[1][1]:7.1f} us", flush=True)
