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

# backward per job (direct C-ABI calls, outputs switched off one at a time): launch 2 = ds tiles | dW1 outer
# tiles, launch 3 = dA/dab outer tiles | dw tiles
from torch_utils import custom_ops  # noqa: E402

lib = custom_ops.get_native()
st = custom_ops.stream_ptr(torch.device("cuda", 0))
P = lambda t: None if t is None else t.data_ptr()  # noqa: E731
for C in (512, 256, 128):
    B, WD, O = 32, 512, 4 * C
    f = lambda *s: torch.randn(*s, device="cuda")  # noqa: E731
    w, A, ab, W1 = f(B, WD), f(3 * C, WD) * 0.05, f(3 * C), f(O, C) * 0.02
    m, s, d = f(B, 3 * C), f(B, C), f(B, O).abs() + 0.5
    ds_in, dd = f(B, C), f(B, O)
    ds_ws, dW1, dA, dab, dw = f(lib.vfm_style_demod_bwd_workspace_floats(B, C, WD, O)), f(O, C), f(3 * C, WD), f(3 * C), f(B, WD)
    res = []
    for tag, outs in [("all", (dW1, dA, dab, dw)), ("no dW1", (None, dA, dab, dw)), ("ds only", (None, None, None, None)),
                      ("no dA/dab", (dW1, None, None, dw)), ("no dw", (dW1, dA, dab, None))]:
        def fn(outs=outs):
            rc = lib.vfm_style_demod_bwd(w.data_ptr(), WD, A.data_ptr(), W1.data_ptr(), m.data_ptr(), s.data_ptr(),
                                         d.data_ptr(), ds_in.data_ptr(), dd.data_ptr(), 1.0, 1.0, B, C, WD, O,
                                         ds_ws.data_ptr(), P(outs[0]), P(outs[1]), P(outs[2]), P(outs[3]), st)
            assert rc == 0, rc
        res.append(f"{tag} {bench(fn):6.1f}")
    print(f"C={C} bwd us: " + " | ".join(res), flush=True)
