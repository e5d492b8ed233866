"""Generate golden vectors for the StyleGAN-lineage ops FROM THE REFERENCE ITSELF.

Runs only in the build container (it imports /root/reference, which does not
exist on the GPU box). Output: tests/golden/ops_golden.npz (inputs, outputs and
input gradients, float64) consumed by tests/test_oracle_ops.py (oracle pin) and
tests/test_ops_gpu.py (HIP parity).

The reference's CUDA plugins cannot run here, so the vectors come from its pure
torch `_ref` paths (upfirdn2d.py:166, bias_act.py:90, filtered_lrelu.py:120) and
`conv2d_resample` (conv2d_resample.py:46), which define the ops' semantics.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_ops.py
"""
import json
import os
import sys

import numpy as np
import torch

REF = os.environ.get("VFM_REFERENCE", "/root/reference")
sys.path.insert(0, REF)

from torch_utils.ops import upfirdn2d, bias_act, filtered_lrelu, conv2d_resample  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ops_golden.npz")
torch.manual_seed(1234)
arrays = {}
meta = {"upfirdn2d": [], "bias_act": [], "filtered_lrelu": [], "conv2d_resample": []}


def rnd(*shape):
    return torch.randn(*shape, dtype=torch.float64)


def put(prefix, **tensors):
    for k, v in tensors.items():
        if v is None:
            continue
        arrays[f"{prefix}/{k}"] = v.detach().cpu().numpy()


# ---------------------------------------------------------------- upfirdn2d
blur13 = torch.arange(-6, 7, dtype=torch.float32).div(2.0).square().neg().exp2()
blur13 = blur13 / blur13.sum()                      # training/loss.py:229-230 blur, sigma=2
upf_cases = [
    dict(api="upsample2d", shape=[2, 3, 16, 16], f=[1, 3, 3, 1], kw=dict(up=2)),
    dict(api="downsample2d", shape=[2, 3, 16, 16], f=[1, 3, 3, 1], kw=dict(down=2)),
    dict(api="filter2d", shape=[2, 3, 20, 20], f="blur13", kw=dict()),
    dict(api="upfirdn2d", shape=[1, 2, 9, 13], f="rand3x5", kw=dict(up=2, down=2, padding=[1, 2, 0, -1], flip_filter=True, gain=2.0)),
    dict(api="upfirdn2d", shape=[2, 2, 8, 8], f="rand4x4", kw=dict(up=4, down=1, padding=[2, 1, 2, 1])),
    dict(api="upfirdn2d", shape=[2, 2, 32, 24], f="rand4x4", kw=dict(up=1, down=4, padding=[1, 1, 0, 2])),
    dict(api="upfirdn2d", shape=[1, 3, 7, 11], f="rand5x3", kw=dict(up=[3, 2], down=[2, 3], padding=[4, 3, 2, 5])),
    dict(api="upsample2d", shape=[2, 4, 16, 16], f="sep8", kw=dict(up=2)),
    dict(api="upfirdn2d", shape=[2, 3, 34, 70], f=[1, 2, 1], kw=dict(up=1, down=1, padding=1)),
    dict(api="upfirdn2d", shape=[1, 1, 1, 1], f=None, kw=dict()),
]
for i, case in enumerate(upf_cases):
    x = rnd(*case["shape"]).requires_grad_(True)
    fdesc = case["f"]
    if fdesc == "blur13":
        f = blur13.clone()
    elif isinstance(fdesc, str) and fdesc.startswith("rand"):
        fh, fw = (int(v) for v in fdesc[4:].split("x"))
        f = torch.rand(fh, fw, dtype=torch.float32) + 0.1
    elif fdesc == "sep8":
        f = upfirdn2d.setup_filter(torch.rand(8) + 0.2, separable=True)
    elif fdesc is None:
        f = None
    else:
        f = upfirdn2d.setup_filter(fdesc)
    fn = getattr(upfirdn2d, case["api"])
    y = fn(x, f, **case["kw"], impl="ref")
    dy = rnd(*y.shape)
    (dx,) = torch.autograd.grad(y, x, dy)
    put(f"upfirdn2d/{i}", x=x, f=(f.double() if f is not None else None), y=y, dy=dy, dx=dx)
    meta["upfirdn2d"].append(dict(api=case["api"], kw=case["kw"], has_f=f is not None))

# ---------------------------------------------------------------- bias_act
acts = ["linear", "relu", "lrelu", "tanh", "sigmoid", "elu", "selu", "softplus", "swish"]
ba_cases = []
for act in acts:
    ba_cases.append(dict(act=act, shape=[2, 5, 4, 6], dim=1, bias=True, kw=dict()))
    ba_cases.append(dict(act=act, shape=[7, 5], dim=1, bias=True, kw=dict(gain=0.7, clamp=0.5)))
ba_cases.append(dict(act="lrelu", shape=[3, 6, 5, 5], dim=1, bias=False, kw=dict(alpha=0.1, gain=1.3)))
ba_cases.append(dict(act="softplus", shape=[4, 8], dim=0, bias=True, kw=dict()))
for i, case in enumerate(ba_cases):
    x = (rnd(*case["shape"]) * 3).requires_grad_(True)
    b = rnd(case["shape"][case["dim"]]).requires_grad_(True) if case["bias"] else None
    y = bias_act.bias_act(x, b, dim=case["dim"], act=case["act"], impl="ref", **case["kw"])
    dy = rnd(*y.shape)
    inputs = [x] + ([b] if b is not None else [])
    grads = torch.autograd.grad(y, inputs, dy, create_graph=True)
    dx = grads[0]
    db = grads[1] if b is not None else None
    # 2nd order: d/dx <dx, v>
    v = rnd(*x.shape)
    ddx = torch.autograd.grad(dx, x, v, allow_unused=True)[0] if dx.requires_grad else None
    if ddx is None:
        ddx = torch.zeros_like(x)
    put(f"bias_act/{i}", x=x, b=b, y=y, dy=dy, dx=dx, db=db, v=v, ddx=ddx)
    meta["bias_act"].append(dict(act=case["act"], dim=case["dim"], bias=case["bias"], kw=case["kw"]))

# ---------------------------------------------------------------- filtered_lrelu
f4 = upfirdn2d.setup_filter([1, 3, 3, 1])
fl_cases = [
    dict(shape=[2, 4, 16, 16], fu="f4", fd="f4", kw=dict(up=2, down=2, padding=3)),
    dict(shape=[2, 3, 12, 12], fu=None, fd="sep12", kw=dict(up=1, down=2, padding=[5, 6, 5, 6], clamp=0.3)),
    dict(shape=[1, 3, 10, 14], fu="sep8", fd=None, kw=dict(up=2, down=1, padding=[3, 4, 3, 4], gain=1.0, slope=0.1)),
    dict(shape=[2, 2, 8, 8], fu="sep16", fd="sep16", kw=dict(up=4, down=4, padding=[7, 8, 7, 8], clamp=0.8, flip_filter=True)),
    dict(shape=[1, 5, 9, 7], fu="f4", fd="f4", kw=dict(up=2, down=2, padding=[2, 3, 1, 4], clamp=1.5), bias=True),
]
for i, case in enumerate(fl_cases):
    def mk(desc):
        if desc is None:
            return None
        if desc == "f4":
            return f4.clone()
        return upfirdn2d.setup_filter(torch.rand(int(desc[3:])) + 0.2, separable=True)
    fu, fd = mk(case["fu"]), mk(case["fd"])
    x = rnd(*case["shape"]).requires_grad_(True)
    b = rnd(case["shape"][1]).requires_grad_(True) if case.get("bias") else None
    y = filtered_lrelu.filtered_lrelu(x, fu, fd, b, impl="ref", **case["kw"])
    dy = rnd(*y.shape)
    inputs = [x] + ([b] if b is not None else [])
    grads = torch.autograd.grad(y, inputs, dy)
    put(f"filtered_lrelu/{i}", x=x, b=b, fu=(fu.double() if fu is not None else None),
        fd=(fd.double() if fd is not None else None), y=y, dy=dy, dx=grads[0],
        db=(grads[1] if b is not None else None))
    meta["filtered_lrelu"].append(dict(kw=case["kw"], has_fu=fu is not None, has_fd=fd is not None,
                                       bias=bool(case.get("bias"))))

# ---------------------------------------------------------------- conv2d_resample
cr_cases = [
    dict(x=[2, 4, 8, 8], w=[6, 4, 3, 3], kw=dict(up=2, padding=1)),
    dict(x=[2, 4, 16, 16], w=[6, 4, 3, 3], kw=dict(down=2, padding=1)),
    dict(x=[2, 4, 8, 8], w=[6, 4, 1, 1], kw=dict(up=2)),
    dict(x=[2, 4, 16, 16], w=[6, 4, 1, 1], kw=dict(down=2)),
    dict(x=[1, 8, 8, 8], w=[8, 2, 3, 3], kw=dict(up=2, padding=1, groups=4, flip_weight=False)),
    dict(x=[2, 4, 9, 9], w=[5, 4, 3, 3], kw=dict(padding=1)),
]
for i, case in enumerate(cr_cases):
    x = rnd(*case["x"]).requires_grad_(True)
    w = rnd(*case["w"]).requires_grad_(True)
    f = upfirdn2d.setup_filter([1, 3, 3, 1])
    y = conv2d_resample.conv2d_resample(x, w, f=f, **case["kw"])
    dy = rnd(*y.shape)
    dx, dw = torch.autograd.grad(y, [x, w], dy)
    put(f"conv2d_resample/{i}", x=x, w=w, f=f.double(), y=y, dy=dy, dx=dx, dw=dw)
    meta["conv2d_resample"].append(dict(kw=case["kw"]))

arrays["meta"] = np.array(json.dumps(meta))
np.savez_compressed(OUT, **arrays)
print(f"wrote {OUT}: {len(arrays)} arrays, {os.path.getsize(OUT) / 1024:.1f} KiB")
