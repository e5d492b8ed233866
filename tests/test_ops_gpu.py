"""HIP parity for upfirdn2d / bias_act / filtered_lrelu / conv2d_resample on MI355X.

Compares the C-ABI kernels (through the reference-compatible Python API) with
the golden vectors generated from the reference's `_ref` ops and with the C
oracle. Tolerances: fp64 1e-10 (same math, different summation order), fp32
2e-5, fp16/bf16 2e-2 / 4e-2 relative to the max magnitude.
"""
import numpy as np
import pytest
import torch

import golden_io
from op_cases import rel_err, upfirdn_params
from oracle import ops_oracle
from torch_utils.ops import upfirdn2d, bias_act, filtered_lrelu, conv2d_resample

pytestmark = pytest.mark.gpu
G = "ops_golden.npz"
DEV = "cuda"
TOL = {torch.float64: 1e-10, torch.float32: 2e-5, torch.float16: 2e-2, torch.bfloat16: 4e-2}


def cu(a, dtype=torch.float64):
    return torch.from_numpy(np.asarray(a)).to(DEV, dtype)


@pytest.fixture(autouse=True)
def _no_ref_fallback(monkeypatch):
    """Any call into the pure-torch reference paths on GPU tensors is a failure."""
    def boom(*a, **k):
        raise AssertionError("HIP path fell back to the torch reference implementation")
    monkeypatch.setattr(upfirdn2d, "_upfirdn2d_ref", boom)
    monkeypatch.setattr(bias_act, "_bias_act_ref", boom)
    monkeypatch.setattr(filtered_lrelu, "_filtered_lrelu_ref", boom)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("channels_last", [False, True])
@pytest.mark.parametrize("i", range(golden_io.count(G, "upfirdn2d")))
def test_upfirdn2d_hip(i, dtype, channels_last):
    arr, meta = golden_io.case(G, "upfirdn2d", i)
    x = cu(arr["x"], dtype)
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    f = cu(arr["f"], torch.float32) if "f" in arr else None
    y = getattr(upfirdn2d, meta["api"])(x, f, **meta["kw"])
    assert y.dtype == dtype and y.shape == arr["y"].shape
    assert rel_err(y.detach().double().cpu(), arr["y"]) < TOL[dtype]
    (dx,) = torch.autograd.grad(y, x, cu(arr["dy"], dtype))
    assert rel_err(dx.double().cpu(), arr["dx"]) < TOL[dtype] * 2


def test_upfirdn2d_matches_oracle_large_and_linear():
    """Full-size property checks: oracle agreement on a 2-tile-wide plane and linearity."""
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2, 8, 96, 160, generator=g, dtype=torch.float64)
    f = upfirdn2d.setup_filter([1, 4, 6, 4, 1])
    y = upfirdn2d.upfirdn2d(x.to(DEV), f.to(DEV), up=2, down=1, padding=[2, 3, 2, 3]).cpu()
    yo = ops_oracle.upfirdn2d(x.numpy(), f.double().numpy(), up=2, down=1, padding=[2, 3, 2, 3], gain=1.0)
    assert rel_err(y, yo) < 1e-10
    a = torch.randn(8, 64, 256, 256, device=DEV)
    b = torch.randn(8, 64, 256, 256, device=DEV)
    fd = f.to(DEV)
    lhs = upfirdn2d.downsample2d(2.5 * a + b, fd)
    rhs = 2.5 * upfirdn2d.downsample2d(a, fd) + upfirdn2d.downsample2d(b, fd)
    assert rel_err(lhs.double().cpu(), rhs.double().cpu()) < 1e-5


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32, torch.float16])
@pytest.mark.parametrize("i", range(golden_io.count(G, "bias_act")))
def test_bias_act_hip(i, dtype):
    arr, meta = golden_io.case(G, "bias_act", i)
    if dtype == torch.float16 and meta["act"] in ("selu", "elu", "softplus", "swish", "tanh", "sigmoid"):
        pytest.skip("fp16 transcendental tails checked in fp32/fp64")
    x = cu(arr["x"], dtype).requires_grad_(True)
    b = cu(arr["b"], dtype).requires_grad_(True) if "b" in arr else None
    y = bias_act.bias_act(x, b, dim=meta["dim"], act=meta["act"], **meta["kw"])
    tol = {torch.float64: 1e-7, torch.float32: 1e-5, torch.float16: 5e-3}[dtype]  # gain/clamp cross the ABI as fp32 (as in bias_act.cpp:32)
    assert rel_err(y.detach().double().cpu(), arr["y"]) < tol
    inputs = [x] + ([b] if b is not None else [])
    grads = torch.autograd.grad(y, inputs, cu(arr["dy"], dtype), create_graph=True)
    assert rel_err(grads[0].detach().double().cpu(), arr["dx"]) < tol * 4
    if b is not None:
        assert rel_err(grads[1].detach().double().cpu(), arr["db"]) < tol * 4
    if dtype == torch.float64 and grads[0].requires_grad:
        ddx = torch.autograd.grad(grads[0], x, cu(arr["v"]), allow_unused=True)[0]
        ddx = torch.zeros_like(x) if ddx is None else ddx
        # alpha/gain/clamp cross the ABI as fp32 (bias_act.cpp:32 takes float): a relative
        # rounding of up to 2^-24 ~ 6e-8 per scalar, so fp64 cannot be tighter than ~1e-7.
        assert rel_err(ddx.cpu(), arr["ddx"]) < 2e-7


def test_bias_act_channels_last_and_large():
    x = torch.randn(4, 96, 33, 47, device=DEV).contiguous(memory_format=torch.channels_last)
    b = torch.randn(96, device=DEV)
    y = bias_act.bias_act(x, b, act='lrelu', clamp=0.7)
    ref = (torch.nn.functional.leaky_relu(x + b[None, :, None, None], 0.2) * np.sqrt(2)).clamp(-0.7, 0.7)
    assert y.is_contiguous(memory_format=torch.channels_last)
    assert rel_err(y.cpu().double(), ref.cpu().double()) < 1e-6


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32, torch.float16])
@pytest.mark.parametrize("i", range(golden_io.count(G, "filtered_lrelu")))
def test_filtered_lrelu_hip(i, dtype):
    arr, meta = golden_io.case(G, "filtered_lrelu", i)
    x = cu(arr["x"], dtype).requires_grad_(True)
    b = cu(arr["b"], dtype).requires_grad_(True) if "b" in arr else None
    fu = cu(arr["fu"], torch.float32) if "fu" in arr else None
    fd = cu(arr["fd"], torch.float32) if "fd" in arr else None
    y = filtered_lrelu.filtered_lrelu(x, fu, fd, b, **meta["kw"])
    tol = {torch.float64: 1e-6, torch.float32: 2e-5, torch.float16: 2e-2}[dtype]
    assert y.shape == arr["y"].shape
    assert rel_err(y.detach().double().cpu(), arr["y"]) < tol
    inputs = [x] + ([b] if b is not None else [])
    grads = torch.autograd.grad(y, inputs, cu(arr["dy"], dtype))
    # Gradients flow through the stored sign bits; elements whose pre-activation sits
    # within rounding of 0 or of the clamp may legitimately flip, so use a norm bound.
    gtol = {torch.float64: 1e-6, torch.float32: 1e-4, torch.float16: 3e-2}[dtype]
    assert rel_err(grads[0].double().cpu(), arr["dx"]) < gtol
    if b is not None:
        assert rel_err(grads[1].double().cpu(), arr["db"]) < gtol


@pytest.mark.parametrize("i", range(golden_io.count(G, "filtered_lrelu")))
def test_filtered_lrelu_signs_match_oracle(i):
    """The packed 2-bit sign tensor equals the oracle's codes on the active region."""
    arr, meta = golden_io.case(G, "filtered_lrelu", i)
    kw = dict(meta["kw"])
    x = cu(arr["x"], torch.float32).requires_grad_(True)   # fused kernel: fp32/fp16/bf16
    fu = cu(arr["fu"], torch.float32) if "fu" in arr else None
    fd = cu(arr["fd"], torch.float32) if "fd" in arr else None
    b = cu(arr["b"], torch.float32) if "b" in arr else None
    cfg = filtered_lrelu._make_cfg(kw.get("up", 1), kw.get("down", 1), kw.get("padding", 0),
                                   kw.get("gain", np.sqrt(2)), kw.get("slope", 0.2), kw.get("clamp"),
                                   kw.get("flip_filter", False))
    fu_ = fu if fu is not None else torch.ones([1, 1], device=DEV)
    fd_ = fd if fd is not None else torch.ones([1, 1], device=DEV)
    bb = b if b is not None else torch.zeros(x.shape[1], dtype=x.dtype, device=DEV)
    res = filtered_lrelu._filtered_lrelu_native(x.detach(), fu_, fd_, bb, None, 0, 0, cfg, True)
    assert res is not None
    _, so = res
    x32 = arr["x"].astype(np.float32).astype(np.float64)
    b32 = arr["b"].astype(np.float32).astype(np.float64) if "b" in arr else None
    _, codes = ops_oracle.filtered_lrelu(x32, arr.get("fu"), arr.get("fd"), b32, **kw)
    s = so.cpu().numpy()
    unpacked = np.stack([(s >> (2 * e)) & 3 for e in range(4)], axis=-1).reshape(s.shape[0], s.shape[1], s.shape[2], -1)
    sh = unpacked.shape[2]
    up, down = kw.get("up", 1), kw.get("down", 1)
    fdw = (1 if fd is None else (fd.shape[-1]))
    yw = arr["y"].shape[3]
    sw_active = yw * down - (down - 1) + (fdw - 1)
    assert np.array_equal(unpacked[:, :, :sh, :sw_active], codes[:, :, :sh, :sw_active])


def test_filtered_lrelu_generic_fallback_path():
    """up=3 has no fused kernel -> generic HIP chain, still matches the oracle."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 3, 10, 10, generator=g, dtype=torch.float64)
    f = upfirdn2d.setup_filter([1, 2, 3, 2, 1])
    y = filtered_lrelu.filtered_lrelu(x.to(DEV), f.to(DEV), f.to(DEV), up=3, down=1, padding=2, clamp=0.5).cpu()
    yo, _ = ops_oracle.filtered_lrelu(x.numpy(), f.double().numpy(), f.double().numpy(), None, up=3, down=1,
                                      padding=2, clamp=0.5)
    assert rel_err(y, yo) < 1e-7      # gain=sqrt(2) and slope cross the ABI as fp32 (filtered_lrelu.cpp:16)


def test_filtered_lrelu_large_fp16_vs_oracle():
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 16, 64, 64, generator=g)
    f = upfirdn2d.setup_filter(torch.rand(12, generator=g) + 0.2, separable=True)
    y = filtered_lrelu.filtered_lrelu(x.to(DEV, torch.float16), f.to(DEV), f.to(DEV), up=2, down=2,
                                      padding=10, clamp=2.0).double().cpu()
    yo, _ = ops_oracle.filtered_lrelu(x.double().numpy(), f.double().numpy(), f.double().numpy(), None,
                                      up=2, down=2, padding=10, clamp=2.0)
    assert rel_err(y, yo) < 2e-2


@pytest.mark.parametrize("i", range(golden_io.count(G, "conv2d_resample")))
def test_conv2d_resample_hip(i):
    arr, meta = golden_io.case(G, "conv2d_resample", i)
    x = cu(arr["x"], torch.float32).requires_grad_(True)
    w = cu(arr["w"], torch.float32).requires_grad_(True)
    y = conv2d_resample.conv2d_resample(x, w, f=cu(arr["f"], torch.float32), **meta["kw"])
    assert rel_err(y.detach().double().cpu(), arr["y"]) < 1e-4
    dx, dw = torch.autograd.grad(y, [x, w], cu(arr["dy"], torch.float32))
    assert rel_err(dx.double().cpu(), arr["dx"]) < 1e-4
    assert rel_err(dw.double().cpu(), arr["dw"]) < 1e-4


def test_errors_are_loud():
    with pytest.raises(Exception):
        upfirdn2d.upfirdn2d(torch.zeros(1, 1, 4, 4, device=DEV, dtype=torch.int32), None)
    with pytest.raises(RuntimeError):
        upfirdn2d.upfirdn2d(torch.zeros(1, 1, 2, 2, device=DEV), torch.ones(5, 5, device=DEV))
