"""Host logic of the op modules on CPU (impl='ref' and CPU tensors), checked
against the reference's golden vectors; argument parsing; autograd plumbing."""
import numpy as np
import pytest
import torch

import golden_io
from op_cases import rel_err
from torch_utils.ops import upfirdn2d, bias_act, filtered_lrelu, conv2d_resample, fma

G = "ops_golden.npz"
t = torch.from_numpy


@pytest.mark.parametrize("i", range(golden_io.count(G, "upfirdn2d")))
def test_upfirdn2d_ref_path(i):
    arr, meta = golden_io.case(G, "upfirdn2d", i)
    x = t(arr["x"]).requires_grad_(True)
    f = t(arr["f"]).float() if "f" in arr else None
    y = getattr(upfirdn2d, meta["api"])(x, f, **meta["kw"])
    assert rel_err(y.detach(), arr["y"]) < 1e-6
    (dx,) = torch.autograd.grad(y, x, t(arr["dy"]))
    assert rel_err(dx, arr["dx"]) < 1e-6


@pytest.mark.parametrize("i", range(golden_io.count(G, "bias_act")))
def test_bias_act_ref_path(i):
    arr, meta = golden_io.case(G, "bias_act", i)
    x = t(arr["x"])
    b = t(arr["b"]) if "b" in arr else None
    y = bias_act.bias_act(x, b, dim=meta["dim"], act=meta["act"], **meta["kw"])
    assert rel_err(y, arr["y"]) < 1e-12


@pytest.mark.parametrize("i", range(golden_io.count(G, "filtered_lrelu")))
def test_filtered_lrelu_ref_path(i):
    arr, meta = golden_io.case(G, "filtered_lrelu", i)
    fu = t(arr["fu"]).float() if "fu" in arr else None
    fd = t(arr["fd"]).float() if "fd" in arr else None
    b = t(arr["b"]) if "b" in arr else None
    y = filtered_lrelu.filtered_lrelu(t(arr["x"]), fu, fd, b, **meta["kw"])
    assert rel_err(y, arr["y"]) < 1e-6


@pytest.mark.parametrize("i", range(golden_io.count(G, "conv2d_resample")))
def test_conv2d_resample_cpu(i):
    arr, meta = golden_io.case(G, "conv2d_resample", i)
    x = t(arr["x"]).requires_grad_(True)
    w = t(arr["w"]).requires_grad_(True)
    y = conv2d_resample.conv2d_resample(x, w, f=t(arr["f"]).float(), **meta["kw"])
    assert rel_err(y.detach(), arr["y"]) < 1e-6
    dx, dw = torch.autograd.grad(y, [x, w], t(arr["dy"]))
    assert rel_err(dx, arr["dx"]) < 1e-6 and rel_err(dw, arr["dw"]) < 1e-6


def test_setup_filter_rules():
    f = upfirdn2d.setup_filter([1, 3, 3, 1])
    assert f.shape == (4, 4) and abs(float(f.sum()) - 1) < 1e-6
    f = upfirdn2d.setup_filter(np.ones(8), gain=4)
    assert f.ndim == 1 and abs(float(f.sum()) - 2) < 1e-6  # gain**(1/2) per separable pass
    assert upfirdn2d.setup_filter(None).shape == (1, 1)
    assert torch.equal(upfirdn2d.setup_filter([1, 2], flip_filter=True, normalize=False), torch.tensor([[4., 2.], [2., 1.]]))


def test_activation_table_surface():
    assert set(bias_act.activation_funcs) == {'linear', 'relu', 'lrelu', 'tanh', 'sigmoid', 'elu', 'selu', 'softplus', 'swish'}
    assert abs(bias_act.activation_funcs['lrelu'].def_gain - np.sqrt(2)) < 1e-12
    assert [bias_act.activation_funcs[k].cuda_idx for k in bias_act.activation_funcs] == list(range(1, 10))


def test_fma_broadcast_grads():
    a = torch.randn(2, 3, 1, 4, dtype=torch.float64, requires_grad=True)
    b = torch.randn(3, 5, 1, dtype=torch.float64, requires_grad=True)
    c = torch.randn(1, 1, 5, 4, dtype=torch.float64, requires_grad=True)
    assert torch.autograd.gradcheck(fma.fma, (a, b, c))


def test_bad_impl_rejected():
    with pytest.raises(AssertionError):
        upfirdn2d.upfirdn2d(torch.zeros(1, 1, 4, 4), None, impl='triton')
