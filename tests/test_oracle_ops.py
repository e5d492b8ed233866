"""Pin the C oracle (oracle/ops_oracle.c) against golden vectors produced by the
reference's own `_ref` ops (tests/golden/make_golden_ops.py). CPU only."""
import numpy as np
import pytest

import golden_io
from op_cases import upfirdn_params, rel_err
from oracle import ops_oracle

G = "ops_golden.npz"


@pytest.mark.parametrize("i", range(golden_io.count(G, "upfirdn2d")))
def test_oracle_upfirdn2d_matches_reference(i):
    arr, meta = golden_io.case(G, "upfirdn2d", i)
    f = arr.get("f")
    p = upfirdn_params(meta["api"], f, meta["kw"])
    y = ops_oracle.upfirdn2d(arr["x"], f if f is not None else np.ones((1, 1)), up=p["up"], down=p["down"],
                             padding=p["padding"], flip_filter=p["flip_filter"], gain=p["gain"])
    assert y.shape == arr["y"].shape
    assert rel_err(y, arr["y"]) < 1e-12


@pytest.mark.parametrize("i", range(golden_io.count(G, "bias_act")))
def test_oracle_bias_act_matches_reference(i):
    arr, meta = golden_io.case(G, "bias_act", i)
    kw = meta["kw"]
    y = ops_oracle.bias_act(arr["x"], arr.get("b"), dim=meta["dim"], act=meta["act"], alpha=kw.get("alpha"),
                            gain=kw.get("gain"), clamp=kw.get("clamp"))
    assert rel_err(y, arr["y"]) < 1e-12


@pytest.mark.parametrize("i", range(golden_io.count(G, "filtered_lrelu")))
def test_oracle_filtered_lrelu_matches_reference(i):
    arr, meta = golden_io.case(G, "filtered_lrelu", i)
    kw = dict(meta["kw"])
    y, codes = ops_oracle.filtered_lrelu(arr["x"], arr.get("fu"), arr.get("fd"), arr.get("b"), **kw)
    assert y.shape == arr["y"].shape
    assert rel_err(y, arr["y"]) < 1e-12
    assert set(np.unique(codes)).issubset({0, 1, 2})
