"""DINOv2-L (BASELINE config 3's encoder) against vectors generated from the reference itself
(tests/golden/make_golden_dinov2.py: reference networks/utils/vfms/dinov2_utils.py:77-128 over a local HF
Dinov2Model, weights from tests/det_init.py): hidden_states[0], hidden_states[12] and last_hidden_state patch
tokens and the pooled CLS output at 256 / 384 / 512 input (scale_factor 0.875: 16 / 24 / 32 patches a side, the
bicubic position-grid resampling) and with the equivariance prior's bicubic downscale.

Stated tolerances:
  fp32 (amp off; on cuda:0 our GEMMs with fp32-equivalent products, our fp32 attention): stored rows max |err| <=
    1e-4 of max |ref|, token norms and pooled output within 1e-4;
  bf16 (the training precision: the tower under bf16 autocast, gemm9 + bf16 flash attention): relative L2 <= 3e-2.
The CPU test runs the same comparison through the torch formulation (the restatement itself) on one case."""
import json
import os

import numpy as np
import pytest
import torch

import dinov2_case as dc
from det_init import det_init

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "dinov2_golden.npz")


@pytest.fixture(scope="module")
def golden():
    z = np.load(GOLDEN)
    return z, json.loads(str(z["meta"]))


def _encoder(tmp_path_factory, device):
    d = tmp_path_factory.mktemp("dinov2") / dc.VFM_DIRNAME
    d.mkdir()
    json.dump(dc.DINOV2_L_CFG, open(d / "config.json", "w"))
    from networks.utils.vfms.dinov2_utils import DINOv2Encoder
    enc = DINOv2Encoder(model_name=str(d), scale_factor=dc.SCALE_FACTOR, patch_from_layers=list(dc.LAYERS),
                        amp_enabled=False)
    det_init(enc.vision_model)
    return enc.eval().to(device)


@pytest.fixture(scope="module")
def encoder_gpu(tmp_path_factory):
    return _encoder(tmp_path_factory, torch.device("cuda", 0))


def _relmax(a, b):
    a, b = a.double().cpu(), torch.as_tensor(b).double()
    return float((a - b).abs().max() / b.abs().max())


def _rel_l2(a, b):
    a, b = a.double().cpu(), torch.as_tensor(b).double()
    return float((a - b).norm() / b.norm())


def _compare(enc, golden, case, device, precision):
    z, meta = golden
    name = case["name"]
    img = dc.image(case["res"], case["seed"])
    assert abs(float(img.double().sum()) - meta[f"{name}/img_sum"]) < 1e-6
    enc.amp_enabled = precision == "bf16"
    try:
        with torch.no_grad():
            feats, pooled = enc.encode_image(img.to(device), case["eq_scale"], case["prior"])
    finally:
        enc.amp_enabled = False
    worst = {}
    for hname, f in zip(dc.HIDDEN_NAMES, feats):
        assert list(f.shape) == meta[f"{name}/{hname}/shape"], (name, hname, tuple(f.shape))
        rows, norms = f[0, ::dc.ROW_STRIDE], f[0].double().norm(dim=-1)
        ref_rows, ref_norms = z[f"{name}/{hname}/rows"], z[f"{name}/{hname}/norms"]
        if precision == "fp32":
            worst[hname] = (_relmax(rows, ref_rows), _relmax(norms, ref_norms))
            assert worst[hname][0] <= 1e-4 and worst[hname][1] <= 1e-4, (name, hname, worst[hname])
        else:
            worst[hname] = _rel_l2(rows, ref_rows)
            assert worst[hname] <= 3e-2, (name, hname, worst[hname])
    ep = _relmax(pooled[0], z[f"{name}/pooled"]) if precision == "fp32" else _rel_l2(pooled[0], z[f"{name}/pooled"])
    assert ep <= (1e-4 if precision == "fp32" else 3e-2), (name, ep)
    print(f"{precision} {name}: {worst} pooled {ep:.2e}")


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "bf16"])
@pytest.mark.parametrize("case", dc.CASES, ids=[c["name"] for c in dc.CASES])
def test_dinov2_large_matches_reference_gpu(encoder_gpu, golden, case, precision):
    _compare(encoder_gpu, golden, case, torch.device("cuda", 0), precision)


@pytest.mark.slow
def test_dinov2_large_matches_reference_cpu(tmp_path_factory, golden):
    """The torch formulation of the tower on the CPU (fp32) on the equivariance-prior case (64 tokens)."""
    enc = _encoder(tmp_path_factory, torch.device("cpu"))
    _compare(enc, golden, dc.CASES[3], torch.device("cpu"), "fp32")
