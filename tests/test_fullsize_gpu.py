"""Full-size parity of the continuous path on cuda:0 against vectors generated from the reference
itself (tests/golden/make_golden_fullsize.py): the SigLIP2-L tower at 512^2 (24 x 1024, patch
features hidden_states[0], [12], last_hidden_state; reference networks/utils/vfms/
siglip2_utils.py:94-137) and the f16d32 stage-0 Generator.forward(validation=True) at 256^2 with
tools/reconstruct/reconstruct.py's settings (num_fp16_res 0; reference networks/generator.py:
1152-1206), weights from tests/det_init.py, posterior noise from the CPU generator as the reference
draws it.

Stated tolerances:
  fp32 (what reconstruct.py runs: tower and decoder in fp32, our GEMM / attention / conv kernels
  with fp32-equivalent f32x6 products):
    hidden states: max |err| <= 1e-4 of max |ref| on the stored rows, token norms within 1e-5;
    latent moments: max |err| <= 1e-4 of max |ref|;
    image: max per-pixel |err| <= 2e-3 (images in [-1, 1]) and PSNR >= 70 dB;
  bf16 (the training precision: tower under bf16 autocast):
    hidden states: relative L2 <= 3e-2; image PSNR >= 30 dB.
"""
import json

import numpy as np
import pytest
import torch

import fullsize_case as fc
from det_init import det_init

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
GOLDEN = __import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "fullsize_golden.npz")


@pytest.fixture(scope="module")
def golden():
    z = np.load(GOLDEN)
    return z, json.loads(str(z["meta"]))


@pytest.fixture(scope="module")
def generator(tmp_path_factory, golden):
    _, meta = golden
    d = tmp_path_factory.mktemp("vfmfull") / fc.VFM_DIRNAME
    d.mkdir()
    json.dump(fc.SIGLIP_L_CFG, open(d / "config.json", "w"))
    from networks.generator import Generator
    G = Generator(label_dim=0, **dict(meta["g_kwargs"], vfm_name=str(d)))
    det_init(G)
    return G.eval().requires_grad_(False).to(DEV)


def _relmax(a, b):
    a, b = a.double(), torch.as_tensor(b).double()
    return float((a - b).abs().max() / b.abs().max())


def _rel_l2(a, b):
    a, b = a.double(), torch.as_tensor(b).double()
    return float((a - b).norm() / b.norm())


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_siglip2_large_hidden_states(generator, golden, precision):
    z, meta = golden
    img = fc.image()
    assert abs(float(img.double().sum()) - meta["img_sum"]) < 1e-6
    enc = generator.vfm_encoder.encoder
    enc.amp_enabled = precision == "bf16"
    try:
        with torch.no_grad():
            feats, _ = generator.vfm_encoder.encode_image(img.to(DEV))
    finally:
        enc.amp_enabled = False
    for name, f in zip(fc.HIDDEN_NAMES, feats):
        rows = f[0, ::fc.ROW_STRIDE].cpu()
        norms = f[0].double().norm(dim=-1).cpu()
        ref_rows, ref_norms = z[f"S/{name}/rows"], z[f"S/{name}/norms"]
        e_max, e_l2 = _relmax(rows, ref_rows), _rel_l2(rows, ref_rows)
        e_norm = _relmax(norms, ref_norms)
        print(f"{precision} {name}: rows relmax {e_max:.3e} relL2 {e_l2:.3e}, norms relmax {e_norm:.3e}")
        if precision == "fp32":
            assert e_max <= 1e-4, (name, e_max)
            assert e_norm <= 1e-5, (name, e_norm)
        else:
            assert e_l2 <= 3e-2, (name, e_l2)


def test_reconstruction_fp32(generator, golden):
    """reconstruct.py's forward: fp32 everywhere."""
    z, _ = golden
    img = fc.image().to(DEV)
    generator.vfm_encoder.encoder.amp_enabled = False
    with torch.no_grad():
        moments = generator.encode(img, return_z_before_quantize=True).cpu()
        torch.manual_seed(fc.EPS_SEED)
        out = generator(img, ["x"], validation=True).gen_img.cpu()
    ref = torch.from_numpy(z["F/gen_img"])
    e_mom = _relmax(moments, z["F/moments"])
    e_px = float((out.double() - ref.double()).abs().max())
    p = fc.psnr(out, ref)
    print(f"fp32 moments relmax {e_mom:.3e}; image max |err| {e_px:.3e}, PSNR {p:.1f} dB")
    assert e_mom <= 1e-4, e_mom
    assert e_px <= 2e-3, e_px
    assert p >= 70.0, p


def test_reconstruction_bf16_tower(generator, golden):
    """The training precision of the tower (bf16 autocast) under the fp32 decoder."""
    z, _ = golden
    img = fc.image().to(DEV)
    enc = generator.vfm_encoder.encoder
    enc.amp_enabled = True
    try:
        with torch.no_grad():
            torch.manual_seed(fc.EPS_SEED)
            out = generator(img, ["x"], validation=True).gen_img.cpu()
    finally:
        enc.amp_enabled = False
    p = fc.psnr(out, torch.from_numpy(z["F/gen_img"]))
    print(f"bf16 tower: image PSNR {p:.1f} dB")
    assert p >= 30.0, p
