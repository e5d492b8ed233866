"""fp32 row kernels that also write their output's exact bf16 pieces for the f32x6 GEMMs (decoder_hip
_ScaleBiasGelu forward / backward, _LayerScaleResidual backward: vfm_*_pc): the pieces are bit-identical to the
GEMMs' own planar split (vfm_split_f32) of the same tensor, and a ConvNeXt-MLP-shaped chain (pwconv1 -> scale +
bias + GELU -> pwconv2 -> bias + layer scale + residual; reference networks/utils/convnext_utils.py:135-142) gives
bit-identical outputs and gradients with the producer pieces on and off."""
import pytest
import torch

from torch_utils import custom_ops
from torch_utils.ops import decoder_hip, gemm_hip

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def test_pieces_match_split():
    g0 = torch.Generator().manual_seed(0)
    h = torch.randn(3, 96, 200, generator=g0).to(DEV)
    s = torch.rand(3, 96, generator=g0).to(DEV) + 0.5
    b = torch.randn(96, generator=g0).to(DEV)
    g = decoder_hip.scale_bias_gelu(h, s, b)
    hit = getattr(g, "_vfm_planar", None)
    assert hit is not None
    ref = torch.empty((3, g.numel()), dtype=torch.bfloat16, device=DEV)
    lib = custom_ops.get_native()
    custom_ops.check(lib.vfm_split_f32(g.clone().data_ptr(), ref.data_ptr(), 1, g.numel(), g.numel(), 0, 0, 1,
                                       custom_ops.VFM_F32, 1, custom_ops.stream_ptr(DEV)), "vfm_split_f32")
    assert torch.equal(hit[1].view(torch.int16), ref.view(torch.int16))


def test_group_norm_pieces_match_split():
    g0 = torch.Generator().manual_seed(2)
    x = torch.randn(2, 64, 16, 16, generator=g0).to(DEV)
    w, b = torch.rand(64, generator=g0).to(DEV) + 0.5, torch.randn(64, generator=g0).to(DEV)
    s = torch.rand(2, 64, generator=g0).to(DEV) + 0.5
    y = decoder_hip.group_norm(x, 16, w, b, 1e-5, style=s, out_dtype=torch.float32)
    hit = getattr(y, "_vfm_planar", None)
    assert hit is not None
    ref = torch.empty((3, y.numel()), dtype=torch.bfloat16, device=DEV)
    lib = custom_ops.get_native()
    custom_ops.check(lib.vfm_split_f32(y.clone().data_ptr(), ref.data_ptr(), 1, y.numel(), y.numel(), 0, 0, 1,
                                       custom_ops.VFM_F32, 1, custom_ops.stream_ptr(DEV)), "vfm_split_f32")
    assert torch.equal(hit[1].view(torch.int16), ref.view(torch.int16))


def _chain(on, monkeypatch):
    monkeypatch.setattr(decoder_hip, "PRODUCER_PIECES", on)
    g0 = torch.Generator().manual_seed(1)
    B, C, P = 4, 128, 256
    x = torch.randn(B, C, P, generator=g0).to(DEV).requires_grad_(True)
    w1 = (torch.randn(4 * C, C, generator=g0) / C ** 0.5).to(DEV).requires_grad_(True)
    w2 = (torch.randn(C, 4 * C, generator=g0) / (4 * C) ** 0.5).to(DEV).requires_grad_(True)
    s = (torch.rand(B, 4 * C, generator=g0) + 0.5).to(DEV).requires_grad_(True)
    b1 = torch.randn(4 * C, generator=g0).to(DEV).requires_grad_(True)
    b2 = torch.randn(C, generator=g0).to(DEV).requires_grad_(True)
    gm = torch.rand(C, generator=g0).to(DEV).requires_grad_(True)
    h = decoder_hip.pointwise(w1, x)
    g = decoder_hip.scale_bias_gelu(h, s, b1)
    y = decoder_hip.pointwise(w2, g)
    out = decoder_hip.layer_scale_residual(y, b2, gm, x)
    dout = torch.randn(out.shape, generator=g0).to(DEV)
    out.backward(dout)
    return [out.detach()] + [t.grad for t in (x, w1, w2, s, b1, b2, gm)]


def test_chain_bitwise_with_and_without_producer_pieces(monkeypatch):
    off = _chain(False, monkeypatch)
    on = _chain(True, monkeypatch)
    for a, b in zip(on, off):
        assert torch.equal(a, b)
