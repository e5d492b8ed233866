"""DiffAugment translation on the HIP shift kernel (csrc/diffaug.hip) against the reference's padded
gather (training/diffaug.py translate_gather, reference training/diffaug.py rand_translation) on the
same shifts: forward and input gradient bit-exact (each output / gradient element is one copied value
or a zero), fp32 and bf16, shifts at the +-ratio extremes."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,C,H,W", [(8, 3, 256, 256), (5, 3, 37, 64)])
def test_translation_matches_gather(dtype, B, C, H, W):
    from training import diffaug
    g = torch.Generator().manual_seed(B * H + W)
    x = torch.randn(B, C, H, W, generator=g).to(dtype).cuda()
    sx, sy = int(H * 0.125 + 0.5), int(W * 0.125 + 0.5)
    tx = torch.randint(-sx, sx + 1, (B, 1, 1), generator=g)
    ty = torch.randint(-sy, sy + 1, (B, 1, 1), generator=g)
    tx[0], ty[0], tx[1], ty[1] = sx, -sy, -sx, sy          # extremes
    tx, ty = tx.cuda(), ty.cuda()
    dy = torch.randn(B, C, H, W, generator=g).to(dtype).cuda()
    xa = x.clone().requires_grad_(True)
    ya = diffaug._Shift2d.apply(xa, tx.reshape(B).contiguous(), ty.reshape(B).contiguous())
    ya.backward(dy)
    xb = x.clone().requires_grad_(True)
    yb = diffaug.translate_gather(xb, tx, ty)
    yb.backward(dy)
    assert torch.equal(ya, yb)
    assert torch.equal(xa.grad, xb.grad)
