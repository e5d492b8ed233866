"""`vfm_pw_gemm_gelu` (csrc/pwgemm.hip): the ConvNeXt MLP channel GEMM with the GELU fused
into its epilogue, against the unfused formulation in fp32 torch
(reference convnext_utils.py:135-138: modulated 1x1 conv -> GELU(erf); backward: the 4C->C
conv's data gradient -> GELU backward).

Tolerances (max error relative to max |ref|): 1e-2 for bf16 outputs (one bf16 ulp is
3.9e-3 relative; the MFMA and the fp32 reference sum in different orders, which can flip
a rounding). MFMA fragment-layout errors show up as O(1) errors."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CASES = [(2, 512, 128, 256), (3, 1024, 256, 384), (2, 2048, 512, 128), (1, 512, 128, 4096), (2, 1024, 256, 2304)]


def _native():
    from torch_utils import custom_ops
    return custom_ops.get_native(), custom_ops


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


def _inputs(B, M, K, N, seed):
    g = torch.Generator().manual_seed(seed)
    A = (torch.randn(M, K, generator=g) / K ** 0.5).bfloat16().cuda()
    X = torch.randn(B, K, N, generator=g).bfloat16().cuda()
    s = (torch.rand(B, M, generator=g) + 0.5).cuda()
    bias = torch.randn(M, generator=g).cuda()
    return A, X, s, bias


@pytest.mark.parametrize("B,M,K,N", CASES)
@pytest.mark.parametrize("write_h", [True, False])
def test_forward_gemm_gelu(B, M, K, N, write_h):
    lib, co = _native()
    A, X, s, bias = _inputs(B, M, K, N, 0)
    h = torch.empty(B, M, N, dtype=torch.bfloat16, device="cuda")
    g = torch.empty_like(h)
    rc = lib.vfm_pw_gemm_gelu(A.data_ptr(), X.data_ptr(), s.data_ptr(), bias.data_ptr(), None,
                              h.data_ptr() if write_h else None, g.data_ptr(), None, None, 0, B, M, K, N,
                              co.stream_ptr())
    torch.cuda.synchronize()
    assert rc == 0
    href = torch.matmul(A.float(), X.float())
    gref = F.gelu(href.bfloat16().float() * s[:, :, None] + bias[None, :, None])
    if write_h:
        assert _rel(h.float(), href) < 1e-2
        gref = F.gelu(h.float() * s[:, :, None] + bias[None, :, None])
    assert _rel(g.float(), gref) < 1e-2


@pytest.mark.parametrize("B,M,K,N", CASES)
def test_backward_gemm_gelu(B, M, K, N):
    lib, co = _native()
    A, X, s, bias = _inputs(B, M, K, N, 1)
    hin = torch.randn(B, M, N, generator=torch.Generator().manual_seed(2)).bfloat16().cuda()
    tiles = lib.vfm_pw_gemm_gelu_tiles(N)
    assert tiles == N // 64
    dh = torch.empty(B, M, N, dtype=torch.bfloat16, device="cuda")
    p0 = torch.empty(B, tiles, M, device="cuda")
    p1 = torch.empty_like(p0)
    rc = lib.vfm_pw_gemm_gelu(A.data_ptr(), X.data_ptr(), s.data_ptr(), bias.data_ptr(), hin.data_ptr(),
                              dh.data_ptr(), None, p0.data_ptr(), p1.data_ptr(), 1, B, M, K, N, co.stream_ptr())
    torch.cuda.synchronize()
    assert rc == 0
    dg = torch.matmul(A.float(), X.float()).bfloat16().float()
    z = (hin.float() * s[:, :, None] + bias[None, :, None]).requires_grad_(True)
    F.gelu(z).backward(dg)
    dz = z.grad
    assert _rel(dh.float(), dz * s[:, :, None]) < 1e-2
    assert _rel(p0.sum(1), (dz * hin.float()).sum(-1)) < 1e-2
    assert _rel(p1.sum(1), dz.sum(-1)) < 1e-2


def test_unsupported_shapes_report_no_kernel():
    lib, co = _native()
    assert lib.vfm_pw_gemm_gelu_tiles(100) == co.VFM_NO_KERNEL
    A, X, s, bias = _inputs(1, 512, 128, 128, 3)
    out = torch.empty(1, 512, 128, dtype=torch.bfloat16, device="cuda")
    for (M, K, N) in [(512, 64, 128), (500, 128, 128), (512, 128, 100)]:
        rc = lib.vfm_pw_gemm_gelu(A.data_ptr(), X.data_ptr(), None, None, None, None, out.data_ptr(), None,
                                  None, 0, 1, M, K, N, co.stream_ptr())
        assert rc == co.VFM_NO_KERNEL
