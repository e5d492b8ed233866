"""Frozen-tower bf16 linears on our 256-tile GEMM (torch_utils/ops/vit_ops.py `_own_linear`,
csrc/gemm9.hip) against the plain PyTorch fp32 reference of the same op (reference
networks/utils/vfms/siglip2_utils.py:114-137: q/k/v/out projections, fc1 + tanh-GELU, fc2 under bf16
autocast). Tolerance: one bf16 output rounding of an fp32-accumulated product plus the bias rounded to
bf16 first (hipBLASLt's bias epilogue): 8e-3 of max |ref|."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K", [(2048, 3072, 1024), (1000, 1024, 4096), (4096, 4096, 1024)])
@pytest.mark.parametrize("act", [None, "gelu_tanh"])
def test_own_linear_matches_fp32(M, N, K, act, monkeypatch):
    from torch_utils.ops import kernel_timer, vit_ops
    monkeypatch.setattr(vit_ops, "OWN_GEMM", True)
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(2, M // 2, K, generator=g).to(torch.bfloat16).cuda()
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).cuda()
    b = torch.randn(N, generator=g).cuda()
    kernel_timer.enable(True)
    with torch.no_grad():
        y = vit_ops.linear_gelu_tanh(x, w, b) if act else vit_ops.linear(x, w, b)
    torch.cuda.synchronize()
    assert any(k.startswith("gemm9<") for k in kernel_timer.summary())
    kernel_timer.enable(False)
    ref = x.float() @ w.float().t() + b.to(torch.bfloat16).float()
    if act:
        ref = F.gelu(ref, approximate="tanh")
    err = float((y.float() - ref).abs().max() / ref.abs().max())
    assert y.dtype == torch.bfloat16 and y.shape == (2, M // 2, N) and err < 8e-3
