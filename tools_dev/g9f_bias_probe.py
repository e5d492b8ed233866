"""Debug probe: a small fp32 MLP on torch_utils.ops.linear (forward linears with bias) whose gradients are
compared between biased f32x6 products on gemm9 (VFM_G9F_BIAS semantics) and on the previous route."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch  # noqa: E402

from torch_utils.ops import gemm_hip, linear  # noqa: E402

torch.manual_seed(0)
T, C, H = 1024, 1024, 4096
l1 = linear.Linear(C, H).cuda()
l2 = linear.Linear(H, C).cuda()
x0 = torch.randn(T, C, device="cuda")


def run(bias9, plan):
    gemm_hip.G9F_BIAS, gemm_hip.G9F_PLAN, gemm_hip.SPLIT9F = bias9, plan, False
    for p in (l1.weight, l1.bias, l2.weight, l2.bias):
        p.grad = None
    x = x0.clone().requires_grad_(True)
    y = l2(torch.nn.functional.gelu(l1(x)))
    (y * torch.linspace(-1, 1, y.numel(), device="cuda").view_as(y)).sum().backward()
    torch.cuda.synchronize()
    return y.detach(), [t.detach().clone() for t in (x.grad, l1.weight.grad, l1.bias.grad, l2.weight.grad, l2.bias.grad)]


def ref():
    x = x0.double().requires_grad_(True)
    w1, b1, w2, b2 = (p.detach().double().requires_grad_(True) for p in (l1.weight, l1.bias, l2.weight, l2.bias))
    y = torch.nn.functional.linear(torch.nn.functional.gelu(torch.nn.functional.linear(x, w1, b1)), w2, b2)
    (y * torch.linspace(-1, 1, y.numel(), device="cuda", dtype=torch.float64).view_as(y)).sum().backward()
    return y.detach(), [x.grad, w1.grad, b1.grad, w2.grad, b2.grad]


yr, gr = ref()
for bias9, plan in ((False, True), (True, True), (False, False), (True, False)):
    y, gs = run(bias9, plan)
    ey = float((y.double() - yr).abs().max() / yr.abs().max())
    eg = [float((g.double() - r).abs().max() / r.abs().max()) for g, r in zip(gs, gr)]
    print(f"bias9={bias9} plan={plan}: y {ey:.2e} grads (x, W1, b1, W2, b2) " + " ".join(f"{e:.2e}" for e in eg), flush=True)
