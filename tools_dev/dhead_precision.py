import os, sys, torch
sys.path.insert(0, "vfm-vae_amd")
from networks.discriminator import make_block
def _rel2(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))
for B,C,L,k in [(16,384,196,9),(8,64,33,9),(16,384,256,9)]:
    torch.manual_seed(B + L)
    blk = make_block(C, k)
    blk[1].weight.data.normal_(1.0, 0.2); blk[1].bias.data.normal_(0.0, 0.2)
    x = torch.randn(B, C, L); r = torch.randn(B, C, L)
    state = {kk: v.detach().clone().double() for kk, v in blk.state_dict().items()}
    bg = blk.cuda().eval(); xg = x.cuda().requires_grad_()
    y = bg(xg); (y * r.cuda()).sum().backward()
    bc = make_block(C, k).double().eval(); bc.load_state_dict(state)
    xc = x.double().requires_grad_(); yc = torch.nn.Sequential.forward(bc, xc); (yc * r.double()).sum().backward()
    print(os.environ.get("VFM_DHEAD_GEMM"), B, C, L, k, "y", _rel2(y, yc), "dx", _rel2(xg.grad, xc.grad), {n: round(_rel2(p.grad, q.grad), 8) for (n, p), q in zip(bg[0].named_parameters(), bc[0].parameters()) if p.grad is not None}, flush=True)

# localise: which of the three products (forward, dcols, dW) on our GEMM moves the gradients
from torch_utils.ops import patchgan_hip
_own = patchgan_hip._gemm_or_mm
for use_torch in ((0,), (1,), (2,), (0, 1, 2), ()):
    calls = [0]

    def pick(A, B, bias=None, **kw):
        i = calls[0] % 3
        calls[0] += 1
        if i in use_torch:
            return torch.mm(A, B) if bias is None else torch.addmm(bias[:, None], A, B)
        return _own(A, B, bias=bias, **kw)
    patchgan_hip._gemm_or_mm = pick
    B, C, L, k = 16, 384, 196, 9
    torch.manual_seed(B + L)
    blk = make_block(C, k)
    blk[1].weight.data.normal_(1.0, 0.2); blk[1].bias.data.normal_(0.0, 0.2)
    x = torch.randn(B, C, L); r = torch.randn(B, C, L)
    state = {kk: v.detach().clone().double() for kk, v in blk.state_dict().items()}
    bg = blk.cuda().eval(); xg = x.cuda().requires_grad_()
    y = bg(xg); (y * r.cuda()).sum().backward()
    bc = make_block(C, k).double().eval(); bc.load_state_dict(state)
    xc = x.double().requires_grad_(); yc = torch.nn.Sequential.forward(bc, xc); (yc * r.double()).sum().backward()
    print("torch for products", use_torch, "calls", calls[0], "y", _rel2(y, yc), "dx", _rel2(xg.grad, xc.grad), flush=True)

# the forward product itself: ours vs hipBLASLt vs fp64 (norm-wise and worst row)
def fwd_stats(A, B, bias=None, **kw):
    ref = A.double() @ B.double() + (0 if bias is None else bias.double()[:, None])
    own = _own(A, B, bias=bias, **kw)
    tm = torch.mm(A, B) if bias is None else torch.addmm(bias[:, None], A, B)
    for name, o in (("own", own), ("torch", tm)):
        e = (o.double() - ref)
        row = e.norm(dim=1) / ref.norm(dim=1)
        print(name, "rel", float(e.norm() / ref.norm()), "worst row", float(row.max()), "max abs", float(e.abs().max()),
              "bias", None if bias is None else float(bias.abs().max()), flush=True)
    return own


patchgan_hip._gemm_or_mm = fwd_stats
torch.manual_seed(16 + 196)
blk = make_block(384, 9)
bg = blk.cuda().eval()
with torch.no_grad():
    bg(torch.randn(16, 384, 196).cuda())
