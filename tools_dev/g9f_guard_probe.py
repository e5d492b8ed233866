"""Debug probe: f32x6 gemm9 products (vfm_gemm9_pieces, bias epilogue) with C, A and B placed inside guarded
buffers; reports any write outside C and any change of A / B / bias."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch  # noqa: E402

from torch_utils.ops import gemm_hip  # noqa: E402

gemm_hip.G9_F32 = True
G = 1 << 20
g = torch.Generator().manual_seed(0)
for (M, N, K, bias_dim) in [(256, 128, 64, 1), (1024, 1024, 4096, 1), (256, 768, 2304, 1), (1024, 3072, 1024, 1),
                            (1024, 4096, 1024, 1), (256, 512, 512, 1), (1024, 128, 64, 1), (512, 256, 512, 0)]:
    A = (torch.rand(M, K, generator=g) * 2 - 1).cuda()
    Bt = (torch.rand(N, K, generator=g) * 2 - 1).cuda()
    bias = torch.rand(M if bias_dim == 0 else N, generator=g).cuda()
    buf = torch.full((2 * G + M * N,), 12345.0, device="cuda")
    out = buf[G:G + M * N].view(M, N)
    A0, B0, b0 = A.clone(), Bt.clone(), bias.clone()
    r = gemm_hip.try_gemm(A, Bt.t(), out=out, bias=bias, bias_dim=bias_dim, route=("g8", 0))
    torch.cuda.synchronize()
    pre = int((buf[:G] != 12345.0).sum()); post = int((buf[G + M * N:] != 12345.0).sum())
    ref = A.double() @ Bt.double().t() + (bias.double()[:, None] if bias_dim == 0 else bias.double())
    e = float((out.double() - ref).abs().max() / ref.abs().max())
    print(M, N, K, bias_dim, "guard writes before/after", pre, post, "A/B/bias changed",
          not torch.equal(A, A0), not torch.equal(Bt, B0), not torch.equal(bias, b0), "err %.2e" % e, flush=True)
