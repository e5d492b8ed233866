import sys, torch
sys.path[:0] = ['/root/repo/vfm-vae_amd', '/root/repo'] if len(sys.argv) < 2 else [sys.argv[1] + '/vfm-vae_amd', sys.argv[1]]
from torch_utils.ops import gemm_hip
gemm_hip.G9_F32 = True
def rel(a, b): return float((a.double()-b.double()).abs().max()/b.double().abs().max())
g = torch.Generator().manual_seed(0)
for (M, N, K) in [(512, 512, 2048), (512, 512, 8192), (1024, 256, 4096), (768, 1024, 1024), (3072, 1024, 1024), (256, 1024, 4096)]:
    for a_kc in (True, False):
        for b_kc in (True, False):
            A = (torch.rand(M, K, generator=g)*2-1).cuda(); Bt = (torch.rand(N, K, generator=g)*2-1).cuda()
            a = A if a_kc else A.t().contiguous().t()
            b = Bt.t() if b_kc else Bt.t().contiguous()
            ref = A.double() @ Bt.double().t()
            out = gemm_hip.try_gemm(a, b, route=("g8", 0))
            auto = gemm_hip.try_gemm(a, b, auto=True)
            print(M, N, K, a_kc, b_kc, "unsplit %.2e" % rel(out, ref), "auto %.2e" % rel(auto, ref), "vendor %.2e" % rel(a @ b, ref), flush=True)
