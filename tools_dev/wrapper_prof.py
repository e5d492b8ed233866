"""cProfile of the GEMM wrapper (gemm_hip.try_gemm) per call: where its host time goes (tools_dev/wrapper_cost.py setup)."""
import cProfile, pstats, sys, os
sys.argv = ["x"]
ROOT = "/root/repo"
sys.path[:0] = [ROOT, os.path.join(ROOT, "vfm-vae_amd"), os.path.join(ROOT, "tools_dev")]
exec(open(os.path.join(ROOT, "tools_dev", "wrapper_cost.py")).read().split("cost(\"try_gemm bf16")[0])
f1 = lambda: gemm_hip.try_gemm(w32, a32, auto=True)
f2 = lambda: gemm_hip.try_gemm(a16, b16.t(), auto=True)
for f in (f1, f2):
    for _ in range(100): f()
    pr = cProfile.Profile(); pr.enable()
    for _ in range(3000): f()
    pr.disable(); torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)
