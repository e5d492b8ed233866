"""Microbench: the ConvNeXt MLP of the wide bf16 decoder blocks (b3: C = 512 at 64^2, b4: C = 256 at
128^2, batch 32) -- fused (gemm8 + GELU epilogues, decoder_hip._ConvNeXtMLPGemm) vs the unfused
chain (hipBLASLt 1x1s + scale_bias_gelu + layer_scale_residual): no-grad forward, autograd forward,
backward; plus the bare bf16 GEMM shapes of those layers on gemm8 vs hipBLASLt."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch

from torch_utils import custom_ops
from torch_utils.ops import decoder_hip, gemm_hip

lib = custom_ops.get_native()


def bench(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def rnd(*shape, dt=torch.bfloat16, scale=1.0):
    return ((torch.rand(*shape, device="cuda") * 2 - 1) * scale).to(dt)


B = int(os.environ.get("MLP_B", "32"))
for C, H in [(512, 64), (256, 128)]:
    P = H * H
    m, x_in = rnd(B, C, P), rnd(B, C, P)
    w1, w2 = rnd(4 * C, C, dt=torch.float32, scale=C ** -0.5), rnd(C, 4 * C, dt=torch.float32, scale=0.5 * C ** -0.5)
    dcoef = torch.rand(B, 4 * C, device="cuda") + 0.5
    b1, b2, gamma = rnd(4 * C, dt=torch.float32), rnd(C, dt=torch.float32), rnd(C, dt=torch.float32)
    dout = rnd(B, C, P)
    leaves = [m, w1, dcoef, b1, w2, b2, gamma, x_in]

    def unfused(ts):
        h = decoder_hip.pointwise(ts[1], ts[0])
        g = decoder_hip.scale_bias_gelu(h, ts[2], ts[3])
        y = decoder_hip.pointwise(ts[4], g)
        return decoder_hip.layer_scale_residual(y, ts[5], ts[6], ts[7])

    def fused(ts):
        return decoder_hip._ConvNeXtMLPGemm.apply(*ts, None)

    res = {}
    for name, fn in [("fused", fused), ("unfused", unfused)]:
        with torch.no_grad():
            res[name + " nograd"] = bench(lambda: fn(leaves) if name == "unfused" else decoder_hip._mlp_gemm_nograd(*leaves))
        ts = [t.detach().clone().requires_grad_(True) for t in leaves]
        res[name + " fwd"] = bench(lambda: fn(ts))
        res[name + " fwd+bwd"] = bench(lambda: fn(ts).backward(dout))
    print(f"C={C} {H}^2 B={B}: " + " | ".join(f"{k} {v:8.1f}us" for k, v in res.items()), flush=True)

    wb = w1.to(torch.bfloat16)
    w2b = w2.to(torch.bfloat16)
    g = rnd(B, 4 * C, P)
    fl1 = 2.0 * B * 4 * C * C * P
    for nm, A, Bm in [("W1 m", wb, m), ("W2 g", w2b, g), ("W2^T dy", w2b.t(), dout), ("W1^T dh", wb.t(), g)]:
        t8 = bench(lambda: gemm_hip.try_gemm(A, Bm, route=("g8", 0)))
        tb = bench(lambda: torch.bmm(A.expand(B, *A.shape), Bm))
        print(f"   {nm:8s} gemm8 {t8:8.1f}us {fl1 / t8 / 1e6:7.1f} TF/s | blas {tb:8.1f}us {fl1 / tb / 1e6:7.1f} TF/s",
              flush=True)
    s_ = dcoef
    t8 = bench(lambda: decoder_hip.gemm_gelu_fwd(wb, m, s_, b1, want_h=True))
    t8n = bench(lambda: decoder_hip.gemm_gelu_fwd(wb, m, s_, b1, want_h=False))
    h = rnd(B, 4 * C, P)
    t8b = bench(lambda: decoder_hip.gemm_gelu_bwd(w2b.t().contiguous(), dout, h, s_, b1))
    gb = (2 * B * 4 * C * P * 2) / 1e3
    print(f"   gelu-epilogue GEMMs: fwd(h,g) {t8:8.1f}us ({gb * 2 / t8:5.2f} TB/s out) | fwd(g) {t8n:8.1f}us | "
          f"bwd {t8b:8.1f}us", flush=True)
    with torch.no_grad():
        tgf = bench(lambda: decoder_hip.scale_bias_gelu(h, s_, b1))
    hr = h.clone().requires_grad_(True)
    dg = rnd(B, 4 * C, P)
    tgb = bench(lambda: decoder_hip.scale_bias_gelu(hr, s_, b1).backward(dg)) - tgf
    print(f"   unfused epilogue kernels: scale_bias_gelu fwd {tgf:8.1f}us | bwd {tgb:8.1f}us", flush=True)
