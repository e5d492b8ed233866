"""Microbench: fused HIP attention (csrc/attention.hip) vs torch SDPA (AOTriton) on the
SigLIP2-L shape (B=32, 1024 tokens, 16 heads x 64) and the DINO ViT-S shape."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch
import torch.nn.functional as F

from torch_utils.ops import attn_hip


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


for B, N, H in [(32, 1024, 16), (64, 197, 6), (32, 1025, 16)]:
    D = H * 64
    qkv = torch.randn(B, N, 3 * D, device="cuda", dtype=torch.bfloat16)
    flops = 4 * B * H * N * N * 64

    def hip():
        return attn_hip.attention_packed(qkv, H)

    def sdpa():
        q, k, v = qkv.view(B, N, 3, H, 64).permute(2, 0, 3, 1, 4).unbind(0)
        return F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, N, D)

    with torch.no_grad():
        th = bench(hip)
        ts = bench(sdpa)
    print(f"B={B} N={N} H={H}: hip {th:.3f} ms ({flops / th / 1e9:.1f} TF/s)   sdpa {ts:.3f} ms "
          f"({flops / ts / 1e9:.1f} TF/s)", flush=True)

# fp32 attention with gradients: adapter (packed qkv, 16 heads, 1024 tokens) and decoder
# (8 heads, 1024 queries / 1025 keys) shapes, forward and forward+backward
for B, Nq, Nk, H in [(32, 1024, 1024, 16), (32, 1024, 1025, 8)]:
    q = torch.randn(B, H, Nq, 64, device="cuda", requires_grad=True)
    k = torch.randn(B, H, Nk, 64, device="cuda", requires_grad=True)
    v = torch.randn(B, H, Nk, 64, device="cuda", requires_grad=True)
    do = torch.randn(B, H, Nq, 64, device="cuda")
    fl_f = 4 * B * H * Nq * Nk * 64
    fl_b = 2.5 * fl_f                # dV, dP, dQ, dK (+ S recompute not counted)
    res = {}
    for name, fn in (("hip", attn_hip.sdpa_f32), ("sdpa", F.scaled_dot_product_attention)):
        with torch.no_grad():
            tf = bench(lambda: fn(q, k, v))
        tfb = bench(lambda: torch.autograd.grad(fn(q, k, v), (q, k, v), do))
        res[name] = (tf, tfb - tf)
    print(f"f32 B={B} Nq={Nq} Nk={Nk} H={H}: " + "   ".join(
        f"{n} fwd {a:.3f} ms ({fl_f / a / 1e9:.1f} TF/s) bwd {b:.3f} ms ({fl_b / b / 1e9:.1f} TF/s)"
        for n, (a, b) in res.items()), flush=True)
