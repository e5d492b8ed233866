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
