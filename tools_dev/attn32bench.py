"""Microbench of the fp32 attention kernels (csrc/attention_f32.hip, f32x6 products) on the step's shapes:
the fusion adapter (B = 32, 1024 tokens, 16 heads x 64), the decoder's 32 x 32 self-attention with its
null key (1024 queries, 1025 keys, 8 heads) and the DINO ViT-S tower (197 tokens, 6 heads). TF/s =
fp32 FLOPs of the op (4 Nq Nk d per head forward, 10 backward) / time. ATTN32_ONLY=adapter runs one shape
(the rocprofv3 --pmc target)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch  # noqa: E402

from torch_utils.ops import attn_hip  # noqa: E402


def bench(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


only = os.environ.get("ATTN32_ONLY")
for name, B, Nq, Nk, H in [("adapter", 32, 1024, 1024, 16), ("decoder32", 32, 1024, 1025, 8), ("dino", 32, 197, 197, 6)]:
    if only and name != only:
        continue
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn(B, H, Nq, 64, device="cuda", generator=g).requires_grad_(True)
    k = torch.randn(B, H, Nk, 64, device="cuda", generator=g).requires_grad_(True)
    v = torch.randn(B, H, Nk, 64, device="cuda", generator=g).requires_grad_(True)
    do = torch.randn(B, H, Nq, 64, device="cuda", generator=g)
    fl = 4.0 * B * H * Nq * Nk * 64

    def fwd():
        with torch.no_grad():
            attn_hip.sdpa_f32(q, k, v)

    def fb():
        o = attn_hip.sdpa_f32(q, k, v)
        torch.autograd.grad(o, (q, k, v), do)

    tf, tfb = bench(fwd), bench(fb)
    print(f"{name:10s} fwd {tf * 1e3:8.1f} us {fl / tf / 1e9:6.1f} TF/s | bwd {(tfb - tf) * 1e3:8.1f} us "
          f"{2.5 * fl / (tfb - tf) / 1e9:6.1f} TF/s", flush=True)
