"""Which SDPA backend takes the decoder self-attention shapes (fp32, null-kv prepended), why
the fused ones reject, and their fwd+bwd times. python tools_dev/sdpa_probe.py"""
import time
import warnings

import torch
import torch.nn.functional as F
from torch.nn.attention import SDPBackend, sdpa_kernel

dev = torch.device("cuda")
torch.manual_seed(0)
for P in (64, 256, 1024):
    B, h, d = 32, 8, 64
    qkv = torch.randn(B, 3 * h * d, P, device=dev)
    q, k, v = qkv.reshape(B, 3, h, d, P).permute(1, 0, 2, 4, 3).unbind(0)
    nk = torch.randn(B, h, 1, d, device=dev)
    k = torch.cat([nk, k], 2)
    v = torch.cat([nk, v], 2)
    for name, be in (("math", SDPBackend.MATH), ("efficient", SDPBackend.EFFICIENT_ATTENTION),
                     ("flash", SDPBackend.FLASH_ATTENTION)):
        qq, kk, vv = (t.detach().contiguous().requires_grad_(True) for t in (q, k, v))
        try:
            with warnings.catch_warnings(record=True) as w, sdpa_kernel([be]):
                warnings.simplefilter("always")
                out = F.scaled_dot_product_attention(qq, kk, vv)
                out.sum().backward()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(5):
                    out = F.scaled_dot_product_attention(qq, kk, vv)
                    out.sum().backward()
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / 5 * 1e3
            print(f"P={P} {name}: ok {ms:.3f} ms fwd+bwd", flush=True)
        except Exception as e:  # noqa: BLE001
            msg = " | ".join(str(x.message)[:300] for x in w)
            print(f"P={P} {name}: rejected: {str(e)[:200]} :: {msg}", flush=True)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        qq = q.detach().clone().requires_grad_(True)
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
            F.scaled_dot_product_attention(qq, k, v).sum().backward()
            torch.cuda.synchronize()
    names = sorted({e.name[:60] for e in prof.events() if "attn" in e.name or "softmax" in e.name})
    print(f"P={P} default picks: {names}", flush=True)
# contiguous q/k/v variant at P=1024
P = 1024
q = torch.randn(B, h, P, d, device=dev, requires_grad=True)
k = torch.randn(B, h, P + 1, d, device=dev, requires_grad=True)
v = torch.randn(B, h, P + 1, d, device=dev, requires_grad=True)
for name, be in (("efficient", SDPBackend.EFFICIENT_ATTENTION),):
    try:
        with sdpa_kernel([be]):
            F.scaled_dot_product_attention(q, k, v).sum().backward()
        print("contiguous efficient ok", flush=True)
    except Exception as e:  # noqa: BLE001
        print("contiguous efficient rejected", str(e)[:300], flush=True)
