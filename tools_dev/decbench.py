"""Micro-benchmark of the decoder HIP kernels at the f16d32 batch-32 shapes.

Prints per kernel: average microseconds, algorithmic GB/s (unique inputs + outputs), and
for the depthwise convs the fp32 VALU TFLOP/s (2*K*K flop per output).
  python tools_dev/decbench.py [--only dw,gn,dwgn,gelu,lsr,blur]
dwgn: the ConvNeXt dwconv -> GroupNorm pair (bf16 blocks), with the GroupNorm statistics from the
dwconv's partials (decoder_hip.GN_STATS) and without."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]
import torch  # noqa: E402

from torch_utils.ops import decoder_hip  # noqa: E402

B = 32
# block: (C, res, K, dtype)
BLOCKS = {"b1": (512, 16, 5, torch.float32), "b2": (512, 32, 7, torch.float32), "b3": (512, 64, 7, torch.bfloat16),
          "b4": (256, 128, 7, torch.bfloat16), "b5": (128, 256, 7, torch.bfloat16)}


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3      # us


def report(name, us, nbytes, flops=None):
    line = f"{name:40s} {us:9.1f} us  {nbytes / us / 1e3:8.1f} GB/s"
    if flops:
        line += f"  {flops / us / 1e6:7.1f} TFLOP/s"
    print(line, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="dw,gn,gelu,lsr,blur")
    args = ap.parse_args()
    only = set(args.only.split(","))
    dev = "cuda"
    lib = decoder_hip._lib
    for bname, (C, R, K, dt) in BLOCKS.items():
        x = torch.randn(B, C, R, R, device=dev, dtype=dt)
        es = x.element_size()
        n = x.numel()
        if "dw" in only:
            w = torch.randn(C, K, K, device=dev) * 0.1
            b = torch.randn(C, device=dev)
            pad = K // 2
            us = timeit(lambda: decoder_hip._dw_fwd(x, w, b, None, pad, "dw"))
            report(f"{bname} dwconv{K} fwd {str(dt)[6:]}", us, 2 * n * es, 2 * K * K * n)
            tiles = lib.vfm_dwconv2d_bwd_weight_tiles(B, C, R, R, K, pad)
            part = torch.empty([tiles, B * C, K * K + 1], dtype=torch.float32, device=dev)
            dy = torch.randn_like(x)

            def bw():
                decoder_hip._check(lib.vfm_dwconv2d_bwd_weight(x.data_ptr(), dy.data_ptr(), part.data_ptr(),
                                                               decoder_hip._code(x), B, C, R, R, K, pad,
                                                               decoder_hip._stream()), "bw")
            us = timeit(bw)
            report(f"{bname} dwconv{K} bwd_w {str(dt)[6:]}", us, 2 * n * es, 2 * K * K * n)
        if "gn" in only:
            G = min(32, C // 4)
            gw, gb = torch.randn(C, device=dev), torch.randn(C, device=dev)
            st = torch.rand(B, C, device=dev)
            us = timeit(lambda: decoder_hip.group_norm(x, G, gw, gb, 1e-5, dt, st))
            report(f"{bname} group_norm fwd", us, 2 * n * es)
            xr = x.clone().requires_grad_(True)
            y = decoder_hip.group_norm(xr, G, gw, gb, 1e-5, dt, st)
            gy = torch.randn_like(y)
            us = timeit(lambda: torch.autograd.grad(y, xr, gy, retain_graph=True))
            report(f"{bname} group_norm bwd", us, 3 * n * es)
        if "dwgn" in only and dt == torch.bfloat16:
            w = torch.randn(C, K, K, device=dev) * 0.1
            b = torch.randn(C, device=dev)
            G = min(32, C // 4)
            gw, gb = torch.randn(C, device=dev), torch.randn(C, device=dev)
            st = torch.rand(B, C, device=dev)
            for fused in (False, True):
                decoder_hip.GN_STATS = fused

                def pair():
                    d = decoder_hip._dw_fwd(x, w, b, None, K // 2, "dwconv2d_fwd", gstat=True)
                    decoder_hip.group_norm(d, G, gw, gb, 1e-5, dt, st)
                us = timeit(pair)
                report(f"{bname} dwconv{K}+group_norm {'fused' if fused else 'plain'}", us, 4 * n * es)
            decoder_hip.GN_STATS = True
        if "gelu" in only:
            h = torch.randn(B, 4 * C, R * R, device=dev, dtype=dt)
            sc, bi = torch.rand(B, 4 * C, device=dev), torch.randn(4 * C, device=dev)
            us = timeit(lambda: decoder_hip.scale_bias_gelu(h, sc, bi))
            report(f"{bname} scale_bias_gelu fwd", us, 2 * h.numel() * es)
            hr = h.clone().requires_grad_(True)
            g = decoder_hip.scale_bias_gelu(hr, sc, bi)
            gg = torch.randn_like(g)
            us = timeit(lambda: torch.autograd.grad(g, hr, gg, retain_graph=True))
            report(f"{bname} scale_bias_gelu bwd", us, 3 * h.numel() * es)
        if "lsr" in only:
            yv = torch.randn(B, C, R * R, device=dev, dtype=dt)
            bb, gm = torch.randn(C, device=dev), torch.randn(C, device=dev)
            xi = torch.randn(B, C, R * R, device=dev, dtype=dt)
            us = timeit(lambda: decoder_hip.layer_scale_residual(yv, bb, gm, xi))
            report(f"{bname} layer_scale_residual fwd", us, 3 * n * es)
        if "blur" in only:
            taps = [1, 2, 1] if bname in ("b1", "b2") else [1, 4, 6, 4, 1]
            xs = torch.randn(B, 4 * C, R // 2, R // 2, device=dev, dtype=dt)
            us = timeit(lambda: decoder_hip.shuffle_blur(xs, taps, 2))
            report(f"{bname} shuffle_blur{len(taps)} fwd", us, 2 * xs.numel() * es)
            xr = xs.clone().requires_grad_(True)
            y = decoder_hip.shuffle_blur(xr, taps, 2)
            gy = torch.randn_like(y)
            us = timeit(lambda: torch.autograd.grad(y, xr, gy, retain_graph=True))
            report(f"{bname} shuffle_blur{len(taps)} bwd", us, 2 * xs.numel() * es)


if __name__ == "__main__":
    main()
