"""Microbenchmark: decoder 1x1-conv GEMMs in the NCHW batched form (stride-0 batch bmm)
vs the channels-last single-GEMM form, forward / data-grad / weight-grad, for every
decoder block shape at batch 32. Prints achieved TFLOP/s per variant.
  python tools_dev/gemm_probe.py"""
import torch

B = 32
# (label, C, res, dtype)   pwconv1: C -> 4C, pwconv2: 4C -> C
SHAPES = [("b0", 512, 8, torch.float32), ("b1", 512, 16, torch.float32), ("b2", 512, 32, torch.float32),
          ("b3", 512, 64, torch.bfloat16), ("b4", 256, 128, torch.bfloat16), ("b5", 128, 256, torch.bfloat16)]


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
    return s.elapsed_time(e) / iters


def main():
    torch.backends.cuda.matmul.allow_tf32 = False
    dev = "cuda"
    for label, C, r, dt in SHAPES:
        P = r * r
        for (I, O) in ((C, 4 * C), (4 * C, C)):
            fl = 2.0 * B * P * I * O
            W = torch.randn(O, I, device=dev, dtype=dt)
            xn = torch.randn(B, I, P, device=dev, dtype=dt)
            dyn = torch.randn(B, O, P, device=dev, dtype=dt)
            xc = torch.randn(B * P, I, device=dev, dtype=dt)
            dyc = torch.randn(B * P, O, device=dev, dtype=dt)
            res = {}
            res["nchw_fwd"] = timeit(lambda: torch.bmm(W.expand(B, O, I), xn))
            res["nhwc_fwd"] = timeit(lambda: xc @ W.t())
            res["nchw_dx"] = timeit(lambda: torch.bmm(W.t().expand(B, I, O), dyn))
            res["nhwc_dx"] = timeit(lambda: dyc @ W)
            if dt == torch.float32:
                res["nchw_dw"] = timeit(lambda: torch.bmm(dyn, xn.transpose(1, 2)).sum(0))
            else:
                res["nchw_dw"] = timeit(lambda: torch.bmm(dyn, xn.transpose(1, 2), out_dtype=torch.float32).sum(0))
            res["nhwc_dw"] = timeit(lambda: dyc.t() @ xc)
            line = " ".join(f"{k}={fl / v / 1e9:7.1f}" for k, v in res.items())
            print(f"{label} {str(dt)[6:]:8s} I={I:5d} O={O:5d} P={P:6d}  TFLOP/s: {line}", flush=True)


if __name__ == "__main__":
    main()
