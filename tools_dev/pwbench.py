"""Time the fused channel GEMM + GELU (vfm_pw_gemm_gelu) against the unfused
hipBLASLt bmm + GELU row kernel at the bf16 decoder shapes (batch 32)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vfm-vae_amd"))
from torch_utils import custom_ops  # noqa: E402
from torch_utils.ops import decoder_hip  # noqa: E402

SHAPES = {"b3 C512 64^2": (512, 4096), "b4 C256 128^2": (256, 16384), "b5 C128 256^2": (128, 65536)}


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    lib = custom_ops.get_native()
    st = custom_ops.stream_ptr()
    B = 32
    for name, (C, N) in SHAPES.items():
        M, K = 4 * C, C
        A = (torch.randn(M, K, device="cuda") / K ** 0.5).bfloat16()
        X = torch.randn(B, K, N, device="cuda").bfloat16()
        s = torch.rand(B, M, device="cuda") + 0.5
        bias = torch.randn(M, device="cuda")
        h = torch.empty(B, M, N, dtype=torch.bfloat16, device="cuda")
        g = torch.empty_like(h)
        tiles = N // 64
        p0 = torch.empty(B, tiles, M, device="cuda")
        p1 = torch.empty_like(p0)
        ux = B * K * N * 2
        uh = B * M * N * 2
        f_grad = lambda: lib.vfm_pw_gemm_gelu(A.data_ptr(), X.data_ptr(), s.data_ptr(), bias.data_ptr(), None,
                                              h.data_ptr(), g.data_ptr(), None, None, 0, B, M, K, N, st)
        f_nograd = lambda: lib.vfm_pw_gemm_gelu(A.data_ptr(), X.data_ptr(), s.data_ptr(), bias.data_ptr(), None,
                                                None, g.data_ptr(), None, None, 0, B, M, K, N, st)
        f_bwd = lambda: lib.vfm_pw_gemm_gelu(A.data_ptr(), X.data_ptr(), s.data_ptr(), bias.data_ptr(),
                                             h.data_ptr(), g.data_ptr(), None, p0.data_ptr(), p1.data_ptr(), 1,
                                             B, M, K, N, st)

        def unfused_fwd():
            hh = torch.bmm(A.expand(B, M, K), X)
            return decoder_hip.scale_bias_gelu(hh, s, bias)

        def unfused_bwd():
            dg = torch.bmm(A.expand(B, M, K), X)
            return decoder_hip._gelu_bwd_only(h, dg, s, bias) if hasattr(decoder_hip, "_gelu_bwd_only") else dg

        t1, t2, t3 = timeit(f_grad), timeit(f_nograd), timeit(f_bwd)
        tm = None
        if C in (128, 256):
            W2 = (torch.randn(C, M, device="cuda") / M ** 0.5).bfloat16()
            xin = torch.randn(B, C, N, device="cuda").bfloat16()
            outm = torch.empty_like(xin)
            b2 = torch.randn(C, device="cuda")
            gam = torch.randn(C, device="cuda")
            tm = timeit(lambda: lib.vfm_convnext_mlp_fwd(A.data_ptr(), X.data_ptr(), s.data_ptr(), bias.data_ptr(),
                                                         W2.data_ptr(), b2.data_ptr(), gam.data_ptr(), xin.data_ptr(),
                                                         outm.data_ptr(), None, None, None, B, C, N, st))
            ym = torch.empty_like(xin)
            tmg = timeit(lambda: lib.vfm_convnext_mlp_fwd(A.data_ptr(), X.data_ptr(), s.data_ptr(), bias.data_ptr(),
                                                          W2.data_ptr(), b2.data_ptr(), gam.data_ptr(), xin.data_ptr(),
                                                          outm.data_ptr(), h.data_ptr(), g.data_ptr(), ym.data_ptr(),
                                                          B, C, N, st))
            print(f"{name}: whole MLP fwd saving h/g/y {tmg:8.1f} us {(4 * ux + 2 * uh) / tmg / 1e3:6.0f} GB/s",
                  flush=True)
        t4 = timeit(unfused_fwd)
        t5 = timeit(lambda: torch.bmm(A.expand(B, M, K), X))
        print(f"{name}: fused fwd(h+g) {t1:8.1f} us {(ux + 2 * uh) / t1 / 1e3:7.0f} GB/s | fwd(g) {t2:8.1f} us "
              f"{(ux + uh) / t2 / 1e3:7.0f} GB/s | bwd {t3:8.1f} us {(ux + 2 * uh) / t3 / 1e3:7.0f} GB/s | "
              f"unfused fwd {t4:8.1f} us (bmm alone {t5:8.1f} us)"
              + (f" | whole MLP fwd {tm:8.1f} us {3 * ux / tm / 1e3:6.0f} GB/s" if tm else ""), flush=True)


if __name__ == "__main__":
    main()
