"""MFMA GEMM with fused epilogues (csrc/gemm.hip, C ABI `vfm_gemm` in include/vfmvae.h).

Replaces hipBLASLt (torch.addmm / torch.bmm) on the hot path's dense products: the frozen
ViT projections (bf16, bias / bias+tanh-GELU epilogue; reference
networks/utils/vfms/siglip2_utils.py:121), and the fp32 1x1 convolutions / linear layers of
the decoder, fusion adapter and discriminators (convnext_utils.py:36-142,
gigagan_utils.py:53-185, ldm_utils.py:55-166), whose fp32 operands run as bf16 MFMA products
of exact piece splits: `f32x6` (default, fp32-equivalent: six piece products, dropped terms
<= ~2^-23 relative) or the opt-in `f32x3` (custom_ops.F32_PRODUCTS; csrc/gemm.hip header).

`gemm(A, B, ...)` takes 2-D or batched 3-D views and the layout of each operand, so no
transposes are materialised. A missing kernel library raises; shapes the kernel does not
cover (contiguous extents not multiples of 8/4 elements) return None from `try_gemm` so the
caller can take its torch path explicitly.
"""
import torch

from .. import custom_ops
from . import kernel_timer

_lib = custom_ops.get_native()
_CODES = {torch.float32: 0, torch.bfloat16: 2}
ACTS = {None: 0, "gelu_tanh": 1, "gelu": 2}


def _layout(t, kdim_last):
    """(is_k_contiguous, leading dim, batch stride) of a [z, rows, cols] / [rows, cols] operand
    view whose last two dims are (outer, k) if kdim_last else (k, outer)."""
    if t.dim() == 2:
        t = t.unsqueeze(0)
        sb = 0
    else:
        sb = t.stride(0) if t.shape[0] > 1 else 0
    r, c = t.stride(1), t.stride(2)
    if c == 1 or t.shape[2] == 1:
        return kdim_last, r, sb
    if r == 1 or t.shape[1] == 1:
        return (not kdim_last), c, sb
    return None


FAST = True                 # large-tile LDS-DMA kernel (csrc/gemm8.hip) where it applies
SPLIT8 = __import__("os").environ.get("VFM_GEMM8_SPLIT", "0") == "1"
FAST_MIN_MN = 1 << 18       # below ~256k outputs the 128-tile kernel fills the chip better


def _split_f32(t3, R, K, kc, ld, sb, cache, stream):
    """bf16 pieces ([hi | mid | lo] for f32x6, [hi | lo] for f32x3) of an fp32 operand view t3
    [z, R, K] (kc: K-contiguous) stacked along K -> (tensor, kcont, ld, batch stride); cached on the
    tensor's storage owner until its version moves when `cache` (parameters)."""
    prec, npc, _ = custom_ops.f32_precision()
    z = t3.shape[0] if sb else 1
    key = None
    if cache:
        base = t3._base if t3._base is not None else t3
        key = (t3.data_ptr(), tuple(t3.shape), t3.stride(), base._version, prec)
        hit = getattr(base, "_vfm_split_f32", None)
        if hit is not None and hit[0] == key and not torch.cuda.is_current_stream_capturing():
            return hit[1]
    if kc:
        dst = torch.empty((z, R, npc * K), dtype=torch.bfloat16, device=t3.device)
        res = (dst, True, npc * K, R * npc * K if sb else 0)
    else:
        dst = torch.empty((z, npc * K, R), dtype=torch.bfloat16, device=t3.device)
        res = (dst, False, R, npc * K * R if sb else 0)
    rc = _lib.vfm_split_f32(t3.data_ptr(), dst.data_ptr(), R, K, ld, sb, res[3], z, prec, int(kc), stream)
    if rc == custom_ops.VFM_NO_KERNEL:
        return None, None, None, None
    custom_ops.check(rc, "vfm_split_f32")
    if key is not None and not torch.cuda.is_current_stream_capturing():
        try:
            base._vfm_split_f32 = (key, res)
        except AttributeError:
            pass
    return res


PLANAR = __import__("os").environ.get("VFM_PLANAR_PIECES", "1") == "1"


def _planar(t3, stream):
    """Planar bf16 pieces [np][numel] of the contiguous fp32 tensor that the operand view t3 covers
    whole (a transpose / unsqueeze of it), cached on that tensor until its version moves, so one
    split serves every product the tensor enters (an activation's forward product and the backward's
    weight gradient, a weight's forward and data-gradient products) -> (pieces, element offset of
    t3's origin, piece stride) or None (the per-product stacked split then applies)."""
    if not PLANAR:
        return None
    base = t3._base if t3._base is not None else t3
    n = base.numel()
    if base.dtype != torch.float32 or not base.is_contiguous() or t3.numel() != n:
        return None
    prec, npc, _ = custom_ops.f32_precision()
    off = (t3.data_ptr() - base.data_ptr()) // 4
    if n % 8 or off % 8 or n * npc * 2 >= (1 << 31):
        return None
    capturing = torch.cuda.is_current_stream_capturing()
    key = (base.data_ptr(), n, base._version, prec)
    hit = getattr(base, "_vfm_planar", None)
    if hit is not None and hit[0] == key and not capturing:
        return hit[1], off, n
    dst = torch.empty((npc, n), dtype=torch.bfloat16, device=base.device)
    rc = _lib.vfm_split_f32(base.data_ptr(), dst.data_ptr(), 1, n, n, 0, 0, 1, prec, 1, stream)
    if rc == custom_ops.VFM_NO_KERNEL:
        return None
    custom_ops.check(rc, "vfm_split_f32")
    if not capturing:
        try:
            base._vfm_planar = (key, dst)
        except AttributeError:
            pass
    return dst, off, n


BF16_OWN = __import__("os").environ.get("VFM_BF16_GEMM", "hip") == "hip"
# fp32 products narrower than 128 (the 8^2 / 16^2 decoder blocks' 1x1s): the exact-fp32 GEMM (`sgemm`,
# csrc/sgemm.hip) by default; VFM_F32_SMALL=hip routes them to the f32x6 128-tile kernel, which measured slower
# at these shapes (r5o bench, profiles/r5_o_f32small_ab.txt)
F32_SMALL_OWN = __import__("os").environ.get("VFM_F32_SMALL", "torch") == "hip"
# bf16 products on gemm9 (csrc/gemm9.hip); False: gemm8's 256-tile pipeline (tests, A/B)
G9 = __import__("os").environ.get("VFM_GEMM9", "1") == "1"
# fp32 (f32x6) products of the 256-tile route on gemm9's persistent kernel (vfm_gemm9_pieces) instead of gemm8:
# same-box bench A/B +1.8 %, f32x6 GEMM time 70.6 -> 65.2 ms/step (profiles/r5_x_g9f32_ab.txt); VFM_GEMM9_F32=0: gemm8
G9_F32 = __import__("os").environ.get("VFM_GEMM9_F32", "1") == "1"


_WS = {}


def _workspace(n, dev):
    """fp32 scratch of at least n floats per (device, stream), reused by that stream's split-K products,
    which it orders (grown on demand; a HIP-graph capture gets a buffer of its own, kept alive by the
    graph's allocation)."""
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream)
    w = _WS.get(key)
    if w is None or w.numel() < n or torch.cuda.is_current_stream_capturing():
        w = torch.empty(n, dtype=torch.float32, device=dev)
        if not torch.cuda.is_current_stream_capturing():
            _WS[key] = w
    return w


def preferred(A, M, N, reduce_batch=False):
    """Where this kernel family is routed (tools_dev/gemmbench.py, tools_dev/g4bench.py, MI355X): fp32
    operands on the bf16-piece kernels (the fp32-equivalent split) at >= 128-wide outputs and for the
    batch-reduced weight gradients at any width -- narrower fp32 products go to the exact-fp32 kernel
    (`sgemm`, csrc/sgemm.hip); bf16 operands of any width on the LDS-DMA one-wave-per-SIMD kernel
    (csrc/gemm9.hip; single products with few output tiles over a deep K run split, `_plan`), or
    hipBLASLt under VFM_BF16_GEMM=torch (A/B)."""
    if A.dtype == torch.bfloat16:
        return BF16_OWN
    if A.dtype != torch.float32:
        return False
    return reduce_batch or (M >= 128 and N >= 128) or F32_SMALL_OWN


def _plan(dtype, M, N, K, z, reduce_batch, splits, auto):
    """Kernel and split of one product: ("g8", kchunk) -- the 256-tile kernel, kchunk virtual
    K-tiles per split (0: no split) -- or ("g128", splits) -- the 128-tile kernel. The rules follow
    tools_dev/gemm6bench.py on MI355X (profiles/r3_f_gemm6bench.txt, f32x6):
      * batch-reduced weight gradients: 256-tile split-K over the batch-concatenated K, 16 splits
        (b2 dW 2048x512x1024x32: 560 vs 583 us on the 128-tile kernel; b0: 66 vs 89 us);
      * fewer than SPLIT_TILES 256-tiles (token-major linears with a small output width, the DINO
        tower's 6304 x 384 / x 1152 products): the 128-tile kernel, which splits fp32 operands in
        registers and fills the chip with 4x the tiles (6304x384x1536: 95 us vs 101 us for the best
        256-tile split-K);
      * otherwise the 256-tile kernel."""
    if dtype == torch.bfloat16 and K % 64 == 0 and G9:
        if reduce_batch:
            # batch-reduced weight gradients (few output tiles over a deep reduction): ~2 items per CU
            tiles = -(-M // 256) * -(-N // 256)
            return "g9r", max(1, min(-(-512 // tiles), z * (K // 64) // 4))
        if splits <= 1:
            tiles = -(-M // 256) * -(-N // 256) * z
            if z == 1 and tiles < 128 and K >= 2048:
                # few output tiles over a deep reduction (e.g. a bf16 linear's weight gradient dy^T x, K =
                # tokens): K splits on gemm9 so the grid covers the CUs (unsplit it ran on `tiles` workgroups)
                return "g9r", max(1, min(-(-256 // tiles), K // 64 // 4))
            return "g9", 0
    if not FAST or K % 64:
        return "g128", splits
    nterm = 1 if dtype == torch.bfloat16 else (6 if custom_ops.f32_precision()[1] == 3 else 3)
    zo = 1 if reduce_batch else z
    V = nterm * (z if reduce_batch else 1) * (K // 64)            # virtual K-tiles per output
    tiles = -(-M // 256) * -(-N // 256) * zo
    if reduce_batch:
        if min(M, N) >= 256 and (SPLIT8 or auto):
            return "g8", max(4, -(-V // REDUCE_SPLITS))
        return "g128", splits
    if splits > 1:
        if not (SPLIT8 and min(M, N) >= 256):
            return "g128", splits
        S0 = max(1, -(-512 // tiles))
        return "g8", max(4, -(-V // S0))
    if M * N < FAST_MIN_MN:
        return "g128", splits
    if auto and tiles < SPLIT_TILES:
        return "g128", splits
    return "g8", 0


SPLIT_TILES = 128           # fewer 256-tiles than this: the 128-tile kernel (auto routing)


# f32x6 routing by _splits9f (batch-reduced weight gradients and few-tile products split on gemm9) instead of
# _plan's choice with gemm9 standing in for gemm8 only: opt-in (VFM_G9F_PLAN=1). Measured slower in the step
# (r5ai: 87.9 img/s, f32x6 GEMM time 65.4 -> 76.7 ms/step): the batched products with few tiles per sample ran
# unsplit at a fraction of the CUs, where the 128-tile kernel's K splits fill the chip
G9F_PLAN = __import__("os").environ.get("VFM_G9F_PLAN", "0") == "1"
SPLIT9F = __import__("os").environ.get("VFM_G9F_SPLIT", "1") == "1"     # 0: f32x6 single products unsplit (A/B)
# biased f32x6 products on gemm9 (VFM_G9F_BIAS=0: on gemm8 / the 128-tile kernel). Through the opt-in planner
# (G9F_PLAN) the few-tile biased linears of the adapter at batch 1 ran unsplit on gemm9 instead of split-K on the
# 128-tile kernel: each product within fp32 rounding of fp64 (3e-6, tools_dev/g9f_bias_probe.py; no stray writes,
# tools_dev/g9f_guard_probe.py) but the K-long fp32 sums are ~8x less accurate than the split ones, which the
# adapter's attention amplifies past the full-size backward pin's 2e-4 (projection errors up to 3e-3); on the
# default route gemm9 only stands in for gemm8, whose K order and rounding it shares
G9F_BIAS = __import__("os").environ.get("VFM_G9F_BIAS", "1") == "1"


_G9F_CHECK = __import__("os").environ.get("VFM_G9F_CHECK") == "1"


def _check9f(a3, b3, out, bias, bias_dim, alpha, reduce_batch, region, *info):
    """Debug (VFM_G9F_CHECK=1): an f32x6 gemm9 product against fp64 torch; prints the ones off by > 1e-5."""
    ref = alpha * torch.matmul(a3.double(), b3.double())
    if reduce_batch:
        ref = ref.sum(0)
    if bias is not None:
        ref = ref + (bias.double()[:, None] if bias_dim == 0 else bias.double())
    o = out.double().reshape(ref.shape) if out.numel() == ref.numel() else out.double()
    e = float((o - ref).abs().max() / (ref.abs().max() + 1e-30))
    if e > 1e-5:
        print(f"[g9f check] {region} A{tuple(a3.shape)}{a3.stride()} B{tuple(b3.shape)}{b3.stride()} bias_dim={bias_dim} "
              f"alpha={alpha} err {e:.2e} info {info}", flush=True)


DEEP9F = __import__("os").environ.get("VFM_G9F_DEEP", "1") == "1"


def _deep9f(M, N, K, z, reduce_batch):
    """The default f32x6 K-split on gemm9: single products with fewer 256-tiles than CUs over a deep reduction
    (the adapter's token-major weight gradients, K = 32 x 1024 tokens), cut into S chunks of at least 16 real
    K-tiles with tiles x S <= 256 (one round of items). tools_dev/g9f_routebench.py (r5aq): 4096x1024x32768
    1905 -> 1479 us, 1024x4096x32768 1828 -> 1451, 1024x1024x32768 557 -> 447 against the 128-tile kernel's
    split-K; at S = 6 for 48 tiles (288 items, a second round of 32) it lost (1578 -> 1980), and the DINO tower's
    K <= 1536 products lose on gemm9 at any split. None: the product keeps _plan's route."""
    if reduce_batch or not DEEP9F:
        return None
    tiles = -(-M // 256) * -(-N // 256) * z
    if tiles >= 256:
        return None
    if z > 1:
        # batched products with few tiles per sample (the 16^2 decoder block's 1x1s, 512 x 256 per sample over
        # K = 2048): chunks of at least 4 real K-tiles of each sample, partials combined per sample
        if K < 1024:
            return None
        S = min(256 // tiles, (K // 64) // 4)
        return S if S >= 2 else None
    if K < 8192:
        return None
    S = min(256 // tiles, (K // 64) // 16)
    return S if S >= 2 else None


def _splits9f(M, N, K, z, reduce_batch):
    """K splits of an f32x6 product on gemm9's persistent kernel (one workgroup per CU walking the items): the
    batch-reduced weight gradients and the single products with fewer output tiles than CUs (the DINO tower's
    6304 x 384 products, the token-major linears' weight gradients) cut their reduction into chunks of at least
    4 real K-tiles until about 256 items fill the chip; batched products run unsplit."""
    tiles = -(-M // 256) * -(-N // 256) * (1 if reduce_batch else z)
    if not reduce_batch and (z > 1 or tiles >= 256 or not SPLIT9F):
        return 1
    vr = (K // 64) * (z if reduce_batch else 1)
    return max(1, min(-(-256 // tiles), vr // 4))
REDUCE_SPLITS = 16          # splits of a batch-reduced weight gradient on the 256-tile kernel


def try_gemm(A, B, out=None, bias=None, bias_dim=None, act=None, alpha=1.0, beta=0.0, out_dtype=None,
             splits=1, reduce_batch=False, cache_a=False, cache_b=False, auto=False, route=None):
    """C = epi(alpha * A @ B + beta * out). A: [M, K] or [z, M, K]; B: [K, N] or [z, K, N]
    (any strides with one unit-stride dim each). bias: fp32 [N] (bias_dim=1) or [M]
    (bias_dim=0). Returns C ([M, N] / [z, M, N], or [M, N] when reduce_batch sums over z),
    or None when no kernel covers the shapes/strides. `route` forces a plan
    (("g8", kchunk) / ("g128", splits): microbenchmarks). An fp32 product the bf16-piece kernels do not
    take (contiguous extents that are not 16-B multiples: the equivariance decodes' 1 x 1 / 3 x 3 planes)
    runs on the exact-fp32 kernel (`sgemm`) instead of returning None."""
    res = _try_gemm(A, B, out, bias, bias_dim, act, alpha, beta, out_dtype, splits, reduce_batch, cache_a, cache_b,
                    auto, route)
    if (res is None and SGEMM and route is None and A.dtype == torch.float32 and B.dtype == torch.float32
            and A.is_cuda and (out_dtype or A.dtype) == torch.float32):
        res = sgemm(A, B, out=out, bias=bias, bias_dim=bias_dim, act=act, alpha=alpha, beta=beta,
                    reduce_batch=reduce_batch)
    return res


def _try_gemm(A, B, out, bias, bias_dim, act, alpha, beta, out_dtype, splits, reduce_batch, cache_a, cache_b, auto,
              route):
    if A.dtype != B.dtype or A.dtype not in _CODES or not A.is_cuda:
        return None
    a3 = A if A.dim() == 3 else A.unsqueeze(0)
    b3 = B if B.dim() == 3 else B.unsqueeze(0)
    z = max(a3.shape[0], b3.shape[0])
    if a3.shape[0] not in (1, z) or b3.shape[0] not in (1, z):
        return None
    M, K = a3.shape[1], a3.shape[2]
    K2, N = b3.shape[1], b3.shape[2]
    if K != K2:
        raise RuntimeError(f"gemm: inner dims differ ({K} vs {K2})")
    if (FOLD and auto and A.dtype == torch.float32 and not reduce_batch and splits == 1 and a3.shape[0] == 1
            and z > 1 and FOLD_MIN <= N < 128 and (N & (N - 1)) == 0):
        # per-sample planes narrower than a tile (the 8 x 8 decoder block's 1x1 convs): one product over
        # the batch-folded N = z P columns (csrc/gemm.hip vfm_gemm_fold)
        out = _try_fold(a3, b3, M, N, K, z, out, bias, bias_dim, act, alpha, beta, out_dtype)
        if out is not None:
            return out
    if auto and not preferred(A, M, N, reduce_batch):
        if SGEMM and A.dtype == torch.float32 and (out_dtype or A.dtype) == torch.float32:
            return sgemm(a3, b3, out=out, bias=bias, bias_dim=bias_dim, act=act, alpha=alpha, beta=beta,
                         reduce_batch=reduce_batch, batched_out=(A.dim() == 3 or B.dim() == 3))
        return None
    g9f = None                                  # f32x6 on gemm9: K splits of the product (see _splits9f)
    if (auto and route is None and G9_F32 and A.dtype == torch.float32 and beta == 0.0 and act is None
            and (out_dtype or A.dtype) == torch.float32 and K % 64 == 0 and min(M, N) >= 128
            and custom_ops.f32_precision()[0] == custom_ops.VFM_F32):
        g9f = _splits9f(M, N, K, z, reduce_batch) if G9F_PLAN else _deep9f(M, N, K, z, reduce_batch)
        if g9f is not None and bias is not None and (g9f > 1 or reduce_batch or not G9F_BIAS):
            g9f = None
    if auto and splits == 1 and A.dtype != torch.bfloat16:
        # few output tiles over a deep reduction (weight gradients of token-major linears):
        # split K so the grid covers the 256 CUs several times (128-tile kernel)
        tiles = -(-M // 128) * -(-N // 128) * z
        if tiles < 512 and K >= 2048:
            splits = max(1, min(-(-1024 // tiles), K // 512, 64))
        elif z == 1 and tiles < 256 and K >= 1152 and A.dtype == torch.float32:
            # the DINO tower's narrow-output products (6304 x 384 x 1536 / 1152: 150 128-tiles on 256 CUs):
            # three K splits, 79 -> 67 us and 60 -> 56 us (tools_dev/dinobench.py, profiles/r4_ah_dinobench.txt)
            splits = 3
    la = _layout(a3, True)                       # A rows = m, cols = k
    lb = _layout(b3.transpose(1, 2), True)       # B^T rows = n, cols = k
    if la is None or lb is None:
        return None
    a_kc, lda, sA = la
    b_kc, ldb, sB = lb
    if a3.shape[0] == 1:
        sA = 0
    if b3.shape[0] == 1:
        sB = 0
    out_dtype = out_dtype or A.dtype
    zc = 1 if reduce_batch else z
    if out is None:
        if beta != 0.0:
            raise RuntimeError("gemm: beta != 0 needs `out`")
        out = torch.empty((zc, M, N) if (A.dim() == 3 or B.dim() == 3) and not reduce_batch else (M, N),
                          dtype=out_dtype, device=A.device)
    o3 = out if out.dim() == 3 else out.unsqueeze(0)
    if o3.stride(2) != 1 or o3.dtype != out_dtype:
        raise RuntimeError("gemm: output must be row-major in the requested dtype")
    ldc, sC = o3.stride(1), (o3.stride(0) if o3.shape[0] > 1 else 0)
    bias_mode = 0
    if bias is not None:
        bias = bias.detach().float().contiguous()
        bias_mode = 1 if bias_dim in (None, 1) else 2
    flops = 2.0 * z * M * N * K
    nbytes = gemm_bytes(a3, b3, M, N, K, z, out_dtype, reduce_batch)
    stream = custom_ops.stream_ptr(A.device)
    kern, arg = route or (("g8", 0) if g9f is not None else _plan(A.dtype, M, N, K, z, reduce_batch, splits, auto))
    tb = lambda v: "true" if v else "false"
    if kern == "g9r" and A.dtype == torch.bfloat16:
        # batch-reduced / K-split product on gemm9 (fp32 partials of arg chunks + fixed-order combine)
        S = max(1, int(arg))
        n = _lib.vfm_gemm9_workspace_floats(M, N, K, z, S, int(reduce_batch))
        if n > 0 and (reduce_batch or z == 1) and beta == 0.0 and bias is None and act is None:
            ws = _workspace(n, A.device)
            region = f"gemm9<bf16,{tb(a_kc)},{tb(b_kc)},true>"
            if kernel_timer.SHAPES:
                region += f"[{M}x{N}x{K}x{z}s{S}]"
            with kernel_timer.region(region, nbytes, flops, "mfma", first_only=True):
                rc = _lib.vfm_gemm9_ex(a3.data_ptr(), b3.data_ptr(), out.data_ptr(), _CODES[out_dtype], M, N, K, z,
                                       int(a_kc), lda, sA, int(b_kc), ldb, sB, ldc, float(alpha), ws.data_ptr(), S,
                                       int(reduce_batch), stream)
            if rc != custom_ops.VFM_NO_KERNEL:
                custom_ops.check(rc, "vfm_gemm9_ex")
                return out
        kern, arg = "g8", 0
    if kern == "g9" and A.dtype == torch.bfloat16 and not reduce_batch:
        # one wave per SIMD, 128 x 128 per wave, LDS-DMA staging two K-tiles ahead (csrc/gemm9.hip)
        region = f"gemm9<bf16,{tb(a_kc)},{tb(b_kc)},{tb(out_dtype == torch.float32)}>"
        if kernel_timer.SHAPES:
            region += f"[{M}x{N}x{K}x{z}]"
        with kernel_timer.region(region, nbytes, flops, "mfma", first_only=True):
            rc = _lib.vfm_gemm9(a3.data_ptr(), b3.data_ptr(), out.data_ptr(), custom_ops.ptr(bias), _CODES[out_dtype],
                                M, N, K, z, int(a_kc), lda, sA, int(b_kc), ldb, sB, ldc, sC, float(alpha), float(beta),
                                bias_mode, ACTS[act], stream)
        if rc != custom_ops.VFM_NO_KERNEL:
            custom_ops.check(rc, "vfm_gemm9")
            return out
        kern, arg = "g8", 0
    if kern == "g8":
        # 256 tiles + LDS-DMA pipeline (csrc/gemm8.hip); fp32 operands as their bf16 pieces along
        # K, the kernel accumulating the piece products of every K-tile
        psA = psB = 0
        if A.dtype == torch.float32:
            prec, _, tag = custom_ops.f32_precision()
            # planar pieces of the whole tensor where the view covers one (shared with the other
            # products of that tensor), else the per-product stacked split
            pl = _planar(a3, stream)
            if pl is not None:
                Ak, fa_kc, flda, fsA, psA, a_off = pl[0], a_kc, lda, sA, pl[2], pl[1]
            else:
                (Ak, fa_kc, flda, fsA), a_off = _split_f32(a3, M, K, a_kc, lda, sA, cache_a, stream), 0
            pl = _planar(b3, stream)
            if pl is not None:
                Bk, fb_kc, fldb, fsB, psB, b_off = pl[0], b_kc, ldb, sB, pl[2], pl[1]
            else:
                (Bk, fb_kc, fldb, fsB), b_off = _split_f32(b3, N, K, b_kc, ldb, sB, cache_b, stream), 0
        else:
            prec, tag = custom_ops.VFM_BF16, "bf16"
            Ak, fa_kc, flda, fsA, Bk, fb_kc, fldb, fsB = a3, a_kc, lda, sA, b3, b_kc, ldb, sB
            a_off = b_off = 0
        S9 = g9f if g9f is not None else 1
        if (Ak is not None and Bk is not None and A.dtype == torch.float32 and G9_F32 and int(arg) == 0
                and (bias is None or G9F_BIAS)
                and S9 is not None and (g9f is not None or not reduce_batch) and beta == 0.0 and act is None
                and out_dtype == torch.float32 and prec == custom_ops.VFM_F32):
            # f32x6 on the persistent one-wave-per-SIMD kernel: the six piece products of a real K-tile as
            # consecutive virtual K-tiles (csrc/gemm9.hip vfm_gemm9_pieces); K splits / the batch reduction
            # through fp32 partials and the fixed-order combine
            ws9 = None
            if S9 > 1 or reduce_batch:
                n9 = _lib.vfm_gemm9_workspace_floats(M, N, K, z, S9, int(reduce_batch))
                ws9 = _workspace(max(n9, 1), A.device)
            region = f"gemm9<f32x6,{tb(fa_kc)},{tb(fb_kc)},true>"
            if kernel_timer.SHAPES:
                region += f"[{M}x{N}x{K}x{z}{'r' if reduce_batch else ''}{'s%d' % S9 if S9 > 1 else ''}]"
            with kernel_timer.region(region, nbytes, flops, "mfma", first_only=True):
                rc = _lib.vfm_gemm9_pieces(Ak.data_ptr() + 2 * a_off, Bk.data_ptr() + 2 * b_off, out.data_ptr(),
                                           custom_ops.ptr(bias), M, N, K, z, int(fa_kc), flda, fsA, psA, int(fb_kc),
                                           fldb, fsB, psB, ldc, sC, float(alpha), bias_mode, custom_ops.ptr(ws9),
                                           int(S9), int(reduce_batch), stream)
            if rc != custom_ops.VFM_NO_KERNEL:
                custom_ops.check(rc, "vfm_gemm9_pieces")
                if _G9F_CHECK:
                    _check9f(a3, b3, out, bias, bias_dim, alpha, reduce_batch, region, fa_kc, fb_kc, a_off, b_off, psA, psB)
                return out
        if Ak is not None and Bk is not None:
            kchunk = int(arg)
            ws = None
            if kchunk > 0 or reduce_batch:
                n = _lib.vfm_gemm8_workspace_floats(prec, M, N, K, z, kchunk, int(reduce_batch))
                if n < 0:
                    raise custom_ops.NativeError("vfm_gemm8: split-K workspace too large")
                ws = torch.empty(max(n, 1), dtype=torch.float32, device=A.device) if n > 0 else None
            # one timer region per kernel instantiation (rocprof: gemm8_kernel<AK, BK, OUTF32>)
            region = f"gemm8<{tag},{tb(fa_kc)},{tb(fb_kc)},{tb(out_dtype == torch.float32)}>"
            if kernel_timer.SHAPES:
                region += f"[{M}x{N}x{K}x{z}{'r' if reduce_batch else ''}{'k%d' % kchunk if kchunk else ''}]"
            with kernel_timer.region(region, nbytes, flops, "mfma", first_only=True):
                rc = _lib.vfm_gemm8_pieces(Ak.data_ptr() + 2 * a_off, Bk.data_ptr() + 2 * b_off, out.data_ptr(),
                                           custom_ops.ptr(bias), prec, _CODES[out_dtype], M, N, K, z, int(fa_kc), flda,
                                           fsA, psA, int(fb_kc), fldb, fsB, psB, ldc, sC, float(alpha), float(beta),
                                           bias_mode, ACTS[act], custom_ops.ptr(ws), kchunk, int(reduce_batch), stream)
            if rc != custom_ops.VFM_NO_KERNEL:
                custom_ops.check(rc, "vfm_gemm8")
                return out
        splits = 1 if kern == "g8" else splits
    else:
        splits = int(arg)
    ws = None
    if splits > 1 or reduce_batch:
        n = _lib.vfm_gemm_workspace_floats(M, N, z, splits, int(reduce_batch))
        ws = torch.empty(n, dtype=torch.float32, device=A.device)
    if A.dtype == torch.bfloat16:
        in_code, tag = custom_ops.VFM_BF16, "bf16"
    else:
        in_code, _, tag = custom_ops.f32_precision()
    # one region per gemm_kernel<AK, BK, NP, OUTF32> instantiation; split-K / batch-reduced
    # launches (kernel + gemm_reduce_kernel) are their own region
    region = f"gemm<{tag},{tb(a_kc)},{tb(b_kc)},{tb(out_dtype == torch.float32)}>"
    if kernel_timer.SHAPES:
        region += f"[{M}x{N}x{K}x{z}{'r' if reduce_batch else ''}{'s%d' % splits if splits > 1 else ''}]"
    with kernel_timer.region(region, nbytes, flops, "mfma", first_only=True):
        rc = _lib.vfm_gemm(A.data_ptr(), B.data_ptr(), out.data_ptr(), custom_ops.ptr(bias), custom_ops.ptr(ws),
                           in_code, _CODES[out_dtype], M, N, K, z, int(a_kc), lda, sA, int(b_kc), ldb, sB,
                           ldc, sC, float(alpha), float(beta), bias_mode, ACTS[act], int(splits), int(reduce_batch),
                           custom_ops.stream_ptr(A.device))
    if rc == custom_ops.VFM_NO_KERNEL:
        return None
    custom_ops.check(rc, "vfm_gemm")
    return out


FOLD_MIN = 8                # narrowest per-sample plane the batch-folded product takes
# Off by default: on the 8 x 8 block's shapes the folded product leaves 64-256 128-tiles and measured
# 34-40 TF/s in the step against hipBLASLt's exact fp32 bmm at 43-61 (r4g bench: 10.6 vs 6.4 ms/step)
FOLD = __import__("os").environ.get("VFM_GEMM_FOLD", "0") == "1"


def _try_fold(a3, b3, M, N, K, z, out, bias, bias_dim, act, alpha, beta, out_dtype):
    """C[z] = epi(alpha A B[z] + beta C[z]) as one batch-folded product, or None (layout not covered)."""
    if b3.stride(2) != 1 or b3.shape[0] != z:
        return None
    la = _layout(a3, True)
    if la is None:
        return None
    a_kc, lda, _ = la
    out_dtype = out_dtype or a3.dtype
    if out is None:
        if beta != 0.0:
            raise RuntimeError("gemm: beta != 0 needs `out`")
        out = torch.empty((z, M, N), dtype=out_dtype, device=a3.device)
    if out.dim() != 3 or out.stride(2) != 1 or out.dtype != out_dtype:
        return None
    bias_mode = 0
    if bias is not None:
        bias = bias.detach().float().contiguous()
        bias_mode = 1 if bias_dim in (None, 1) else 2
    prec, _, tag = custom_ops.f32_precision()
    lgp = N.bit_length() - 1
    tb = lambda v: "true" if v else "false"
    region = f"gemm_fold<{tag},{tb(a_kc)},{tb(out_dtype == torch.float32)}>"
    if kernel_timer.SHAPES:
        region += f"[{M}x{N}x{K}x{z}]"
    with kernel_timer.region(region, gemm_bytes(a3, b3, M, N, K, z, out_dtype), 2.0 * z * M * N * K, "mfma", first_only=True):
        rc = _lib.vfm_gemm_fold(a3.data_ptr(), b3.data_ptr(), out.data_ptr(), custom_ops.ptr(bias), prec,
                                _CODES[out_dtype], M, lgp, K, z, int(a_kc), lda, b3.stride(1), b3.stride(0),
                                out.stride(1), out.stride(0), float(alpha), float(beta), bias_mode, ACTS[act],
                                custom_ops.stream_ptr(a3.device))
    if rc == custom_ops.VFM_NO_KERNEL:
        return None
    custom_ops.check(rc, "vfm_gemm_fold")
    return out


def gemm_bytes(a3, b3, M, N, K, z, out_dtype, reduce_batch=False):
    """Algorithmic HBM bytes of one product: A, B and C once each at their own element size (a
    batch-shared operand -- leading extent 1 -- counted once)."""
    e = a3.element_size()
    eo = 4 if out_dtype == torch.float32 else 2
    return int((a3.shape[0] * M * K + b3.shape[0] * K * N) * e + (1 if reduce_batch else z) * M * N * eo)


def gemm(A, B, **kw):
    """try_gemm that raises instead of returning None."""
    out = try_gemm(A, B, **kw)
    if out is None:
        raise custom_ops.NativeError(f"vfm_gemm does not cover A {tuple(A.shape)} {A.stride()} / "
                                     f"B {tuple(B.shape)} {B.stride()} {A.dtype}")
    return out


# ---------------------------------------------------------------------------------------------------------------
# Exact-fp32 products on the fp32-input MFMA (csrc/sgemm.hip): the narrow fp32 products (outputs under 128 wide:
# the 4^2 / 8^2 decoder blocks' 1x1s and GigaGAN projections, the adapter's 64-wide linears, the mapping / style
# FC layers) that `preferred` keeps off the bf16-piece kernels, and the D heads' 1-D convolutions
# (patchgan_hip.conv1d_folded). VFM_SGEMM=0: those products go back to the library (torch / hipBLASLt) for A/B.
SGEMM = __import__("os").environ.get("VFM_SGEMM", "1") == "1"
SG_TILES = ((128, 128), (128, 64), (64, 128), (64, 64))      # tile codes 0-3; +4: two wave groups (KW = 2)


# relative time of one 32-deep K-tile per tile shape (64 x 64 = 1; the larger tiles reuse operands better:
# 4096^2 runs 130 TF/s on 128 x 128 against ~100 on 64 x 64), a workgroup's fixed prologue + epilogue in K-tiles,
# one 64 x 64 K-tile in us with two workgroups per CU, and the workgroup slots of the chip (256 CUs x 2)
_SG_KT = (4.0, 2.1, 2.1, 1.0)
_SG_FIXED, _SG_KT_US, _SG_SLOTS = 3.0, 1.14, 512


@__import__('functools').lru_cache(maxsize=4096)
def _sg_plan(M, N, K, zt, vt):
    """(tile code, K splits) of an exact-fp32 product with zt independent output planes and vt virtual K-tiles
    (32 deep) per output: the candidate with the least modelled time -- whole rounds of workgroups over the
    chip's 512 slots (wave quantization: the D heads' 588 64 x 64 tiles are 1.15 rounds unsplit, 3.4 split
    three ways), each round as long as one workgroup's K chunk plus its fixed cost, plus the split's partial-sum
    traffic and reduce launch; 64 x 64 first, a larger tile only when modelled >= 3 % faster (a lone workgroup
    per CU does not get the two-per-CU rate the model assumes, which favours the small tile in practice). The
    model reproduces the sweeps of tools_dev/sgemmbench.py within ~10 % (profiles/r6_sgemmbench.txt: e.g.
    D-head k9 forward 247 us unsplit, 171 us in three). Deep products with >= 1024 128 x 128 tiles take
    128 x 128 unsplit (4096^2: 130 TF/s; at K <= 384 64 x 64 stays faster)."""
    if -(-M // 128) * -(-N // 128) * zt >= 1024 and vt >= 32:
        return 0, 1
    best = None
    for tile in (3, 1, 2, 0):
        kt = _SG_KT[tile]
        bm, bn = SG_TILES[tile]
        tiles = -(-M // bm) * -(-N // bn) * zt
        for s in range(1, max(1, min(16, vt // 4)) + 1):
            rounds = -(-tiles * s // _SG_SLOTS)
            t = rounds * (-(-vt // s) + _SG_FIXED) * kt * _SG_KT_US
            if s > 1:
                t += 4.0 + s * zt * M * N * 8 / 5e6            # partials written + read at ~5 TB/s, the reduce launch
            if best is None or t < best[0] * 0.97:             # prefer the earlier (larger-tile, less-split) plan on ties
                best = (t, tile, s)
    return best[1], best[2]


def _sg_layouts(t3, outer, kdim):
    """Candidate (k_contiguous, leading dim) layouts of a [z, ., .] fp32 view whose dims `outer` / `kdim` are the
    outer (m or n) and reduction indices, K-contiguous first; extents of 1 take any stride."""
    so, sk = t3.stride(outer), t3.stride(kdim)
    no, nk = t3.shape[outer], t3.shape[kdim]
    out = []
    if sk == 1 or nk == 1:
        out.append((True, so if no > 1 else -(-nk // 4) * 4))
    if so == 1 or no == 1:
        out.append((False, sk if nk > 1 else -(-no // 4) * 4))
    return out


def sgemm(a3, b3, out=None, bias=None, bias_dim=None, act=None, alpha=1.0, beta=0.0, reduce_batch=False,
          splits=None, tile=None, batched_out=None):
    """Exact-fp32 C = epi(alpha A @ B + beta C) on csrc/sgemm.hip for fp32 views A [z|1, M, K] / [M, K],
    B [z|1, K, N] / [K, N]; returns C ([z, M, N], or [M, N] for 2-D operands or reduce_batch) or None when the
    layouts are not covered (a contiguous extent or leading dim not a multiple of 4 floats, unaligned base)."""
    if a3.dtype != torch.float32 or b3.dtype != torch.float32 or not a3.is_cuda:
        return None
    if batched_out is None:
        batched_out = a3.dim() == 3 or b3.dim() == 3
    a3 = a3 if a3.dim() == 3 else a3.unsqueeze(0)
    b3 = b3 if b3.dim() == 3 else b3.unsqueeze(0)
    z = max(a3.shape[0], b3.shape[0])
    M, K, N = a3.shape[1], a3.shape[2], b3.shape[2]
    if b3.shape[1] != K:
        raise RuntimeError(f"sgemm: inner dims differ ({K} vs {b3.shape[1]})")
    if min(M, N, K) <= 0:
        return None
    sA = a3.stride(0) if a3.shape[0] > 1 else 0
    sB = b3.stride(0) if b3.shape[0] > 1 else 0
    lk = (a3.shape, a3.stride(), b3.shape, b3.stride())
    lay = _SG_LAYOUT_CACHE.get(lk)
    if lay is None:
        # a layout whose contiguous extent and leading dim are in 16-B units first (the kernel's 16-B loads),
        # else any (bounds-checked scalar loads: the equivariance decodes' 3 x 3 / 6 x 6 planes)
        vec = lambda kc, ld, n_out: ld % 4 == 0 and (K if kc else n_out) % 4 == 0
        la = sorted(_sg_layouts(a3, 1, 2), key=lambda c: not vec(c[0], c[1], M))
        lb = sorted(_sg_layouts(b3, 2, 1), key=lambda c: not vec(c[0], c[1], N))
        lay = (la[0], lb[0]) if la and lb else ()
        if len(_SG_LAYOUT_CACHE) < 4096:
            _SG_LAYOUT_CACHE[lk] = lay
    if not lay:
        return None
    (a_kc, lda), (b_kc, ldb) = lay
    zc = 1 if reduce_batch else z
    if out is None:
        if beta != 0.0:
            raise RuntimeError("sgemm: beta != 0 needs `out`")
        out = torch.empty((zc, M, N) if batched_out and not reduce_batch else (M, N), dtype=torch.float32,
                          device=a3.device)
    o3 = out if out.dim() == 3 else out.unsqueeze(0)
    if o3.dtype != torch.float32 or o3.stride(2) != 1:
        raise RuntimeError("sgemm: output must be row-major fp32")
    ldc, sC = o3.stride(1), (o3.stride(0) if o3.shape[0] > 1 else 0)
    bias_mode = 0
    if bias is not None:
        bias = bias.detach().float().contiguous()
        bias_mode = 1 if bias_dim in (None, 1) else 2
    # batch folding: per-sample planes narrower than a 64-wide tile (the 4 x 4 block's P = 16) as one product
    lgp = 0
    if (not reduce_batch and z > 1 and a3.shape[0] == 1 and b3.shape[0] == z and not b_kc and N < 64
            and N >= 4 and (N & (N - 1)) == 0 and ldb >= N and ldc == N and sC == M * N and splits in (None, 1)):
        lgp = N.bit_length() - 1
    zt = 1 if (reduce_batch or lgp) else z
    Ne = z * N if lgp else N
    vt = (z if reduce_batch else 1) * -(-K // 32)
    ptile, psplit = _sg_plan(M, Ne, K, zt, vt)
    tile = ptile if tile is None else tile
    splits = (1 if lgp else psplit) if splits is None else splits
    bm, bn = SG_TILES[tile & 3]
    ws = None
    if splits > 1 or reduce_batch:
        n = _lib.vfm_sgemm_workspace_floats(M, N, z, splits, int(reduce_batch))
        ws = _workspace(max(n, 1), a3.device)
    region = _sg_region(a_kc, b_kc, bm, bn, 1 + (tile >> 2))
    if kernel_timer.SHAPES:
        region += f"[{M}x{N}x{K}x{z}{'r' if reduce_batch else ''}{'s%d' % splits if splits > 1 else ''}]"
    with kernel_timer.region(region, gemm_bytes(a3, b3, M, N, K, z, torch.float32, reduce_batch),
                             2.0 * z * M * N * K, "mfma", first_only=True):
        rc = _lib.vfm_sgemm(a3.data_ptr(), b3.data_ptr(), out.data_ptr(), custom_ops.ptr(bias), M, Ne, K, z,
                            int(a_kc), lda, sA, int(b_kc), ldb, sB, ldc, sC, float(alpha), float(beta), bias_mode,
                            ACTS[act], lgp, custom_ops.ptr(ws), int(splits), int(reduce_batch), int(tile),
                            custom_ops.stream_ptr(a3.device))
    if rc == custom_ops.VFM_NO_KERNEL:
        return None
    custom_ops.check(rc, "vfm_sgemm")
    if _SG_CHECK:
        _check_sg(a3, b3, out, bias, bias_dim, act, alpha, beta, reduce_batch,
                  dict(tile=tile, splits=splits, lgp=lgp, a_kc=a_kc, lda=lda, sA=sA, b_kc=b_kc, ldb=ldb, sB=sB, ldc=ldc,
                       sC=sC))
    return out


_SG_CHECK = __import__("os").environ.get("VFM_SGEMM_CHECK") == "1"
_SG_LAYOUT_CACHE = {}       # (shapes, strides) -> chosen (k-contiguous, leading dim) of A and B


@__import__('functools').lru_cache(maxsize=64)
def _sg_region(a_kc, b_kc, bm, bn, kw):
    tb = lambda v: "true" if v else "false"
    return f"sgemm<{tb(a_kc)},{tb(b_kc)},{bm},{bn},{kw}>"


def _check_sg(a3, b3, out, bias, bias_dim, act, alpha, beta, reduce_batch, info):
    """Debug (VFM_SGEMM_CHECK=1, beta == 0 products): an sgemm product against fp64 torch; prints the ones off by
    more than 1e-5 of |A||B|."""
    if beta != 0.0 or act is not None:
        return
    A64, B64 = a3.double(), b3.double()
    ref, bnd = alpha * torch.matmul(A64, B64), abs(alpha) * torch.matmul(A64.abs(), B64.abs())
    if reduce_batch:
        ref, bnd = ref.sum(0), bnd.sum(0)
    if bias is not None:
        bb = bias.double()[:, None] if bias_dim == 0 else bias.double()
        ref, bnd = ref + bb, bnd + bb.abs()
    o = out.double().reshape(ref.shape) if out.numel() == ref.numel() else None
    if o is None:
        print(f"[sgemm check] shape mismatch out {tuple(out.shape)} ref {tuple(ref.shape)} {info}", flush=True)
        return
    e = float(((o - ref).abs() / (bnd + 1e-30)).max())
    if e > 1e-5:
        print(f"[sgemm check] err {e:.2e} A{tuple(a3.shape)}{a3.stride()} B{tuple(b3.shape)}{b3.stride()} "
              f"out{tuple(out.shape)}{out.stride()} bias_dim={bias_dim} red={reduce_batch} {info}", flush=True)
