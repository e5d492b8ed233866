"""LPIPS VGG16 feature stack on the HIP implicit-GEMM convolution (csrc/conv.hip).

Replaces the torchvision `vgg16().features[:30]` forward/backward of the reference's LPIPS
(training/lpips.py:126-163; MIOpen fp32 Winograd on ROCm) with 13 fused conv3x3 + bias + ReLU
launches on NHWC fp32 activations (fp32-equivalent products through the f32x6 bf16 split, the
f32x3 split opt-in: custom_ops.F32_PRODUCTS), torch max-pool on the channels_last views, and a backward that
runs the data gradients on the same kernel with flipped/transposed weights, the ReLU derivative
of the layer below fused into the epilogue where no pool sits in between. VGG is frozen: no
weight gradients.

`vgg16_taps(x, convs)` returns the five LPIPS taps (relu1_2, relu2_2, relu3_3, relu4_3,
relu5_3) as NCHW-shaped views of NHWC tensors.
"""
import torch
import torch.nn.functional as F

from .. import custom_ops
from . import kernel_timer

_lib = custom_ops.get_native()

# torchvision vgg16 cfg D up to relu5_3: conv channels, 'M' pool; taps after these conv indices
_CFG = [64, 64, 'M', 128, 128, 'M', 256, 256, 256, 'M', 512, 512, 512, 'M', 512, 512, 512]
_TAPS = (1, 3, 6, 9, 12)          # conv ordinal (0-based) whose ReLU output is a tap


def _plan():
    ops, ci = [], 0
    for v in _CFG:
        if v == 'M':
            ops.append(('pool',))
        else:
            ops.append(('conv', ci))
            if ci in _TAPS:
                ops.append(('tap', _TAPS.index(ci)))
            ci += 1
    return ops


PLAN = _plan()


def split_weight(w2d, npieces=None):
    """fp32 [Cout, K] tap-major weights -> bf16 pieces [np, Cout, Kp] (Kp = K rounded up to 64, zero
    padded): np = 3: hi = bf16(w), mid = bf16(w - hi), lo = bf16(w - hi - mid) (w = hi + mid + lo
    exactly); np = 2: hi, lo -- round-to-nearest, as the kernels' own split."""
    npieces = npieces or custom_ops.f32_precision()[1]
    Cout, K = w2d.shape
    Kp = -(-K // 64) * 64
    r = torch.zeros(Cout, Kp, dtype=torch.float32, device=w2d.device)
    r[:, :K] = w2d
    out = torch.empty(npieces, Cout, Kp, dtype=torch.bfloat16, device=w2d.device)
    for p in range(npieces):
        out[p] = r.to(torch.bfloat16)
        r = r - out[p].float()
    return out


def chunk_major(w2d, cin):
    """[Cout, 9 cin] tap-major (k = tap cin + c) -> the kernel's order for cin >= 32: channel-chunk-major,
    tap-minor (k = (c // 32) 288 + tap 32 + c % 32; csrc/conv.hip StageA::load_wide). cin < 32 stays."""
    if cin < 32:
        return w2d
    Cout = w2d.shape[0]
    return w2d.reshape(Cout, 9, cin // 32, 32).permute(0, 2, 1, 3).reshape(Cout, 9 * cin)


def tap_major(w2d, cin):
    """Inverse of chunk_major."""
    if cin < 32:
        return w2d
    Cout = w2d.shape[0]
    return w2d.reshape(Cout, cin // 32, 9, 32).permute(0, 2, 1, 3).reshape(Cout, 9 * cin)


def conv3x3(x, w, bias=None, relu=False, mask=None):
    """x: NHWC fp32 [B, H, W, Cin] contiguous; w: [np, Cout, Kp] pieces from split_weight of the
    [Cout, 9*Cin] weights in the kernel's k order (chunk_major) -> [B, H, W, Cout] = relu?(conv(x) + bias) (x (mask > 0) when
    given)."""
    B, H, W, Cin = x.shape
    npc, Cout, Kp = w.shape
    prec, np_mode, tag = custom_ops.f32_precision()
    if npc != np_mode:
        raise RuntimeError(f"conv3x3: weights split into {npc} pieces, the {tag} mode needs {np_mode}")
    if not x.is_contiguous() or Kp < 9 * Cin or (mask is not None and mask.shape != (B, H, W, Cout)):
        raise RuntimeError("conv3x3: NHWC contiguous input, split [np, Cout, >= 9*Cin] weights, mask of the output shape")
    out = torch.empty(B, H, W, Cout, dtype=torch.float32, device=x.device)
    flops = 2 * B * H * W * Cout * 9 * Cin
    # one timer region per kernel instantiation (BN = 128 / 64 output channels per tile), as
    # rocprofv3 names them: conv3x3_kernel<BM, 128, NP> / <128, 64, NP> (kernel_timer.rocprof_name)
    with kernel_timer.region(f"conv3x3_nhwc<{tag},{128 if Cout % 128 == 0 else 64}>",
                             4 * (x.numel() + out.numel() + Cout * 9 * Cin), flops, "mfma"):
        rc = _lib.vfm_conv3x3_nhwc_f32(x.data_ptr(), w.data_ptr(), prec, Kp, custom_ops.ptr(bias),
                                       custom_ops.ptr(mask), out.data_ptr(), B, H, W, Cin, Cout, int(relu),
                                       custom_ops.stream_ptr(x.device))
    custom_ops.check(rc, "vfm_conv3x3_nhwc_f32")
    return out


def prepare(convs):
    """Per nn.Conv2d: forward weights [Cout, 9*Cin'] (Cin' = Cin padded to 4 for the image layer),
    data-gradient weights [Cin, 9*Cout] (flipped taps) -- both as split_weight pieces --, bias and
    the fp32 weight; cached on the module until the weight's version (or the product mode) moves."""
    out = []
    for m in convs:
        key = (m.weight.data_ptr(), m.weight._version, m.bias.data_ptr(), m.bias._version, custom_ops.F32_PRODUCTS)
        hit = getattr(m, "_vfm_vgg_prep", None)
        if hit is None or hit[0] != key:
            w = m.weight.detach().float()
            Cout, Cin = w.shape[:2]
            cp = max(Cin, 4)
            wf = torch.zeros(Cout, 3, 3, cp, dtype=torch.float32, device=w.device)
            wf[..., :Cin] = w.permute(0, 2, 3, 1)
            wb = w.flip(2, 3).permute(1, 2, 3, 0).reshape(Cin, 9 * Cout)
            hit = (key, (split_weight(chunk_major(wf.reshape(Cout, 9 * cp), cp).contiguous()),
                         split_weight(chunk_major(wb, Cout).contiguous()), m.bias.detach().float().contiguous(), w))
            m._vfm_vgg_prep = hit
        out.append(hit[1])
    return out


def _nchw(t):
    return t.permute(0, 3, 1, 2)


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def forward_chain(x, prep):
    """(taps, ReLU outputs, pool indices) of the stack on x (NCHW fp32, or a tuple of same-shape NCHW
    batches stacked along the batch on the way into the first layer): taps / outputs NHWC."""
    xs = x if isinstance(x, (tuple, list)) else (x,)
    B1, C, H, W = xs[0].shape
    B = B1 * len(xs)
    h = torch.zeros(B, H, W, 4, dtype=torch.float32, device=xs[0].device)
    for i, xi in enumerate(xs):
        h[i * B1:(i + 1) * B1, :, :, :C] = xi.permute(0, 2, 3, 1)
    ys, pools, taps = [], [], []
    for op in PLAN:
        if op[0] == 'conv':
            wf, _, b, _ = prep[op[1]]
            h = conv3x3(h, wf, b, relu=True)
            ys.append(h)
        elif op[0] == 'tap':
            taps.append(h)
        else:
            p = maxpool2x2(h)
            if p is not None:
                pools.append(None)        # the backward recomputes the argmax from the pool input
                h = p
            else:
                p, idx = F.max_pool2d(_nchw(h), 2, 2, return_indices=True)
                pools.append(idx)
                h = _nhwc(p)
    return taps, ys, pools


def maxpool2x2(h):
    """NHWC fp32 2x2 / stride-2 max pool on csrc/pool.hip (no indices), or None when the kernel does
    not take the shape (odd sizes, C % 4)."""
    B, H, W, C = h.shape
    if not (h.is_contiguous() and h.dtype == torch.float32 and C % 4 == 0 and H % 2 == 0 and W % 2 == 0):
        return None
    out = torch.empty(B, H // 2, W // 2, C, dtype=torch.float32, device=h.device)
    with kernel_timer.region("maxpool2x2_fwd<f32>", 4 * (h.numel() + out.numel())):
        rc = _lib.vfm_maxpool2x2_nhwc_f32(h.data_ptr(), out.data_ptr(), B, H, W, C, custom_ops.stream_ptr(h.device))
    if rc == custom_ops.VFM_NO_KERNEL:
        return None
    custom_ops.check(rc, "vfm_maxpool2x2_nhwc_f32")
    return out


def maxpool2x2_bwd(g, x, gt):
    """(max-pool backward of g [B, H/2, W/2, C] + gt [B, H, W, C] or None) * (x > 0), NHWC fp32, with
    the argmax recomputed from the pool input x (csrc/pool.hip; bit-identical to the torch chain)."""
    g = g.contiguous()
    B, H, W, C = x.shape
    out = torch.empty_like(x)
    nb = 4 * (2 * x.numel() + g.numel() + (x.numel() if gt is not None else 0))
    with kernel_timer.region("maxpool2x2_bwd<f32>", nb):
        rc = _lib.vfm_maxpool2x2_bwd_nhwc_f32(g.data_ptr(), x.data_ptr(), None if gt is None else gt.data_ptr(),
                                              out.data_ptr(), B, H, W, C, custom_ops.stream_ptr(x.device))
    custom_ops.check(rc, "vfm_maxpool2x2_bwd_nhwc_f32")
    return out


class _VGG16Taps(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, x, prep):
        taps, ys, pools = forward_chain(x, prep)
        ctx.prep = prep
        ctx.in_shape = x.shape
        if ctx.needs_input_grad[0]:
            ctx.save_for_backward(*ys, *pools)
        return tuple(_nchw(t) for t in taps)

    @staticmethod
    def backward(ctx, *gtaps):
        saved = ctx.saved_tensors
        return backward_chain(saved[:13], saved[13:], ctx.prep, ctx.in_shape, gtaps), None


class _VGG16TapsPair(custom_ops.FastFunction):
    """The stack over two same-shape batches (LPIPS's input and target) in ONE pass of 2B images: every
    layer is per-sample, so the taps are bit-identical to two separate passes, and the deep layers
    (16 x 16 / 32 x 32 planes) get twice the tiles. The backward runs only for the batch whose input
    needs a gradient (the generated image; the target is a data batch)."""

    @staticmethod
    def forward(ctx, x0, x1, prep):
        taps, ys, pools = forward_chain((x0, x1), prep)
        B = x0.shape[0]
        ctx.prep, ctx.in_shape, ctx.B = prep, x0.shape, B
        need = ctx.needs_input_grad[:2]
        if any(need):
            ctx.save_for_backward(*ys, *[p for p in pools if p is not None])
            ctx.pool_none = [p is None for p in pools]
        outs = [_nchw(t) for t in taps]
        return tuple(t[:B] for t in outs) + tuple(t[B:] for t in outs)

    @staticmethod
    def backward(ctx, *g):
        saved = ctx.saved_tensors
        ys = saved[:13]
        it = iter(saved[13:])
        pools = [None if none else next(it) for none in ctx.pool_none]
        B = ctx.B
        grads = []
        for half, need in enumerate(ctx.needs_input_grad[:2]):
            gt = g[5 * half:5 * half + 5]
            if not need or all(t is None for t in gt):
                grads.append(None)
                continue
            sl = slice(half * B, (half + 1) * B)
            grads.append(backward_chain([y[sl] for y in ys], [None if p is None else p[sl] for p in pools],
                                        ctx.prep, ctx.in_shape, gt))
        return grads[0], grads[1], None


def vgg16_taps_pair(x0, x1, convs):
    """(taps of x0, taps of x1) from one pass over both batches (see _VGG16TapsPair)."""
    outs = _VGG16TapsPair.apply(x0, x1, prepare(convs))
    return outs[:5], outs[5:]


def backward_chain(ys, pools, prep, in_shape, gtaps, conv=None):
    """Input gradient of the tap stack from the saved ReLU outputs `ys`, pool indices and tap
    gradients. `conv` (default conv3x3) runs every data-gradient conv; tests pass an fp64 torch
    conv to check the kernels against the same ReLU / pool decisions."""
    conv = conv or conv3x3
    g = None           # gradient wrt the current NHWC activation (walking the plan backwards)
    masked = False     # g already carries the ReLU derivative of the conv that produced it
    pi = len(pools)
    skip_tap = False   # the tap below a pool was added by the fused pool backward
    for at in range(len(PLAN) - 1, -1, -1):
        op = PLAN[at]
        if op[0] == 'tap':
            if skip_tap:
                skip_tap = False
                continue
            gt = gtaps[op[1]]
            if gt is not None:
                gt = _nhwc(gt)
                g = gt if g is None else g + gt
                masked = False
        elif op[0] == 'pool':
            pi -= 1
            if (pools[pi] is None and g is not None and g.dtype == torch.float32 and PLAN[at - 1][0] == 'tap'
                    and PLAN[at - 2][0] == 'conv'):
                # pool backward + the tap gradient + the ReLU derivative of the conv below, one pass
                gt = gtaps[PLAN[at - 1][1]]
                g = maxpool2x2_bwd(g, _pool_input(ys, pi), None if gt is None else _nhwc(gt))
                skip_tap, masked = True, True
                continue
            if g is None:
                continue
            idx = pools[pi]
            if idx is None:    # (a plan without the tap below) the indices from the pool input
                _, idx = F.max_pool2d(_nchw(_pool_input(ys, pi)), 2, 2, return_indices=True)
            g = _nhwc(torch.ops.aten.max_pool2d_with_indices_backward(
                _nchw(g), _nchw(_pool_input(ys, pi)), [2, 2], [2, 2], [0, 0], [1, 1], False, idx))
            masked = False
        elif g is not None:
            ci = op[1]
            if not masked:
                g = g * (ys[ci] > 0)
            _, wb, _, w = prep[ci]
            if ci == 0:
                if conv is conv3x3 and g.dtype == torch.float32:
                    return image_grad(g, w, in_shape)
                return torch.nn.grad.conv2d_input(in_shape, w.to(g.dtype), _nchw(g), padding=1)
            # the op before is conv ci-1 (taps are always followed by a pool): fuse its ReLU derivative
            fuse = PLAN[at - 1][0] == 'conv'
            g = conv(g, wb, None, relu=False, mask=ys[ci - 1] if fuse else None)
            masked = fuse
    return None


def image_grad(g, w, in_shape):
    """Input gradient of the image layer (3 -> 64 channels): g NHWC fp32 [B, H, W, 64], w the fp32
    torch weight [64, 3, 3, 3] -> NCHW [B, 3, H, W] on the VALU kernel vfm_conv3x3_dgrad_small_f32
    (exact fp32 FMAs; replaces MIOpen's fp32 Winograd of torch.nn.grad.conv2d_input)."""
    B, C, H, W = in_shape
    g = g.contiguous()
    K = g.shape[-1]
    out = torch.empty(B, C, H, W, dtype=torch.float32, device=g.device)
    with kernel_timer.region("conv3x3_dgrad_small<f32>", 4 * (g.numel() + out.numel()), 2 * B * H * W * C * 9 * K,
                             "hbm"):
        rc = _lib.vfm_conv3x3_dgrad_small_f32(g.data_ptr(), w.detach().float().contiguous().data_ptr(),
                                              out.data_ptr(), B, H, W, C, K, custom_ops.stream_ptr(g.device))
    custom_ops.check(rc, "vfm_conv3x3_dgrad_small_f32")
    return out


def _pool_input(ys, pool_index):
    """NHWC input of the pool_index-th pool: the output of the conv right before it."""
    convs_before = [1, 3, 6, 9][pool_index]
    return ys[convs_before]


def vgg16_taps(x, convs):
    """x: fp32 NCHW (LPIPS-scaled) on ROCm; convs: the 13 nn.Conv2d of vgg16 features in order."""
    return _VGG16Taps.apply(x, prepare(convs))
