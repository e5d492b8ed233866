"""LPIPS distance head: per VGG tap, channel-unit-normalise both feature maps, squared
difference, 1×1 `lin` (C→1, no bias), spatial mean.

Reference: `training/lpips.py` `LPIPS.forward` (`normalize_tensor`, `** 2`, `lin{kk}.model`,
`spatial_average`). On ROCm tensors the HIP kernels `vfm_lpips_head_fwd/_bwd` (csrc/lpips.hip)
do the normalise→diff→square→lin chain in one pass over the two feature maps (and one
backward), instead of ~8 full-size fp32 torch passes; a missing kernel library raises. CPU
tensors, non-fp32 features or `impl='ref'` run the torch formulation.
"""
import torch

from .. import custom_ops
from . import kernel_timer


def _normalize_tensor(x, eps=1e-10):
    return x / (torch.sqrt(torch.sum(x ** 2, dim=1, keepdim=True)) + eps)


def head_ref(f0, f1, w):
    """Torch formulation (the reference's expression). w: [C] lin weight. Returns [B,1,1,1]."""
    d = (_normalize_tensor(f0) - _normalize_tensor(f1)) ** 2
    r = torch.nn.functional.conv2d(d, w.reshape(1, -1, 1, 1))
    return r.mean([2, 3], keepdim=True)


class _LpipsHead(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, f0, f1, w):
        from .. import custom_ops
        lib = custom_ops.get_native()
        if f0.ndim != 4 or f0.shape != f1.shape or f0.device != f1.device:
            raise RuntimeError(f"lpips head: feature shapes {tuple(f0.shape)} vs {tuple(f1.shape)}")
        B, C, H, W = f0.shape
        HW = H * W
        # channels_last features (the HIP VGG16 stack) run the NHWC kernels in place
        nhwc = C in (64, 128, 256, 512) and all(_is_nhwc(t) for t in (f0, f1))
        if nhwc:
            f0c, f1c = f0, f1
        else:
            f0c, f1c = f0.contiguous(), f1.contiguous()
        wc = w.detach().reshape(-1).float().contiguous()
        if wc.numel() != C or wc.device != f0.device:
            raise RuntimeError(f"lpips head: lin weight has {wc.numel()} entries for {C} channels")
        r = torch.empty(B, HW, dtype=torch.float32, device=f0.device)
        n0 = torch.empty_like(r)
        n1 = torch.empty_like(r)
        nb = 2 * 2 * B * C * HW * 4 + 3 * B * HW * 4
        fn = lib.vfm_lpips_head_fwd_nhwc if nhwc else lib.vfm_lpips_head_fwd
        with kernel_timer.region('lpips_head_fwd_nhwc' if nhwc else 'lpips_head_fwd', nb):
            rc = fn(f0c.data_ptr(), f1c.data_ptr(), wc.data_ptr(), r.data_ptr(), n0.data_ptr(), n1.data_ptr(), B, C, HW,
                    custom_ops.stream_ptr(f0.device))
        custom_ops.check(rc, "vfm_lpips_head_fwd")
        ctx.save_for_backward(f0c, f1c, wc, n0, n1)
        ctx.shape = (B, C, H, W)
        ctx.nhwc = nhwc
        return r.mean(1).reshape(B, 1, 1, 1)

    @staticmethod
    def backward(ctx, gout):
        from .. import custom_ops
        lib = custom_ops.get_native()
        f0, f1, w, n0, n1 = ctx.saved_tensors
        B, C, H, W = ctx.shape
        HW = H * W
        need0, need1 = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        if ctx.needs_input_grad[2]:
            raise RuntimeError("lpips head: the lin weights are frozen (LPIPS is requires_grad_(False))")
        if not (need0 or need1):
            return None, None, None
        gs = (gout.reshape(B).float() / HW).contiguous()
        g0 = torch.empty_like(f0) if need0 else None          # same memory format as the features
        g1 = torch.empty_like(f1) if need1 else None
        nb = 2 * 2 * B * C * HW * 4 + (int(need0) + int(need1)) * B * C * HW * 4 + 2 * B * HW * 4
        fn = lib.vfm_lpips_head_bwd_nhwc if ctx.nhwc else lib.vfm_lpips_head_bwd
        with kernel_timer.region('lpips_head_bwd_nhwc' if ctx.nhwc else 'lpips_head_bwd', nb):
            rc = fn(f0.data_ptr(), f1.data_ptr(), w.data_ptr(), n0.data_ptr(), n1.data_ptr(), gs.data_ptr(),
                    g0.data_ptr() if need0 else None, g1.data_ptr() if need1 else None, B, C, HW,
                    custom_ops.stream_ptr(f0.device))
        custom_ops.check(rc, "vfm_lpips_head_bwd")
        return g0, g1, None


def _is_nhwc(t):
    return t.dim() == 4 and t.permute(0, 2, 3, 1).is_contiguous() and t.data_ptr() % 16 == 0


def lpips_head(f0, f1, w, impl='cuda'):
    """f0, f1: [B, C, H, W] features of the two images; w: lin weight ([1, C, 1, 1] or [C]).
    Returns the tap's contribution [B, 1, 1, 1]."""
    if (impl == 'cuda' and f0.is_cuda and f0.dtype == torch.float32 and f1.dtype == torch.float32
            and not w.requires_grad):
        return _LpipsHead.apply(f0, f1, w.reshape(-1))
    return head_ref(f0, f1, w.reshape(-1))
