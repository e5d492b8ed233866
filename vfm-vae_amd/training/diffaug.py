"""Differentiable augmentation (DiffAugment: color, translation, cutout, resize).

Same policies, parameter ranges and device-RNG draw order as the reference
`training/diffaug.py` (after Zhao et al. 2020), so seeded runs draw identical
augmentations.
"""
import numpy as np
import torch
import torch.nn.functional as F


def DiffAugment(x, policy='', channels_first=True):
    if not policy:
        return x
    if not channels_first:
        x = x.permute(0, 3, 1, 2)
    for p in policy.split(','):
        for fn in AUGMENT_FNS[p]:
            x = fn(x)
    if not channels_first:
        x = x.permute(0, 2, 3, 1)
    return x.contiguous()


def _u(x):
    return torch.rand(x.size(0), 1, 1, 1, dtype=x.dtype, device=x.device)


def rand_brightness(x):
    return x + (_u(x) - 0.5)


def rand_saturation(x):
    m = x.mean(dim=1, keepdim=True)
    return (x - m) * (_u(x) * 2) + m


def rand_contrast(x):
    m = x.mean(dim=[1, 2, 3], keepdim=True)
    return (x - m) * (_u(x) + 0.5) + m


class _Shift2d(torch.autograd.Function):
    """Per-sample integer shift with zero fill on the HIP kernel (csrc/diffaug.hip vfm_shift2d): the
    reference's padded gather, whose backward is the shift by -t (a bijection between in-range pixels)."""

    @staticmethod
    def forward(ctx, x, tx, ty):
        from torch_utils import custom_ops
        x = x.contiguous()
        y = torch.empty_like(x)
        B, C, H, W = x.shape
        lib = custom_ops.get_native()
        custom_ops.check(lib.vfm_shift2d(x.data_ptr(), y.data_ptr(), tx.data_ptr(), ty.data_ptr(),
                                         custom_ops.dtype_code(x), B, C, H, W, 1, custom_ops.stream_ptr(x.device)),
                         "vfm_shift2d")
        ctx.save_for_backward(tx, ty)
        return y

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dy):
        from torch_utils import custom_ops
        tx, ty = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        B, C, H, W = dy.shape
        lib = custom_ops.get_native()
        custom_ops.check(lib.vfm_shift2d(dy.data_ptr(), dx.data_ptr(), tx.data_ptr(), ty.data_ptr(),
                                         custom_ops.dtype_code(dy), B, C, H, W, -1, custom_ops.stream_ptr(dy.device)),
                         "vfm_shift2d")
        return dx, None, None


def rand_translation(x, ratio=0.125):
    B, C, H, W = x.shape
    sx, sy = int(H * ratio + 0.5), int(W * ratio + 0.5)
    tx = torch.randint(-sx, sx + 1, size=[B, 1, 1], device=x.device)
    ty = torch.randint(-sy, sy + 1, size=[B, 1, 1], device=x.device)
    if x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and C * H <= 65535 and B <= 65535:
        return _Shift2d.apply(x, tx.reshape(B).contiguous(), ty.reshape(B).contiguous())
    return translate_gather(x, tx, ty)


def translate_gather(x, tx, ty):
    """The reference formulation: one-pixel zero pad, gather at the clamped shifted grid."""
    B, C, H, W = x.shape
    gb, gx, gy = torch.meshgrid(torch.arange(B, device=x.device), torch.arange(H, device=x.device),
                                torch.arange(W, device=x.device), indexing='ij')
    gx = torch.clamp(gx + tx + 1, 0, H + 1)
    gy = torch.clamp(gy + ty + 1, 0, W + 1)
    xp = F.pad(x, [1, 1, 1, 1, 0, 0, 0, 0])
    return xp.permute(0, 2, 3, 1).contiguous()[gb, gx, gy].permute(0, 3, 1, 2)


def rand_cutout(x, ratio=0.2):
    B, C, H, W = x.shape
    ch, cw = int(H * ratio + 0.5), int(W * ratio + 0.5)
    ox = torch.randint(0, H + (1 - ch % 2), size=[B, 1, 1], device=x.device)
    oy = torch.randint(0, W + (1 - cw % 2), size=[B, 1, 1], device=x.device)
    # the reference scatters zeros at the clamped grid clamp(offset - c // 2 + [0, c), 0, H - 1): a contiguous row
    # (column) range, the window's rows (columns) clamped to the plane. Built by comparisons instead: the scatter
    # (index_put_ with device indices) synchronised the host with the GPU on every call (tools_dev/sync_probe.py)
    r0 = torch.clamp(ox - ch // 2, min=0, max=H - 1)
    r1 = torch.clamp(ox - ch // 2 + ch - 1, min=0, max=H - 1)
    c0 = torch.clamp(oy - cw // 2, min=0, max=W - 1)
    c1 = torch.clamp(oy - cw // 2 + cw - 1, min=0, max=W - 1)
    rows = torch.arange(H, device=x.device).view(1, H, 1)
    cols = torch.arange(W, device=x.device).view(1, 1, W)
    hole = (rows >= r0) & (rows <= r1) & (cols >= c0) & (cols <= c1)        # [B, H, W]
    mask = (~hole).to(x.dtype)
    return x * mask.unsqueeze(1)


def rand_resize(x, min_ratio=0.8, max_ratio=1.2):
    r = np.random.rand() * (max_ratio - min_ratio) + min_ratio
    size = x.shape[3]
    new = int(r * size)
    y = F.interpolate(x, size=new, mode='bilinear')
    if new < size:
        left = int((size - new) / 2.)
        right = size - left - y.shape[3]
        return F.pad(y, (left, right, left, right), "constant", 0.)
    left = int((new - size) / 2.)
    return y[:, :, left:left + size, left:left + size]


AUGMENT_FNS = {
    'color': [rand_brightness, rand_saturation, rand_contrast],
    'translation': [rand_translation],
    'resize': [rand_resize],
    'cutout': [rand_cutout],
}
