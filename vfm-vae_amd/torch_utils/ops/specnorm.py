"""Spectral-norm forward pre-hook for ROCm weights (reference networks/discriminator.py SpectralConv1d:
`SpectralNorm.apply(self, name='weight', n_power_iterations=1, dim=0, eps=1e-12)`). The kernel
library is imported only when the ROCm path runs."""
import torch


class FusedSpectralNormHook:
    """Forward pre-hook standing in for torch's SpectralNorm hook (same parameter / buffer names and
    state-dict keys: weight_orig, weight_u, weight_v): in training mode on a ROCm fp32 weight the
    power iteration, sigma and W / sigma run on csrc/specnorm.hip; otherwise torch's own hook runs."""

    def __init__(self, torch_hook):
        self.fn = torch_hook
        self.name = torch_hook.name

    def __call__(self, module, inputs):
        w = getattr(module, self.name + "_orig")
        if (module.training and w.is_cuda and w.dtype == torch.float32 and w.is_contiguous()
                and self.fn.n_power_iterations == 1 and self.fn.dim == 0):
            from . import specnorm_group
            r = specnorm_group.lookup(module, self.fn)      # the heads' grouped launch (specnorm_group.py)
            if r is None:
                from . import patchgan_hip
                u = getattr(module, self.name + "_u")
                v = getattr(module, self.name + "_v")
                r = patchgan_hip.spectral_norm_weight(w, u, v, self.fn.eps)
            setattr(module, self.name, r)
            return None
        return self.fn(module, inputs)


def install_fused_spectral_norm(module, name="weight"):
    """Replace the SpectralNorm forward pre-hook torch registered on `module` by FusedSpectralNormHook."""
    from torch.nn.utils.spectral_norm import SpectralNorm
    for k, hook in list(module._forward_pre_hooks.items()):
        if isinstance(hook, SpectralNorm) and hook.name == name:
            module._forward_pre_hooks[k] = FusedSpectralNormHook(hook)
            return True
    return False
