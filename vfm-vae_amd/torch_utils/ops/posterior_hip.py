"""Reparameterised sample + KL of the latent posterior in one HIP pass (csrc/posterior.hip;
reference networks/utils/kl_utils.py:30-56). Reached through kl_utils.sample_and_kl for fp32
ROCm moments; the noise is drawn by the caller exactly as DiagonalGaussianDistribution.sample()
draws it, so seeded runs see the same epsilon."""
import torch

from .. import custom_ops
from . import kernel_timer

_lib = custom_ops.get_native()


class _Posterior(custom_ops.FastFunction):
    @staticmethod
    def forward(ctx, params, eps):
        params = params.contiguous()
        B, C2 = params.shape[:2]
        C = C2 // 2
        P = params[0, 0].numel()
        eps = eps.contiguous()
        z = torch.empty((B, C) + tuple(params.shape[2:]), dtype=torch.float32, device=params.device)
        kl = torch.empty([B], dtype=torch.float32, device=params.device)
        with kernel_timer.region("posterior_fwd<f32>", 4 * (params.numel() + 2 * z.numel() + B)):
            custom_ops.check(_lib.vfm_posterior_fwd(params.data_ptr(), eps.data_ptr(), z.data_ptr(), kl.data_ptr(), B, C,
                                                    P, custom_ops.stream_ptr()), "vfm_posterior_fwd")
        ctx.save_for_backward(params, eps)
        return z, kl

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dz, dkl):
        params, eps = ctx.saved_tensors
        B, C2 = params.shape[:2]
        P = params[0, 0].numel()
        dz = None if dz is None else dz.float().contiguous()
        dkl = None if dkl is None else dkl.float().contiguous()
        dp = torch.empty_like(params)
        with kernel_timer.region("posterior_bwd<f32>", 4 * (3 * params.numel())):
            custom_ops.check(_lib.vfm_posterior_bwd(params.data_ptr(), eps.data_ptr(), custom_ops.ptr(dz),
                                                    custom_ops.ptr(dkl), dp.data_ptr(), B, C2 // 2, P,
                                                    custom_ops.stream_ptr()), "vfm_posterior_bwd")
        return dp, None


def sample_kl(params, eps):
    """(mean + exp(clamp(logvar)/2) * eps, 0.5 * sum(mean^2 + var - 1 - logvar) per sample)."""
    return _Posterior.apply(params, eps)
