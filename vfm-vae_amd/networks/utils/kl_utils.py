"""Diagonal Gaussian posterior of the continuous latent
(reference `networks/utils/kl_utils.py:30-68`, after latent-diffusion).

`sample()` draws its noise on the CPU and copies it to the device, as the
reference does (kl_utils.py:41-43), so seeded runs reproduce the reference's
latents bit-for-bit in the noise. `set_noise_source()` lets parity harnesses
inject the exact epsilon instead.
"""
import numpy as np
import torch

_noise_source = None  # callable(shape) -> tensor, for parity tests


def set_noise_source(fn):
    global _noise_source
    _noise_source = fn


class AbstractDistribution:
    def sample(self):
        raise NotImplementedError()

    def mode(self):
        raise NotImplementedError()


class DiracDistribution(AbstractDistribution):
    def __init__(self, value):
        self.value = value

    def sample(self):
        return self.value

    def mode(self):
        return self.value


class DiagonalGaussianDistribution(object):
    def __init__(self, parameters, deterministic=False):
        self.parameters = parameters
        self.mean, self.logvar = torch.chunk(parameters, 2, dim=1)
        self.logvar = torch.clamp(self.logvar, -30.0, 20.0)
        self.deterministic = deterministic
        self.std = torch.exp(0.5 * self.logvar)
        self.var = torch.exp(self.logvar)
        if self.deterministic:
            self.var = self.std = torch.zeros_like(self.mean)

    def sample(self):
        if _noise_source is not None:
            eps = _noise_source(tuple(self.mean.shape))
        else:
            eps = torch.randn(self.mean.shape)
        return self.mean + self.std * eps.to(device=self.parameters.device, dtype=self.mean.dtype)

    def kl(self, other=None):
        if self.deterministic:
            return torch.zeros([1], device=self.mean.device)
        if other is None:
            return 0.5 * torch.sum(self.mean.square() + self.var - 1.0 - self.logvar, dim=[1, 2, 3])
        return 0.5 * torch.sum((self.mean - other.mean).square() / other.var + self.var / other.var - 1.0
                               - self.logvar + other.logvar, dim=[1, 2, 3])

    def nll(self, sample, dims=(1, 2, 3)):
        if self.deterministic:
            return torch.zeros([1], device=self.mean.device)
        return 0.5 * torch.sum(np.log(2.0 * np.pi) + self.logvar + (sample - self.mean).square() / self.var,
                               dim=list(dims))

    def mode(self):
        return self.mean


def _draw_eps(shape, device, dtype):
    """The noise DiagonalGaussianDistribution.sample() draws (same source, shape and order)."""
    eps = _noise_source(tuple(shape)) if _noise_source is not None else torch.randn(shape)
    if torch.device(device).type == 'cuda' and eps.device.type == 'cpu':
        # through pinned memory, asynchronously: a pageable host-to-device copy blocks the host until the GPU
        # has drained its queue (tools_dev/sync_probe.py); the staging block is kept until the copy has run
        return eps.to(dtype=dtype).pin_memory().to(device=device, non_blocking=True)
    return eps.to(device=device, dtype=dtype)


def sample_and_kl(parameters, need_kl=True):
    """(DiagonalGaussianDistribution(parameters).sample(), .kl() or None). fp32 ROCm moments run
    the fused HIP kernel (torch_utils/ops/posterior_hip.py: one forward and one backward launch
    instead of the ~12 elementwise / reduction kernels below); elsewhere the class itself."""
    if parameters.is_cuda and parameters.dtype == torch.float32 and parameters.dim() >= 3:
        from torch_utils.ops import posterior_hip
        B, C2 = parameters.shape[:2]
        eps = _draw_eps((B, C2 // 2) + tuple(parameters.shape[2:]), parameters.device, torch.float32)
        z, kl = posterior_hip.sample_kl(parameters, eps)
        return z, (kl if need_kl else None)
    post = DiagonalGaussianDistribution(parameters)
    z = post.sample()
    return z, (post.kl() if need_kl else None)


def normal_kl(mean1, logvar1, mean2, logvar2):
    ref = next(o for o in (mean1, logvar1, mean2, logvar2) if isinstance(o, torch.Tensor))
    logvar1, logvar2 = [t if isinstance(t, torch.Tensor) else torch.tensor(t).to(ref) for t in (logvar1, logvar2)]
    return 0.5 * (-1.0 + logvar2 - logvar1 + torch.exp(logvar1 - logvar2) + (mean1 - mean2) ** 2 * torch.exp(-logvar2))
