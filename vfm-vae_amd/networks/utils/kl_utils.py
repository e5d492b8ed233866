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


def normal_kl(mean1, logvar1, mean2, logvar2):
    ref = next(o for o in (mean1, logvar1, mean2, logvar2) if isinstance(o, torch.Tensor))
    logvar1, logvar2 = [t if isinstance(t, torch.Tensor) else torch.tensor(t).to(ref) for t in (logvar1, logvar2)]
    return 0.5 * (-1.0 + logvar2 - logvar1 + torch.exp(logvar1 - logvar2) + (mean1 - mean2) ** 2 * torch.exp(-logvar2))
