import torch
from . import functional  # noqa: F401


class Normalize(torch.nn.Module):
    def __init__(self, mean, std):
        super().__init__()
        self.mean, self.std = mean, std

    def forward(self, x):
        return functional.normalize(x, self.mean, self.std)


class RandomCrop(torch.nn.Module):
    def __init__(self, size):
        super().__init__()
        self.size = size

    def forward(self, x):
        h, w = x.shape[-2:]
        i = int(torch.randint(0, h - self.size + 1, size=(1,)).item())
        j = int(torch.randint(0, w - self.size + 1, size=(1,)).item())
        return x[..., i:i + self.size, j:j + self.size]
