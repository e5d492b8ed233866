import torch


def normalize(x, mean, std):
    mean = torch.as_tensor(mean, dtype=x.dtype, device=x.device).view(-1, 1, 1)
    std = torch.as_tensor(std, dtype=x.dtype, device=x.device).view(-1, 1, 1)
    return (x - mean) / std
