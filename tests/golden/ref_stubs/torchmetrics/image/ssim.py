import torch


class StructuralSimilarityIndexMeasure(torch.nn.Module):
    def __init__(self, data_range=None, **kw):
        super().__init__()

    def forward(self, a, b):
        raise NotImplementedError("SSIM is not exercised by the golden configs")
