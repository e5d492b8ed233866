"""Synthetic image source with the dataset interface the training loop uses.

Benchmarks and smoke runs train on seeded uniform uint8 images of the
configured resolution (the loop's preprocessing `uint8 / 255` is applied as for
real data, reference training_loop.py:306-307). Labels are unconditional
'cls2text' strings, ignored when `conditional: False`. `resolutions` (a list) gives
a dynamic-resolution stream: consecutive batches cycle through the sizes, one size
per (micro-)batch bucket (BASELINE config 3: 256/384/512).
"""
import torch


class SyntheticDataset:
    def __init__(self, resolution=256, num_channels=3, label_type='cls2text', label_dim=0, pool_batches=4,
                 device=None, seed=0, resolutions=None, **_unused):
        self.resolution = resolution
        self.resolutions = list(resolutions) if resolutions else [resolution]
        self.num_channels = num_channels
        self.label_type = label_type
        self.label_dim = label_dim
        self.label_shape = [label_dim]
        self.image_shape = [num_channels, resolution, resolution]
        self.pool_batches = pool_batches
        self.device = device
        self.seed = seed

    def __len__(self):
        return 1 << 30

    def make_pool(self, batch_size, device, seed=None):
        g = torch.Generator().manual_seed(self.seed if seed is None else seed)
        n = max(self.pool_batches, len(self.resolutions))
        sizes = [self.resolutions[i % len(self.resolutions)] for i in range(n)]
        pool = [torch.randint(0, 256, (batch_size, self.num_channels, r, r), dtype=torch.uint8, generator=g)
                for r in sizes]
        return [p.to(device) for p in pool]

    def iterate(self, batch_size, rank=0, world=1, seed=0):
        dev = self.device or (torch.device('cuda') if torch.cuda.is_available() else torch.device('cpu'))
        pool = self.make_pool(batch_size, dev, seed=self.seed * 1000 + rank)
        labels = ['a photo'] * batch_size
        i = 0
        while True:
            yield pool[i % len(pool)], labels
            i += 1
