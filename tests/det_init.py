"""Deterministic, name-keyed re-initialisation of every parameter and buffer.

Both the reference modules (in tests/golden/make_golden_networks.py) and this
package's modules (in the parity tests) are overwritten with the same values,
so their outputs can be compared without shipping 500 MB of weights as
fixtures. Values depend only on the tensor's state-dict name and shape.
"""
import zlib

import torch


def _gen(name):
    return torch.Generator().manual_seed(zlib.crc32(name.encode()) & 0x7FFFFFFF)


def canonical(name):
    """Collapse layout differences between transformers versions (SiglipVisionModel
    nested `vision_model.vision_model.*` in 4.x vs flat `vision_model.*` in 5.x)."""
    return name.replace('vision_model.vision_model.', 'vision_model.')


def value_for(name, shape):
    name = canonical(name)
    g = _gen(name)
    leaf = name.rsplit('.', 1)[-1]
    n = 1
    for s in shape:
        n *= s
    if len(shape) == 0:
        return torch.tensor(0.1 + 0.05 * float(torch.rand([], generator=g)))      # noise_strength etc.
    if leaf in ('weight_u', 'weight_v'):
        v = torch.randn(shape, generator=g)
        return v / v.norm()
    if leaf in ('noise_const', 'freqs', 'phases', 'probe', 'cls_token', 'null_kv'):
        return torch.randn(shape, generator=g) * 0.5
    if 'pos_embed' in name or 'position_embedding' in name:
        return torch.randn(shape, generator=g) * 0.1
    if leaf == 'gamma':
        return 0.5 + 0.2 * torch.randn(shape, generator=g)
    if leaf in ('bias', 'q_bias', 'v_bias', 'in_proj_bias') or leaf.endswith('_bias'):
        return 0.05 * torch.randn(shape, generator=g)
    if leaf == 'blur_weight' or leaf == 'resample_filter' or leaf == 'transform' or leaf == 'zero_k_bias':
        return None                                                                # keep constructor value
    if leaf in ('shift', 'scale'):
        return None
    if leaf == 'x_avg' or leaf == 'vocab_usage':
        return torch.zeros(shape)
    if len(shape) == 1:                                                            # norm weights
        return 1.0 + 0.1 * torch.randn(shape, generator=g)
    fan_in = n // shape[0]
    return torch.randn(shape, generator=g) / max(fan_in, 1) ** 0.5


@torch.no_grad()
def det_init(module, prefix=''):
    """Overwrite params + buffers of `module` in place; returns list of names touched."""
    touched = []
    persistent = set(module.state_dict().keys())
    items = list(module.named_parameters()) + list(module.named_buffers())
    for name, t in items:
        if name not in persistent:          # non-persistent buffers (constants) keep their values
            continue
        full = prefix + name
        if t.dtype in (torch.int64, torch.int32, torch.bool, torch.uint8):
            continue
        v = value_for(full, tuple(t.shape))
        if v is None:
            continue
        t.copy_(v.to(t.dtype))
        touched.append(full)
    return touched
