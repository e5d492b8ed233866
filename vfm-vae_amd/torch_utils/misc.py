"""Small tensor/module helpers used across the training path.

Covers the parts of the reference `torch_utils/misc.py` that the hot path calls:
shape assertions (`assert_shape`, reference :92-105, used by the generator's
legacy layers), profiler ranges (`profiled_function`, :110-116), parameter /
buffer iteration for broadcasts and copies, and the snapshot-time replica check
(`check_ddp_consistency`, :218-229). The reference's data-loader sampler and
module-summary printer are not part of this path (synthetic / WebDataset input
streams shard themselves, training/data_wds.py).
"""
import functools
import re

import torch


def assert_shape(tensor, ref_shape):
    """Raise AssertionError unless tensor.shape matches ref_shape (None = any size)."""
    if tensor.ndim != len(ref_shape):
        raise AssertionError(f"Wrong number of dimensions: got {tensor.ndim}, expected {len(ref_shape)}")
    bad = [(i, int(g), int(w)) for i, (g, w) in enumerate(zip(tensor.shape, ref_shape))
           if w is not None and int(g) != int(w)]
    if bad:
        i, g, w = bad[0]
        raise AssertionError(f"Wrong size for dimension {i}: got {g}, expected {w}")


def profiled_function(fn):
    """Run `fn` inside a profiler range of its own name (trace parity with the reference)."""
    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        with torch.autograd.profiler.record_function(fn.__name__):
            return fn(*args, **kwargs)
    return wrapper


def named_params_and_buffers(module):
    """[(name, tensor)] over parameters then buffers, in registration order."""
    return [*module.named_parameters(), *module.named_buffers()]


def params_and_buffers(module):
    return [t for _, t in named_params_and_buffers(module)]


@torch.no_grad()
def copy_params_and_buffers(src_module, dst_module, require_all=False):
    """Copy same-named tensors src -> dst (missing names raise only if require_all)."""
    src = dict(named_params_and_buffers(src_module))
    for name, dst in named_params_and_buffers(dst_module):
        s = src.get(name)
        if s is not None:
            dst.copy_(s)
        elif require_all:
            raise KeyError(name)


@torch.no_grad()
def check_ddp_consistency(module, ignore_regex=None):
    """Assert every rank holds the same parameters/buffers as rank 0 (NaNs compare equal)."""
    prefix = type(module).__name__ + "."
    for name, t in named_params_and_buffers(module):
        full = prefix + name
        if ignore_regex is not None and re.fullmatch(ignore_regex, full):
            continue
        mine = t.detach().nan_to_num() if t.is_floating_point() else t.detach()
        rank0 = mine.clone()
        torch.distributed.broadcast(rank0, src=0)
        if not torch.equal(mine, rank0):
            raise AssertionError(f"replica mismatch in {full}")
