"""Small tensor/module helpers used across the training path.

Same call surface as the reference `torch_utils/misc.py` (assert_shape :92-105,
profiled_function :110-116, params_and_buffers / copy_params_and_buffers,
check_ddp_consistency :218-229, print_module_summary, InfiniteSampler), written
fresh for this package.
"""
import contextlib
import re
import warnings

import numpy as np
import torch

_constants = {}


def constant(value, shape=None, dtype=None, device=None, memory_format=None):
    """Cached device constant (avoids re-uploading the same small tensor)."""
    arr = np.asarray(value)
    dtype = dtype or torch.get_default_dtype()
    device = torch.device("cpu") if device is None else torch.device(device)
    memory_format = memory_format or torch.contiguous_format
    key = (arr.shape, arr.dtype.str, arr.tobytes(), None if shape is None else tuple(shape), dtype, device, memory_format)
    t = _constants.get(key)
    if t is None:
        t = torch.as_tensor(arr.copy(), dtype=dtype, device=device)
        if shape is not None:
            t = t.expand(tuple(shape))
        t = t.contiguous(memory_format=memory_format)
        _constants[key] = t
    return t


nan_to_num = torch.nan_to_num


@contextlib.contextmanager
def suppress_tracer_warnings():
    flt = ("ignore", None, torch.jit.TracerWarning, None, 0)
    warnings.filters.insert(0, flt)
    try:
        yield
    finally:
        warnings.filters.remove(flt)


def assert_shape(tensor, ref_shape):
    """Raise AssertionError unless tensor.shape matches ref_shape (None = any)."""
    if tensor.ndim != len(ref_shape):
        raise AssertionError(f"Wrong number of dimensions: got {tensor.ndim}, expected {len(ref_shape)}")
    for i, (got, want) in enumerate(zip(tensor.shape, ref_shape)):
        if want is None:
            continue
        if isinstance(want, torch.Tensor):
            want = int(want)
        if int(got) != int(want):
            raise AssertionError(f"Wrong size for dimension {i}: got {got}, expected {want}")


def profiled_function(fn):
    """Wrap fn in a profiler range named after it (kept for trace parity)."""
    def wrapper(*args, **kwargs):
        with torch.autograd.profiler.record_function(fn.__name__):
            return fn(*args, **kwargs)
    wrapper.__name__ = fn.__name__
    wrapper.__doc__ = fn.__doc__
    return wrapper


class InfiniteSampler(torch.utils.data.Sampler):
    """Endless, optionally shuffled index stream partitioned over ranks."""

    def __init__(self, dataset, rank=0, num_replicas=1, shuffle=True, seed=0, window_size=0.5):
        assert len(dataset) > 0 and num_replicas > 0 and 0 <= rank < num_replicas and 0 <= window_size <= 1
        self.dataset = dataset
        self.rank = rank
        self.num_replicas = num_replicas
        self.shuffle = shuffle
        self.seed = seed
        self.window_size = window_size

    def __iter__(self):
        order = np.arange(len(self.dataset))
        rnd = None
        window = 0
        if self.shuffle:
            rnd = np.random.RandomState(self.seed)
            rnd.shuffle(order)
            window = int(np.rint(order.size * self.window_size))
        idx = 0
        while True:
            i = idx % order.size
            if idx % self.num_replicas == self.rank:
                yield order[i]
            if window >= 2:
                j = (i - rnd.randint(window)) % order.size
                order[i], order[j] = order[j], order[i]
            idx += 1


def params_and_buffers(module):
    assert isinstance(module, torch.nn.Module)
    return list(module.parameters()) + list(module.buffers())


def named_params_and_buffers(module):
    assert isinstance(module, torch.nn.Module)
    return list(module.named_parameters()) + list(module.named_buffers())


@torch.no_grad()
def copy_params_and_buffers(src_module, dst_module, require_all=False):
    src = dict(named_params_and_buffers(src_module))
    for name, tensor in named_params_and_buffers(dst_module):
        if name in src:
            tensor.copy_(src[name])
        elif require_all:
            raise KeyError(name)


@contextlib.contextmanager
def ddp_sync(module, sync):
    if isinstance(module, torch.nn.parallel.DistributedDataParallel) and not sync:
        with module.no_sync():
            yield
    else:
        yield


def check_ddp_consistency(module, ignore_regex=None):
    """Assert that every rank holds identical parameters/buffers (broadcast + compare)."""
    for name, tensor in named_params_and_buffers(module):
        full = type(module).__name__ + "." + name
        if ignore_regex is not None and re.fullmatch(ignore_regex, full):
            continue
        t = tensor.detach()
        if t.is_floating_point():
            t = torch.nan_to_num(t)
        other = t.clone()
        torch.distributed.broadcast(tensor=other, src=0)
        assert (t == other).all(), full


def print_module_summary(module, inputs, max_nesting=3, skip_redundant=True):
    """Print per-submodule output shapes and parameter counts for one forward."""
    assert isinstance(module, torch.nn.Module) and isinstance(inputs, (tuple, list))
    rows = []
    nesting = [0]

    def pre_hook(_mod, _inputs):
        nesting[0] += 1

    def post_hook(mod, _inputs, outputs):
        nesting[0] -= 1
        if nesting[0] <= max_nesting:
            outs = list(outputs) if isinstance(outputs, (tuple, list)) else [outputs]
            rows.append((mod, [t for t in outs if isinstance(t, torch.Tensor)]))

    hooks = []
    for m in module.modules():
        hooks.append(m.register_forward_pre_hook(pre_hook))
        hooks.append(m.register_forward_hook(post_hook))
    outputs = module(*inputs)
    for h in hooks:
        h.remove()
    names = {mod: name for name, mod in module.named_modules()}
    seen = set()
    table = [["Module", "Parameters", "Output shape", "Datatype"]]
    for mod, outs in rows:
        n_params = sum(p.numel() for p in mod.parameters(recurse=False) if id(p) not in seen)
        for p in mod.parameters(recurse=False):
            seen.add(id(p))
        if skip_redundant and not n_params and not outs:
            continue
        shape = str(list(outs[0].shape)) if outs else "-"
        dtype = str(outs[0].dtype).split(".")[-1] if outs else "-"
        table.append([names.get(mod, "?") or "<top>", str(n_params) if n_params else "-", shape, dtype])
    widths = [max(len(r[i]) for r in table) for i in range(4)]
    for r in table:
        print("  ".join(c.ljust(w) for c, w in zip(r, widths)))
    return outputs
