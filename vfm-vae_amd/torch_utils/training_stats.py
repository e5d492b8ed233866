"""Training statistics: cheap on-device accumulation, cross-rank reduction per tick.

Same surface as the reference `torch_utils/training_stats.py` (report :56,
report0 :103, Collector :113, init_multiprocessing). Moments [n, sum, sum^2]
are accumulated on the reporting tensor's device in fp64 and reduced with one
all_reduce per `Collector.update()`.
"""
import re

import numpy as np
import torch

import dnnlib

_num_moments = 3
_reduce_dtype = torch.float32
_counter_dtype = torch.float64
_rank = 0
_sync_device = None
_sync_called = False
_counters = dict()     # name -> {device: tensor[3]}
_cumulative = dict()   # name -> tensor[3] (cpu)


def init_multiprocessing(rank, sync_device):
    global _rank, _sync_device
    assert not _sync_called
    _rank = rank
    _sync_device = sync_device


def report(name, value):
    """Accumulate the elements of `value` under `name`; returns value unchanged."""
    if name not in _counters:
        _counters[name] = dict()
    elems = torch.as_tensor(value)
    if elems.numel() == 0:
        return value
    elems = elems.detach().flatten().to(_reduce_dtype)
    moments = torch.stack([torch.ones_like(elems).sum(), elems.sum(), elems.square().sum()])
    moments = moments.to(_counter_dtype)
    device = moments.device
    if device not in _counters[name]:
        _counters[name][device] = torch.zeros_like(moments)
    _counters[name][device].add_(moments)
    return value


def report0(name, value):
    report(name, value if _rank == 0 else [])
    return value


class Collector:
    """Collects the statistics reported since the previous update()."""

    def __init__(self, regex='.*', keep_previous=True):
        self._regex = re.compile(regex)
        self._keep_previous = keep_previous
        self._cumulative = dict()
        self._moments = dict()
        self.update()
        self._moments.clear()

    def names(self):
        return [name for name in _counters if self._regex.fullmatch(name)]

    def update(self):
        if not self._keep_previous:
            self._moments.clear()
        for name, cumulative in _sync(self.names()):
            if name not in self._cumulative:
                self._cumulative[name] = torch.zeros([_num_moments], dtype=_counter_dtype)
            delta = cumulative - self._cumulative[name]
            self._cumulative[name].copy_(cumulative)
            if float(delta[0]) != 0:
                self._moments[name] = delta

    def _get_delta(self, name):
        assert self._regex.fullmatch(name)
        if name not in self._moments:
            self._moments[name] = torch.zeros([_num_moments], dtype=_counter_dtype)
        return self._moments[name]

    def num(self, name):
        return float(self._get_delta(name)[0])

    def mean(self, name):
        d = self._get_delta(name)
        return float('nan') if int(d[0]) == 0 else float(d[1] / d[0])

    def std(self, name):
        d = self._get_delta(name)
        if int(d[0]) == 0 or not np.isfinite(float(d[1])):
            return float('nan')
        if int(d[0]) == 1:
            return 0.0
        mean = float(d[1] / d[0])
        raw_var = float(d[2] / d[0])
        return np.sqrt(max(raw_var - np.square(mean), 0))

    def as_dict(self):
        stats = dnnlib.EasyDict()
        for name in self.names():
            stats[name] = dnnlib.EasyDict(num=self.num(name), mean=self.mean(name), std=self.std(name))
        return stats

    def __getitem__(self, name):
        return self.mean(name)


def _sync(names):
    """Sum the per-device counters (and across ranks) into _cumulative; one collective."""
    global _sync_called
    if len(names) == 0:
        return []
    _sync_called = True
    deltas = []
    device = _sync_device if _sync_device is not None else torch.device('cpu')
    for name in names:
        delta = torch.zeros([_num_moments], dtype=_counter_dtype, device=device)
        for counter in _counters[name].values():
            delta.add_(counter.to(device))
            counter.copy_(torch.zeros_like(counter))
        deltas.append(delta)
    deltas = torch.stack(deltas)
    if _sync_device is not None and torch.distributed.is_initialized():
        torch.distributed.all_reduce(deltas)
    deltas = deltas.cpu()
    for idx, name in enumerate(names):
        if name not in _cumulative:
            _cumulative[name] = torch.zeros([_num_moments], dtype=_counter_dtype)
        _cumulative[name].add_(deltas[idx])
    return [(name, _cumulative[name]) for name in names]


default_collector = Collector()
