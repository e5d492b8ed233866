"""Per-tick training statistics with one cross-rank reduction per collection.

Call surface of the reference `torch_utils/training_stats.py` (`report` :56,
`report0` :103, `Collector` :113, `init_multiprocessing`), re-designed around a
single registry object:

* every reported name owns one fp64 accumulator ``[count, sum, sum_sq]`` that
  lives on the device the values were reported from (no host sync per report);
* ``StatsRegistry.drain()`` folds all accumulators into one ``[names, 3]``
  matrix, all-reduces it once (rank-consistent name order: sorted), and adds it
  to the running totals on the host;
* a ``Collector`` remembers the totals it saw last time, so its view is the
  delta since its previous ``update()`` -- several collectors can coexist.
"""
import math
import re

import torch

import dnnlib

__all__ = ["init_multiprocessing", "report", "report0", "Collector", "default_collector"]


class StatsRegistry:
    """Owns the device-side accumulators and the host-side running totals."""

    def __init__(self):
        self.rank = 0
        self.sync_device = None        # device of the all_reduce (None: no cross-rank reduction)
        self.frozen = False            # set once the first drain ran (rank/device cannot change after)
        self.live = {}                 # name -> {device: fp64 tensor [3]}
        self.totals = {}               # name -> fp64 cpu tensor [3]

    def configure(self, rank, sync_device):
        if self.frozen and (rank, sync_device) != (self.rank, self.sync_device):
            raise RuntimeError("training_stats.init_multiprocessing() must run before the first Collector.update()")
        self.rank, self.sync_device = rank, sync_device

    def add(self, name, value):
        slots = self.live.setdefault(name, {})
        x = torch.as_tensor(value)
        if x.numel() == 0:
            return
        x = x.detach().reshape(-1).float()
        # (new_full: a fill kernel; new_tensor(python number) would be a blocking host-to-device copy on a GPU)
        acc = torch.stack([x.new_full((), float(x.numel())), x.sum(), (x * x).sum()]).double()
        cur = slots.get(acc.device)
        if cur is None:
            slots[acc.device] = acc
        else:
            cur += acc

    def drain(self, names):
        """Move the live accumulators of `names` into the totals (one collective)."""
        if not names:
            return
        self.frozen = True
        dev = self.sync_device if self.sync_device is not None else torch.device("cpu")
        block = torch.zeros([len(names), 3], dtype=torch.float64, device=dev)
        for row, name in enumerate(names):
            for acc in self.live.get(name, {}).values():
                block[row] += acc.to(dev)
                acc.zero_()
        if self.sync_device is not None and torch.distributed.is_initialized():
            torch.distributed.all_reduce(block)
        block = block.cpu()
        for row, name in enumerate(names):
            tot = self.totals.get(name)
            if tot is None:
                self.totals[name] = block[row].clone()
            else:
                tot += block[row]


_registry = StatsRegistry()


def init_multiprocessing(rank, sync_device):
    """`sync_device` = device of the per-tick all_reduce (None in single-process runs)."""
    _registry.configure(rank, sync_device)


def report(name, value):
    """Accumulate every element of `value` under `name`; returns `value` unchanged."""
    _registry.add(name, value)
    return value


def report0(name, value):
    """`report` on rank 0 only (other ranks register the name with no samples)."""
    _registry.add(name, value if _registry.rank == 0 else [])
    return value


class _Moments:
    __slots__ = ("n", "s", "ss")

    def __init__(self, n=0.0, s=0.0, ss=0.0):
        self.n, self.s, self.ss = n, s, ss

    @property
    def mean(self):
        return self.s / self.n if self.n else float("nan")

    @property
    def std(self):
        if not self.n or not math.isfinite(self.s):
            return float("nan")
        if self.n == 1:
            return 0.0
        m = self.s / self.n
        return math.sqrt(max(self.ss / self.n - m * m, 0.0))


class Collector:
    """Statistics reported since this collector's previous `update()`.

    regex: names to collect (full match). keep_previous: keep the last
    non-empty interval of a name that received nothing in the current one.
    """

    def __init__(self, regex=".*", keep_previous=True):
        self._pattern = re.compile(regex)
        self._keep_previous = keep_previous
        self._seen = {}                # name -> totals at the previous update (cpu [3])
        self._view = {}                # name -> _Moments of the last interval
        self.update()
        self._view.clear()

    def names(self):
        return sorted(n for n in _registry.live if self._pattern.fullmatch(n))

    def update(self):
        names = self.names()
        _registry.drain(names)
        if not self._keep_previous:
            self._view.clear()
        for name in names:
            tot = _registry.totals.get(name)
            if tot is None:
                continue
            prev = self._seen.get(name)
            d = tot - prev if prev is not None else tot.clone()
            self._seen[name] = tot.clone()
            if float(d[0]) != 0.0:
                self._view[name] = _Moments(float(d[0]), float(d[1]), float(d[2]))

    def _moments(self, name):
        if not self._pattern.fullmatch(name):
            raise KeyError(f"{name!r} is not collected by this Collector")
        return self._view.get(name, _Moments())

    def num(self, name):
        return self._moments(name).n

    def mean(self, name):
        return self._moments(name).mean

    def std(self, name):
        return self._moments(name).std

    def as_dict(self):
        out = dnnlib.EasyDict()
        for name in self.names():
            m = self._moments(name)
            out[name] = dnnlib.EasyDict(num=m.n, mean=m.mean, std=m.std)
        return out

    def __getitem__(self, name):
        return self.mean(name)


default_collector = Collector()
