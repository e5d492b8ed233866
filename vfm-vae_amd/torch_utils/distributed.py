"""Process-group setup and data-parallel gradient synchronisation over RCCL.

Replaces the reference `torch_utils/distributed.py:24-83` (init, rank helpers,
print0) and the training loop's post-backward flat all-reduce
(`training/training_loop.py:272-289`, `sync_grads` / `sharded_all_mean`).

MI355X design: one process per GPU; backend 'nccl' (= RCCL on ROCm) over xGMI
when CUDA/HIP devices exist, 'gloo' otherwise (CPU tests). `GradBucketer`
launches bucketed all-reduces from post-accumulate-grad hooks on a dedicated
communication stream, so the gradient exchange of the decoder's last blocks
overlaps the backward of its first blocks. The averaging keeps the reference
semantics exactly: sum over ranks / world, * gain, nan_to_num(nan=0,
posinf=1e5, neginf=-1e5), cast to the parameter dtype.
"""
import os
import math

import torch

from . import training_stats


def init(backend=None):
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29500')
    os.environ.setdefault('RANK', '0')
    os.environ.setdefault('LOCAL_RANK', '0')
    os.environ.setdefault('WORLD_SIZE', '1')
    use_gpu = torch.cuda.is_available()
    if backend is None:
        backend = 'nccl' if use_gpu else 'gloo'
    if use_gpu:
        torch.cuda.set_device(int(os.environ.get('LOCAL_RANK', '0')))
    if not torch.distributed.is_initialized():
        kwargs = {}
        if use_gpu and backend == 'nccl':
            kwargs['device_id'] = torch.device('cuda', int(os.environ.get('LOCAL_RANK', '0')))
        torch.distributed.init_process_group(backend=backend, init_method='env://', **kwargs)
    sync_device = torch.device('cuda') if (get_world_size() > 1 and use_gpu) else None
    training_stats.init_multiprocessing(rank=get_rank(), sync_device=sync_device)


def is_available():
    return torch.distributed.is_available()


def is_initialized():
    return torch.distributed.is_initialized()


def get_rank():
    return torch.distributed.get_rank() if torch.distributed.is_initialized() else 0


def get_world_size():
    return torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1


def should_stop():
    return False


def update_progress(cur, total):
    _ = cur, total


def print0(*args, **kwargs):
    if get_rank() == 0:
        print(*args, **kwargs)


def destroy_process_group():
    if is_initialized():
        torch.distributed.destroy_process_group()


# ---------------------------------------------------------------------------
# Reference-equivalent flat synchronisation (kept as the semantic baseline).


def sharded_all_mean(tensor, shard_size=2 ** 23):
    """All-reduce a flat tensor in shards and divide by the world size
    (reference training_loop.py:272-278)."""
    assert tensor.dim() == 1
    shards = tensor.tensor_split(math.ceil(tensor.numel() / shard_size))
    for s in shards:
        torch.distributed.all_reduce(s)
    return torch.cat(shards) / get_world_size()


def sync_grads(network, gain=None):
    """Flat, unoverlapped gradient averaging with the reference's exact semantics
    (reference training_loop.py:281-289)."""
    params = [p for p in network.parameters() if p.grad is not None]
    if not params:
        return
    flat = torch.cat([p.grad.flatten().float() for p in params])
    if get_world_size() > 1:
        flat = sharded_all_mean(flat)
    if gain is not None:
        flat = flat * gain
    torch.nan_to_num(flat, nan=0, posinf=1e5, neginf=-1e5, out=flat)
    for p, g in zip(params, flat.split([p.numel() for p in params])):
        p.grad = g.reshape(p.shape).to(p.dtype)


# ---------------------------------------------------------------------------
# Overlapped bucketed all-reduce.


class GradBucketer:
    """Bucketed, backward-overlapped gradient averaging for one module.

    Parameters are grouped in reverse registration order (roughly the order
    their gradients become ready in backward) into buckets of ~`bucket_mb`
    of fp32. Each parameter gets a post-accumulate-grad hook; when the last
    parameter of a bucket has its gradient, the bucket is packed into a flat
    fp32 buffer and all-reduced asynchronously on `comm_stream`. `finish()`
    waits for all buckets, applies /world * gain + nan_to_num and writes the
    averaged gradients back (reference sync_grads semantics).

    A parameter whose gradient is never produced in a step (frozen branch)
    simply leaves its bucket incomplete; `finish()` flushes incomplete buckets
    synchronously (zero-filling missing grads only when another rank produced
    them is impossible to know locally, so such parameters must be frozen on
    every rank alike, as in the reference's train_mode handling).
    """

    def __init__(self, module, bucket_mb=32.0, world_size=None, group=None):
        self.module = module
        self.group = group
        self.world = world_size or get_world_size()
        self.params = [p for p in module.parameters() if p.requires_grad]
        self.bucket_elems = max(1, int(bucket_mb * 2 ** 20 / 4))
        self.buckets = []
        cur, n = [], 0
        for p in reversed(self.params):
            cur.append(p)
            n += p.numel()
            if n >= self.bucket_elems:
                self.buckets.append(cur)
                cur, n = [], 0
        if cur:
            self.buckets.append(cur)
        self.index = {}
        for bi, b in enumerate(self.buckets):
            for p in b:
                self.index[id(p)] = bi
        self.comm_stream = torch.cuda.Stream() if (torch.cuda.is_available() and self.params and
                                                   self.params[0].is_cuda) else None
        self.hooks = []
        self._reset()
        for p in self.params:
            self.hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    def _reset(self):
        self.ready = [0] * len(self.buckets)
        self.pending = {}
        self.enabled = True

    def remove(self):
        for h in self.hooks:
            h.remove()
        self.hooks = []

    def _on_grad(self, p):
        if not self.enabled or self.world <= 1:
            return
        bi = self.index.get(id(p))
        if bi is None:
            return
        self.ready[bi] += 1
        if self.ready[bi] == len(self.buckets[bi]):
            self._launch(bi)

    def _launch(self, bi):
        params = self.buckets[bi]
        if any(p.grad is None for p in params):
            return
        flat = torch.cat([p.grad.detach().flatten().float() for p in params])
        if self.comm_stream is not None:
            self.comm_stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(self.comm_stream):
                flat.record_stream(self.comm_stream)
                work = torch.distributed.all_reduce(flat, group=self.group, async_op=True)
        else:
            work = torch.distributed.all_reduce(flat, group=self.group, async_op=True)
        self.pending[bi] = (flat, work)

    def finish(self, gain=None):
        """Complete every bucket; returns nothing, gradients are averaged in place."""
        params_with_grad = [p for p in self.params if p.grad is not None]
        if not params_with_grad:
            self._reset()
            return
        if self.world > 1:
            for bi in range(len(self.buckets)):
                if bi not in self.pending and all(p.grad is not None for p in self.buckets[bi]):
                    self._launch(bi)
            for bi, (flat, work) in sorted(self.pending.items()):
                work.wait()
                if self.comm_stream is not None:
                    torch.cuda.current_stream().wait_stream(self.comm_stream)
                self._scatter(self.buckets[bi], flat, gain)
            done = set(self.pending)
            for bi, b in enumerate(self.buckets):   # partially produced buckets: flat sync, same math
                if bi in done:
                    continue
                ps = [p for p in b if p.grad is not None]
                if ps:
                    flat = torch.cat([p.grad.flatten().float() for p in ps])
                    torch.distributed.all_reduce(flat, group=self.group)
                    self._scatter(ps, flat, gain)
        else:
            for b in self.buckets:
                ps = [p for p in b if p.grad is not None]
                if ps:
                    self._scatter(ps, torch.cat([p.grad.flatten().float() for p in ps]), gain)
        self._reset()

    def _scatter(self, params, flat, gain):
        if self.world > 1:
            flat = flat / self.world
        if gain is not None:
            flat = flat * gain
        torch.nan_to_num(flat, nan=0, posinf=1e5, neginf=-1e5, out=flat)
        for p, g in zip(params, flat.split([p.numel() for p in params])):
            p.grad.copy_(g.reshape(p.shape))
