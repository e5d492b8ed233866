"""Process-group setup and data-parallel gradient synchronisation over RCCL.

Replaces the reference `torch_utils/distributed.py:24-83` (init, rank helpers,
print0) and the training loop's post-backward flat all-reduce
(`training/training_loop.py:272-289`, `sync_grads` / `sharded_all_mean`).

MI355X design: one process per GPU; backend 'nccl' (= RCCL on ROCm) over xGMI
when CUDA/HIP devices exist, 'gloo' otherwise (CPU tests). The gradient
exchange itself lives next to the optimizer step (`training.training_loop.
FlatGradSync`: bucketed all-reduces launched from post-accumulate-grad hooks on
a dedicated communication stream, reference averaging semantics).
"""
import os

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
