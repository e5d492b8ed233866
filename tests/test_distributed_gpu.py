"""The RCCL gradient all-reduce path of FlatGradSync on one GPU (reference
training/training_loop.py:272-289 sync_grads; here bucketed all-reduces launched from
post-accumulate-grad hooks on a side comm stream, training/training_loop.py FlatGradSync).

RCCL refuses two ranks on one device, so the multi-rank semantics are covered by the gloo tests
(tests/test_distributed.py); this test runs a 1-rank NCCL (= RCCL) process group with the
collective path forced on, so the comm-stream ordering (wait_stream before each bucket's
all_reduce, the compute stream waiting on the comm stream in finish), several in-flight buckets
and the rank-agreement all-reduce execute on the hardware, and checks the gradients against a
plain backward.
"""
import copy
import socket

import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_flat_grad_sync_rccl_comm_stream_one_rank():
    import torch.distributed as tdist
    from training.training_loop import FlatGradSync
    if tdist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    tdist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                             device_id=torch.device("cuda:0"))
    try:
        torch.manual_seed(0)
        net = nn.Sequential(nn.Linear(64, 512), nn.GELU(), nn.Linear(512, 512), nn.GELU(), nn.Linear(512, 64)).cuda()
        ref = copy.deepcopy(net)
        sync = FlatGradSync(net, bucket_mb=0.25, collective=True)
        for step in range(3):
            x = torch.randn(256, 64, device="cuda")
            sync.prepare()
            net(x).square().mean().backward()
            sync.finish(gain=0.5)
            ref.zero_grad(set_to_none=True)
            ref(x).square().mean().backward()
            torch.cuda.synchronize()
            for p, q in zip(net.parameters(), ref.parameters()):
                torch.testing.assert_close(p.grad, 0.5 * q.grad, rtol=1e-6, atol=1e-7)
        assert sync.comm_stream is not None
        assert len(sync.buckets) > 1, sync.buckets
        sync.prepare()               # consumes the last step's rank-agreement check
    finally:
        tdist.destroy_process_group()
