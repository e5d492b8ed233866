"""No library GEMM or convolution in the training step.

The benchmark iteration (BASELINE configs[1]: stage-0 SigLIP2-L, here at batch 8 to keep the test short; the
per-image shapes are the bench's) is run once per equivariance outcome -- the shape classes the timed steps draw
-- under a TorchDispatchMode that records every aten matrix product / convolution on a ROCm tensor: hipBLASLt
(`Cijk_*` kernels) and MIOpen would run exactly there. Every product of the step must be on our kernels
(csrc/gemm9.hip, gemm8.hip, gemm.hip, sgemm.hip, conv.hip, ...), so the list must be empty."""
import os
import traceback

import pytest
import torch
import yaml
from torch.utils._python_dispatch import TorchDispatchMode

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
LIB_OPS = ("aten.mm", "aten.bmm", "aten.addmm", "aten.baddbmm", "aten.addbmm", "aten.matmul", "aten.linear",
           "aten.convolution", "aten._convolution", "aten.cudnn_convolution", "aten.miopen_convolution",
           "aten.convolution_backward", "aten._scaled_dot_product", "aten.addmv", "aten.mv", "aten.dot")


class _Record(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.hits = []

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        if name.startswith(LIB_OPS) and any(isinstance(a, torch.Tensor) and a.is_cuda for a in args):
            where = [f"{os.path.relpath(f.filename, ROOT)}:{f.lineno}" for f in traceback.extract_stack()
                     if ROOT in f.filename and "tests" not in f.filename][-3:]
            node = torch._C._current_autograd_node()
            shapes = [tuple(a.shape) for a in args if isinstance(a, torch.Tensor)]
            self.hits.append((name, shapes, node.name() if node is not None else "fwd", " < ".join(where)))
        return func(*args, **(kwargs or {}))


def test_stage0_step_runs_no_library_gemm():
    from train import resolve_config
    from training.training_loop import configure_backends, construct_networks, construct_iteration
    c = resolve_config(yaml.safe_load(open(os.path.join(PKG, "configs", "vfm_vae_f16d32_siglip2_stage_0_synthetic.yaml"))))
    configure_backends(c.get("cudnn_benchmark", True))
    torch.manual_seed(0)
    batch = 8
    G, G_ema, D = construct_networks(c.G_kwargs, c.D_kwargs, DEV)
    step = construct_iteration(G, D, G_ema, DEV, c.loss_kwargs, c.G_opt_kwargs, c.D_opt_kwargs, batch_size=batch,
                               ema_kimg=c.ema_kimg, ema_rampup=c.ema_rampup)
    g = torch.Generator().manual_seed(0)
    img = (torch.randint(0, 256, (batch, 3, 256, 256), dtype=torch.uint8, generator=g).float() / 255.).to(DEV)
    labels = ["a photo"] * batch
    eqt = step.G.equivariance_transform
    rec = _Record()
    for i, v in enumerate(eqt.variants()):
        eqt.forced = v
        step([img], [labels], i * batch)          # warm (first use of each shape class)
        with rec:
            step([img], [labels], i * batch)
    eqt.forced = None
    torch.cuda.synchronize()
    uniq = {}
    for h in rec.hits:
        uniq.setdefault((h[0], str(h[1]), h[2], h[3]), 0)
        uniq[(h[0], str(h[1]), h[2], h[3])] += 1
    msg = "\n".join(f"{n:3d}x {k[0]} {k[1]} [{k[2]}] {k[3]}" for k, n in sorted(uniq.items(), key=lambda kv: -kv[1]))
    assert not rec.hits, f"library GEMM / convolution calls in the step:\n{msg}"
