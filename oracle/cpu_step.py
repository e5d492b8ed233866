"""CPU restatement of one VFM-VAE training iteration — TEST/BASELINE INFRASTRUCTURE.

Runs the same TrainingIteration (D phase + G phase + sync + Adam + EMA) on the
host with every op in its pure-torch form (the `impl='ref'` formulations that
tests/test_networks_parity.py pins to the reference's golden vectors). Used only
as bench.py's `cpu_baseline` leg ("port": this package's CPU restatement of the
reference algorithm; the reference itself cannot travel to the GPU box).
"""
import copy
import os
import random
import time

import numpy as np
import torch
import yaml


def time_iteration(cfg_path, batch=1, threads=0, iters=5, warmup=2):
    """`warmup` untimed iterations, then the median of `iters` timed ones."""
    import dnnlib
    from train import resolve_config
    from torch_utils.ops import decoder_ops
    from training.training_loop import TrainingIteration, make_optimizer
    n = threads or min(16, os.cpu_count() or 1)
    torch.set_num_threads(n)
    decoder_ops.set_force_ref(True)
    dev = torch.device("cpu")
    c = resolve_config(yaml.safe_load(open(cfg_path)))
    torch.manual_seed(c.get("random_seed", 42))
    random.seed(0)
    np.random.seed(0)
    G = dnnlib.util.construct_class_by_name(label_dim=0, **c.G_kwargs).train().requires_grad_(False)
    D = dnnlib.util.construct_class_by_name(c_dim=G.c_dim, **c.D_kwargs).train().requires_grad_(False)
    loss = dnnlib.util.construct_class_by_name(device=dev, G=G, D=D, **c.loss_kwargs)
    it = TrainingIteration(G, D, copy.deepcopy(G).eval(), loss, make_optimizer(G.parameters(), c.G_opt_kwargs, dev),
                           make_optimizer(D.parameters(), c.D_opt_kwargs, dev), batch_size=batch,
                           ema_kimg=c.ema_kimg, ema_rampup=c.ema_rampup)
    res = c.training_set_kwargs.get("resolution", 256)
    g = torch.Generator().manual_seed(0)
    img = torch.randint(0, 256, (batch, 3, res, res), dtype=torch.uint8, generator=g).float() / 255.
    for i in range(warmup):
        it([img], [["a photo"] * batch], i * batch)
    times = []
    for i in range(iters):
        t0 = time.perf_counter()
        it([img], [["a photo"] * batch], (warmup + i) * batch)
        times.append(time.perf_counter() - t0)
    decoder_ops.set_force_ref(False)
    dt = float(np.median(times))
    return {"value": round(batch / dt, 5), "unit": "images/sec", "cores": torch.get_num_threads(),
            "host_cpus": os.cpu_count(), "kind": "port",
            "sample": f"median of {iters} full stage-0 iterations (D+G+Adam+EMA) after {warmup} warm-up, batch "
                      f"{batch}, {res}px, same architectures, fp32 torch CPU ops; {dt:.2f} s per iteration "
                      f"(min {min(times):.2f}, max {max(times):.2f})"}
