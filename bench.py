#!/usr/bin/env python
"""VFM-VAE training throughput on MI355X.

Metric (BASELINE.json): train images/sec at 256^2, f16d32, SigLIP2-L encoder,
stage-0 strong-alignment loss mix (L1 + LPIPS + multiscale + adaptive VF + KL +
StyleGAN-T D), batch 32 per GPU. One "step" = one full training iteration of
training/training_loop.py (D phase + G phase + gradient sync + Adam + G_ema).

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Prints ONE JSON line on rank 0 (value = images/sec over all ranks, max-over-rank
step time). Extra keys: `roofline` (dominant HIP kernel, HIP-event timed during
the timed region) and `cpu_baseline` (the pure-torch CPU restatement of the same
iteration on the host cores, bounded sample).
"""
import argparse
import gc
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "vfm-vae_amd")
for _p in (PKG, ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np
import torch
import yaml

CONFIG = os.path.join(PKG, "configs", "vfm_vae_f16d32_siglip2_stage_0_synthetic.yaml")
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "pmc_traffic.json")
BF16_PEAK_TFLOPS = 2500.0      # dense
FLOP_TABLE = os.path.join(ROOT, "profiles", "r2_flops.json")
TIMED_SEED = 4631


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=32, help="images per GPU")
    ap.add_argument("--config", default=CONFIG)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-gc-freeze", action="store_true")
    ap.add_argument("--no-kernel-timer", action="store_true",
                    help="A/B: no per-launch HIP events in the timed region (no roofline object)")
    ap.add_argument("--timer-steps", type=int, default=1,
                    help="kernel timing in every n-th timed step only (1 = all timed steps, the default). The timed "
                         "steps draw different equivariance outcomes (decode scales), so a region's launches differ in "
                         "shape from step to step: timing only steps 0, 4, 8, 12, 16 (round 5's default) averaged those "
                         "steps' draws and read the decoder kernels 20-30 %% below their rocprof average over all 20 "
                         "steps (gpurun_out r6o, profiles/r6_timer_vs_rocprof_*.txt)")
    ap.add_argument("--timer-every", type=int, default=20,
                    help="per-launch HIP events on 1/n of each kernel region's launches, stratified by launch "
                         "position within a step: position j of the k-th timed step is timed when (j + k) %% n == 0, "
                         "so with n = 20 over the 20 timed steps every position of a step's launch sequence is timed "
                         "exactly once, in a different step for each position (every step's draw enters). The same "
                         "number of timed launches as 1/4 of every 4th step. Not every launch of whole steps: "
                         "back-to-back event-bound launches run serialised, which timed the LPIPS conv 27 %% below its "
                         "rocprof duration (profiles/r4_am_bench.json)")
    ap.add_argument("--timer-prepass", type=int, default=-1,
                    help="untimed steps after the warm-up in which every kernel region is timed (stratified as "
                         "--timer-every) to rank the regions and fill `all_kernels`; they draw the timed steps' own "
                         "seeded sequence of equivariance outcomes, so with the default (-1: as many as --steps) they "
                         "run the timed steps' shape mix. The timed steps then count and time only the dominant "
                         "region, so the timer's per-launch bookkeeping stays out of the measured wall time (~2 %% "
                         "with every region timed, profiles/r6_bm_timer_overhead_ab.txt). 0: every region timed "
                         "inside the timed steps")
    ap.add_argument("--trace", action="store_true", help="per-phase wall times during warmup (stderr)")
    ap.add_argument("--graphs", nargs="?", const="on", default="off", choices=["auto", "on", "off"],
                    help="replay the D phase's no-grad generator forward from HIP graphs (DESIGN.md §5). Default off: "
                         "the same eager path at N = 1 and N > 1 (the replay measured +1.1 %% over 7 same-box pairs, "
                         "inside the bench noise, profiles/r4_al_graphs_ab.txt); on = opt in for one process; auto = "
                         "on for a single process with the default config only")
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu: the same main() on the host (the 2-rank gloo test of the world > 1 branch, "
                         "tests/test_distributed.py); the bench proper is cuda")
    ap.add_argument("--force-ref-ops", action="store_true", help="A/B: torch formulation of the decoder ops")
    ap.add_argument("--tunableop", choices=["off", "use", "tune"], default="off",
                    help="GEMM solution table (torch TunableOp over hipBLASLt/rocBLAS): 'use' reads the "
                         "committed table without tuning, 'tune' measures every GEMM shape and writes "
                         "the table to --tunableop-out")
    ap.add_argument("--tunableop-out", default=os.path.join(ROOT, "gpurun_out", "tunableop", "gemm_results.csv"))
    return ap.parse_args(argv)


TUNABLEOP_TABLE = os.path.join(PKG, "tunableop", "gemm_results.csv")


def setup_tunableop(mode, out_path):
    """TunableOp: per-shape GEMM solution choice. 'use' loads the committed table (tuned on an
    MI355X with this image; validators = torch/ROCm/hipBLASLt versions + gfx950) and never
    tunes, so a fresh box pays no tuning time; shapes missing from the table keep the default
    heuristic. Nothing is written back into the repo."""
    if mode == "off":
        return None
    import torch.cuda.tunable as tun
    tun.enable(True)
    if mode == "use":
        if not os.path.exists(TUNABLEOP_TABLE):
            raise FileNotFoundError(TUNABLEOP_TABLE)
        tun.tuning_enable(False)
        tun.set_filename(os.path.join("/tmp", f"vfm_tunableop_{os.getpid()}.csv"))
        ok = tun.read_file(TUNABLEOP_TABLE)
        return {"mode": "use", "table": os.path.relpath(TUNABLEOP_TABLE, ROOT), "loaded": bool(ok),
                "entries": len(tun.get_results())}
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(int(os.environ.get("VFM_TUNE_MS", "25")))
    tun.set_max_tuning_iterations(int(os.environ.get("VFM_TUNE_ITERS", "20")))
    tun.set_filename(out_path)
    return {"mode": "tune", "out": out_path}


def build(cfg_path, batch_gpu, device, world, graphs=False):
    """G, G_ema, D, loss, optimisers and the TrainingIteration, through the SAME helpers
    training_loop() uses (training/training_loop.py construct_networks / construct_iteration /
    configure_backends), so the measured iteration is the one train.py runs."""
    from train import resolve_config
    from training.training_loop import configure_backends, construct_networks, construct_iteration
    c = resolve_config(yaml.safe_load(open(cfg_path)))
    configure_backends(c.get("cudnn_benchmark", True))
    torch.manual_seed(c.get("random_seed", 42))
    random.seed(c.get("random_seed", 42))
    np.random.seed(c.get("random_seed", 42))
    G, G_ema, D = construct_networks(c.G_kwargs, c.D_kwargs, device, label_dim=0)
    step = construct_iteration(G, D, G_ema, device, c.loss_kwargs, c.G_opt_kwargs, c.D_opt_kwargs,
                               batch_size=batch_gpu * world, accumulate_gradients=1, ema_kimg=c.ema_kimg,
                               ema_rampup=c.ema_rampup, graph_nograd_forward=graphs)
    return c, step


def _fp32_mode():
    from torch_utils import custom_ops
    return {"f32x6": "f32x6 (three exact bf16 pieces per operand, six products, fp32 accumulation)",
            "f32x3": "f32x3 OPT-IN (hi/lo, three products, ~2^-15.5 per product: below fp32)"}[custom_ops.F32_PRODUCTS]


def _log(rank, msg):
    """Progress on stderr (the JSON line is the only stdout output)."""
    if rank == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def step_flops(draws, hits, batch, steps, value):
    """Step-level MFMA fraction: the timed steps' matrix-work FLOPs (GEMM / conv / attention
    products, per image, per equivariance outcome of each phase: profiles/r2_flops.json from
    tools_dev/count_flops.py) x images/s / dense bf16 peak. Each step draws one outcome in its
    D phase and one in its G phase; the G phase is priced with or without the VFM tower
    depending on whether it reused the D phase's features."""
    if not os.path.exists(FLOP_TABLE):
        return None
    tab = json.load(open(FLOP_TABLE))
    if len(draws) != 2 * steps or len(hits) != steps:
        return {"error": f"{len(draws)} equivariance draws / {len(hits)} steps (expected 2 per step)"}
    key = lambda v: f"{float(v[0])},{int(bool(v[2]))}"
    total = 0.0
    for i in range(steps):
        vd, vg = draws[2 * i], draws[2 * i + 1]
        g = tab["G"][key(vg)]
        total += tab["D"][key(vd)] + (g["1"] if hits[i] and g.get("1") is not None else g["0"])
    per_img = total / steps
    achieved = value * per_img / 1e12
    return {"flops_per_img": round(per_img / 1e12, 4), "unit": "TFLOP/img", "achieved_tflops": round(achieved, 1),
            "peak_tflops": BF16_PEAK_TFLOPS, "frac": round(achieved / BF16_PEAK_TFLOPS, 4),
            "reuse_steps": int(sum(1 for h in hits if h)), "table": os.path.relpath(FLOP_TABLE, ROOT)}


def cpu_baseline(cfg_path, threads):
    """The same iteration through the pure-torch CPU restatement, batch 1 (bounded sample)."""
    from oracle import cpu_step
    return cpu_step.time_iteration(cfg_path, batch=1, threads=threads)


def main(argv=None):
    args = parse_args(argv)
    from torch_utils import distributed as dist
    from torch_utils.ops import decoder_ops, kernel_timer
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env > 1:
        dist.init()
    rank, world = dist.get_rank(), dist.get_world_size()
    assert world == args.gpus or world_env == 1, f"--gpus {args.gpus} but WORLD_SIZE {world}"
    on_gpu = args.device == "cuda"
    if on_gpu:
        device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        torch.cuda.set_device(device)
    else:
        device = torch.device("cpu")

    def sync():
        if on_gpu:
            torch.cuda.synchronize()
    if args.force_ref_ops:
        decoder_ops.set_force_ref(True)
    use_graphs = on_gpu and (args.graphs == "on" or (args.graphs == "auto" and world == 1 and args.config == CONFIG))
    if args.tunableop == "tune":
        use_graphs = False               # a GEMM cannot be tuned inside a HIP-graph capture
    if use_graphs:
        os.environ.setdefault("VFM_EXPERIMENTAL_GRAPHS", "1")    # the bench opts in explicitly
    tunable = setup_tunableop(args.tunableop, args.tunableop_out)
    if tunable:
        _log(rank, f"tunableop: {tunable}")

    t_start = time.perf_counter()
    c, step = build(args.config, args.batch, device, world, graphs=use_graphs)
    _log(rank, f"built in {time.perf_counter() - t_start:.1f}s")
    from training.data_synthetic import SyntheticDataset
    pool = SyntheticDataset(resolution=c.training_set_kwargs.resolution, seed=rank).make_pool(args.batch, device)
    labels = ['a photo'] * args.batch

    def one(i, cur_nimg):
        img = pool[i % len(pool)].to(torch.float32) / 255.
        step([img], [labels], cur_nimg)

    # The equivariance regulariser (stage-0 config) decodes at 1/4..1 scale on random
    # steps: run every shape class once first so no kernel load/compile (MIOpen,
    # hipBLASLt) lands in the timed region. These extra steps are untimed warm-up.
    eqt = step.G.equivariance_transform
    t1 = time.perf_counter()
    for v in eqt.variants():
        eqt.forced = v
        one(0, 0)
    eqt.forced = None
    sync()
    _log(rank, f"shape warm-up ({len(eqt.variants())} variants): {time.perf_counter() - t1:.1f}s")
    gr = getattr(step.loss, "graphed_nograd", None)
    if gr is not None:
        _log(rank, f"D-phase G forward: {len(gr.graphs)} HIP graphs captured"
                   + (f"; capture disabled ({gr.disabled})" if gr.disabled else ""))
    step.trace = (lambda m: _log(rank, m)) if args.trace else None
    if args.trace:
        _gc_t = {}

        def _gc_cb(phase, info):
            if phase == "start":
                _gc_t["t"] = time.perf_counter()
            elif info.get("generation", 0) >= 1:
                d = time.perf_counter() - _gc_t.get("t", time.perf_counter())
                if d > 0.01:
                    _log(rank, f"gc gen{info['generation']} took {d:.3f}s collected {info.get('collected')}")
        gc.callbacks.append(_gc_cb)
    cur = 0
    for i in range(args.warmup):
        t1 = time.perf_counter()
        one(i, cur)
        cur += args.batch * world
        sync()
        _log(rank, f"warmup {i + 1}/{args.warmup}: {time.perf_counter() - t1:.2f}s")
    if not args.trace:
        step.trace = None
    prepass, target = None, None
    n_pre = args.steps if args.timer_prepass < 0 else args.timer_prepass
    if on_gpu and not args.no_kernel_timer and n_pre > 0:
        # rank the kernel regions over untimed steps; the timed steps below time only the dominant one. The
        # pre-pass draws the timed steps' seeded outcome sequence (same shapes, same stratified sampling)
        t1 = time.perf_counter()
        pseed = TIMED_SEED + 1000 * rank
        random.seed(pseed)
        np.random.seed(pseed % 2**32)
        torch.manual_seed(pseed)
        kernel_timer.enable(True, max(1, args.timer_every))
        kernel_timer.calibrate()
        for i in range(n_pre):
            kernel_timer.new_step(True)
            one(args.warmup + i, cur)
            cur += args.batch * world
        sync()
        pre = kernel_timer.summary()
        kernel_timer.enable(False)
        target = kernel_timer.dominant_name(pre)
        prepass = (pre, args.steps / n_pre)
        _log(rank, f"timer pre-pass ({n_pre} steps, every region): {time.perf_counter() - t1:.1f}s; "
                   f"timed steps time {target}")
    # Long-lived objects (modules, optimiser state, autograd caches) leave the collector's
    # young generations: a full collection over them mid-step stalls the launch stream
    # for ~100 ms. training_loop.py does the same after its first iteration.
    gc.collect()
    if not args.no_gc_freeze:
        gc.freeze()
    sync()
    if world > 1:
        torch.distributed.barrier()
    sync()
    # equivariance outcomes drawn inside the timed region (+ VFM feature reuse per step), to price
    # the timed steps from the FLOP table (profiles/r2_flops.json; host-side bookkeeping only)
    draws, hits = [], []
    # the timed steps draw their equivariance outcomes (and noise) from a fixed seed, so runs with any
    # --warmup time the same sequence of outcomes. TIMED_SEED: the 20-step sequence whose priced work
    # (3.672 TFLOP/img, 15 feature-reuse steps) is the expectation of the stage-0 draw distribution
    # (3.672 TFLOP/img, 15.4 reuse steps per 20; simulated over 4e5 steps from profiles/r2_flops.json)
    seed = TIMED_SEED + 1000 * rank
    random.seed(seed)
    np.random.seed(seed % 2**32)
    torch.manual_seed(seed)
    eq_fwd = eqt.forward
    eqt.forward = lambda *a, **k: draws.append(eq_fwd(*a, **k)) or draws[-1]
    venc = step.G.vfm_encoder
    every = max(1, args.timer_every)
    kernel_timer.enable(on_gpu and not args.no_kernel_timer, every)
    calib_us = kernel_timer.calibrate() * 1e3 if (on_gpu and not args.no_kernel_timer) else None
    kernel_timer.set_target(target)
    t0 = time.perf_counter()
    tsteps = max(1, args.timer_steps)
    for i in range(args.steps):
        h0 = getattr(venc, "reuse_hits", 0)
        kernel_timer.new_step(i % tsteps == 0)
        one(args.warmup + i, cur)
        hits.append(getattr(venc, "reuse_hits", 0) - h0)
        cur += args.batch * world
        if args.trace:                      # diagnostics only: per-step wall time (synchronising)
            sync()
            _log(rank, f"step {i + 1}: {time.perf_counter() - t0:.3f}s cumulative")
    sync()
    if world > 1:
        torch.distributed.barrier()
    sync()
    dt = time.perf_counter() - t0
    kernel_timer.enable(False)
    eqt.forward = eq_fwd
    _log(rank, f"timed {args.steps} steps: {dt:.2f}s")
    if args.trace and on_gpu:
        ms = torch.cuda.memory_stats(device)
        _log(rank, "memory: peak alloc {:.1f} GB, reserved {:.1f} GB, alloc retries {}, device allocs {}, frees {}, "
             "gc counts {}".format(ms.get("allocated_bytes.all.peak", 0) / 2**30, ms.get("reserved_bytes.all.peak", 0) / 2**30,
                                   ms.get("num_alloc_retries", 0), ms.get("num_device_alloc", 0),
                                   ms.get("num_device_free", 0), gc.get_count()))
    if world > 1:
        t = torch.tensor([dt], device=device)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = dt / args.steps * 1e3
    value = args.batch * world * args.steps / dt

    traffic_table = None
    if os.path.exists(PMC_TRAFFIC):       # committed PMC passes of this workload (tools_dev/pmc_traffic.py)
        traffic_table = json.load(open(PMC_TRAFFIC)).get("kernels")
    roof = kernel_timer.dominant_roofline(HBM_PEAK_GBS, BF16_PEAK_TFLOPS, traffic_table, prepass=prepass) \
        if on_gpu else None
    if roof is not None:
        roof["traffic_source"] = os.path.relpath(PMC_TRAFFIC, ROOT) if roof.get("traffic") else None
        n_t = len(range(0, args.steps, tsteps))
        where = (f"all {args.steps} timed steps" if tsteps == 1 else
                 f"{n_t} of the {args.steps} timed steps (every {tsteps}th)")
        roof["timer_calibration_us"] = round(calib_us, 2) if calib_us is not None else None
        roof["timer_sampling"] = ((f"1/{every} of each kernel region's launches, stratified by launch position within "
                                   f"a step (position j of the k-th timed step when (j + k) % {every} == 0) in "
                                   if every > 1 else "every launch in ") + where + ", all launches counted"
                                  + (f"; only the roofline kernel's region is timed in the timed steps, the ranking, "
                                     f"runner_up and all_kernels come from {n_pre} untimed pre-pass steps drawing the "
                                     f"timed steps' seeded outcome sequence (every region, the same stratified 1/{every}) "
                                     f"with totals scaled to {args.steps} steps" if prepass is not None else ""))
    step_mfma = step_flops(draws, hits, args.batch, args.steps, value) if args.config == CONFIG else None
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            _log(rank, "cpu baseline ...")
            cpu = cpu_baseline(args.config, args.cpu_threads)
        except Exception as e:   # reported, never fatal for the GPU number
            cpu = {"error": repr(e)[:200]}
    if rank == 0:
        line = {
            "metric": "train images/sec @256^2 f16d32 (SigLIP2-L, stage-0 strong alignment)",
            "value": round(value, 3), "unit": "images/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic uint8 256x256x3 (seeded), random-init weights of the named architectures",
            "config": {"workload": "f16d32 SigLIP2-L stage-0 strong-alignment training iteration (D+G+sync+Adam+EMA)",
                       "model": "VFM-VAE f16d32 (SigLIP2-L @512 + ConvNeXt decoder + DINO ViT-S D + LPIPS-VGG16)",
                       "global_batch": args.batch * world, "batch_per_gpu": args.batch, "seq_len": 1024,
                       "resolution": 256, "parallelism": f"dp{world}",
                       "decoder_ops": "torch" if args.force_ref_ops else "hip",
                       "d_phase_g_forward": ("hip_graph" if (gr is not None and not gr.disabled and gr.graphs)
                                             else "eager"),
                       "precision": ("bf16 where the reference autocasts (SigLIP2 tower, decoder blocks 3-5); the "
                                     "reference's fp32 legs (decoder blocks 0-2, adapter, fp32 attention, LPIPS VGG16, "
                                     "DINO D) with fp32-equivalent products: " + _fp32_mode()),
                       "gemm_table": tunable["table"] if tunable and tunable["mode"] == "use" else None},
            "roofline": roof,
            "step_mfma": step_mfma,
            "cpu_baseline": cpu,
            # A/B switches set for this run (empty: every default, the tested product path)
            "env_knobs": {k: v for k, v in sorted(os.environ.items()) if k.startswith("VFM_")},
        }
        print(json.dumps(line), flush=True)
    if tunable and tunable["mode"] == "tune":
        _log(rank, f"tunableop table is written at exit: {tunable['out']}")
    if world > 1:
        torch.distributed.barrier()
        dist.destroy_process_group()


def smoke_step():
    """One tiny training iteration on cuda:0 through the native kernels (used by smoke())."""
    import copy
    import tempfile
    import dnnlib
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import net_cases
    from training.training_loop import TrainingIteration, make_optimizer
    from networks.generator import Generator
    from networks.discriminator import ProjectedDiscriminator
    from training.loss import TotalLoss
    dev = torch.device("cuda:0")
    d = os.path.join(tempfile.mkdtemp(), net_cases.VFM_DIRNAME)
    os.makedirs(d)
    json.dump(dict(net_cases.SIGLIP_CFG, layer_norm_eps=1e-6), open(os.path.join(d, "config.json"), "w"))
    torch.manual_seed(0)
    G = Generator(label_dim=0, **net_cases.g_kwargs(d)).train().requires_grad_(False).to(dev)
    D = ProjectedDiscriminator(c_dim=0, **net_cases.D_KWARGS).train().requires_grad_(False).to(dev)
    loss = TotalLoss(device=dev, G=G, D=D, **net_cases.loss_kwargs(d))
    opt = dict(class_name='torch.optim.Adam', lr=1e-4, betas=[0.0, 0.99], eps=1e-8)
    it = TrainingIteration(G, D, copy.deepcopy(G).eval(), loss, make_optimizer(G.parameters(), opt, dev),
                           make_optimizer(D.parameters(), opt, dev), batch_size=2)
    img = torch.rand(2, 3, 64, 64, device=dev)
    print("smoke: networks built, running the iteration", flush=True)
    it([img], [['x', 'x']], 0)
    torch.cuda.synchronize()
    for n, p in G.named_parameters():
        assert torch.isfinite(p).all(), n


if __name__ == "__main__":
    main()
