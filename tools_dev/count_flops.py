"""Matrix-work FLOPs of one bench.py training iteration, per image, per equivariance outcome.

  python tools_dev/count_flops.py [--batch 2] [--out profiles/r2_flops.json]

Runs the bench configuration's D and G phases on the CPU (torch formulation of every op)
under torch.utils.flop_counter.FlopCounterMode, one forced equivariance variant at a time:

  D[v]            D phase whose no-grad generator forward drew variant v
  G[v][reuse]     G phase drawing v, with (reuse=1) or without (reuse=0) the VFM tower
                  features handed over from the D phase (networks/utils/vfm_utils.py)

FLOPs counted: every GEMM, batched GEMM, convolution (forward and both backward products)
and attention product (QK^T, PV and their gradients), i.e. the work that maps onto MFMA.
Elementwise / normalisation work is not counted. bench.py sums these entries over the
outcomes its timed steps actually drew, so `step_mfma.frac` is reproducible from this file.
The counts are linear in the batch; the table stores FLOPs per image.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vfm-vae_amd"), ROOT]

import torch  # noqa: E402
from torch.utils import flop_counter as fc  # noqa: E402


def _register_cpu_attention():
    ops = torch.ops.aten
    if ops._scaled_dot_product_flash_attention_for_cpu not in fc.flop_registry:
        fc.register_flop_formula(ops._scaled_dot_product_flash_attention_for_cpu, get_raw=False)(
            lambda q, k, v, *a, out_shape=None, **kw: fc.sdpa_flop_count(q, k, v))
        fc.register_flop_formula(ops._scaled_dot_product_flash_attention_for_cpu_backward, get_raw=False)(
            lambda go, q, k, v, *a, out_shape=None, **kw: fc.sdpa_backward_flop_count(go, q, k, v))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r2_flops.json"))
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    _register_cpu_attention()
    import bench
    dev = torch.device("cpu")
    c, step = bench.build(bench.CONFIG, args.batch, dev, 1, graphs=False)
    eqt = step.G.equivariance_transform
    enc = step.G.vfm_encoder
    from training.data_synthetic import SyntheticDataset
    pool = SyntheticDataset(resolution=c.training_set_kwargs.resolution, seed=0).make_pool(args.batch, dev)
    labels = ['a photo'] * args.batch
    D_phase, G_phase = step.phases
    draws = []
    orig_fwd = eqt.forward

    def logged(validation):
        out = orig_fwd(validation)
        draws.append(out)
        return out

    eqt.forward = logged

    def count(phase, img, cur):
        draws.clear()
        with fc.FlopCounterMode(display=False) as m:
            step.run_phase(phase, [img], [labels], cur)
        assert len(draws) == 1, f"{phase.name} phase drew {len(draws)} equivariance outcomes"
        return m.get_total_flops() / args.batch

    table = {"D": {}, "G": {}}
    cur = 0
    for v in eqt.variants():
        key = f"{v[0]},{int(v[2])}"
        t0 = time.time()
        img = pool[0].float() / 255.
        eqt.forced = v
        table["D"][key] = count(D_phase, img, cur)
        # G phase without reuse (features dropped), then with the D phase's features
        enc.clear_features()
        table["G"][key] = {"0": count(G_phase, img, cur)}
        img = pool[1 % len(pool)].float() / 255.
        step.run_phase(D_phase, [img], [labels], cur)
        hits = getattr(enc, "reuse_hits", 0)
        g1 = count(G_phase, img, cur)
        table["G"][key]["1"] = g1 if getattr(enc, "reuse_hits", 0) == hits + 1 else None
        eqt.forced = None
        print(f"variant {key}: D {table['D'][key] / 1e12:.3f} TF/img, G {table['G'][key]['0'] / 1e12:.3f} / "
              f"{(g1 / 1e12):.3f} (reuse) TF/img  [{time.time() - t0:.0f}s]", flush=True)
    res = {"what": "matrix-work FLOPs per image of one training iteration (tools_dev/count_flops.py)",
           "config": os.path.relpath(bench.CONFIG, ROOT), "batch_counted": args.batch,
           "key": "'<eq_scale>,<is_eq_prior>' of the phase's equivariance draw; G[key][reuse]",
           "D": table["D"], "G": table["G"]}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
