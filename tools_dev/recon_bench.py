"""Reconstruction-tool throughput at the full f16d32 SigLIP2-L config on one GPU: random-init
G_ema snapshot, N synthetic PNGs (non-square, so the Resize/CenterCrop path runs), the tool's
own loop (decode → G(x, validation=True) → uint8 → PNG), then evaluate.py on the pairs.
  python tools_dev/recon_bench.py [--n 256] [--batch 32]"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vfm-vae_amd", "tools"))
sys.path.insert(0, os.path.join(ROOT, "vfm-vae_amd", "tools", "reconstruct"))
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")

import numpy as np  # noqa: E402
import torch  # noqa: E402

import common  # noqa: E402

CFG = os.path.join(ROOT, "vfm-vae_amd", "configs", "vfm_vae_f16d32_siglip2_stage_0_strong_alignment.yaml")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    from PIL import Image
    import reconstruct
    import evaluate
    tmp = tempfile.mkdtemp(dir="/tmp")
    src = os.path.join(tmp, "src")
    os.makedirs(src)
    rng = np.random.default_rng(0)
    for i in range(a.n):
        Image.fromarray(rng.integers(0, 256, (300, 280, 3), dtype=np.uint8)).save(os.path.join(src, f"{i:05d}.png"))
    print(f"wrote {a.n} images", flush=True)
    rank = common.Rank()
    torch.manual_seed(0)
    G = common.build_vae(CFG, 256, rank.device)
    ck = os.path.join(tmp, "snap.pth")
    torch.save({"G_ema": G.state_dict()}, ck)
    G = common.build_vae(CFG, 256, rank.device)
    common.load_vae_weights(G, ck, rank.device)
    print("model ready", flush=True)
    out = os.path.join(tmp, "rec")
    # warm-up pass over one batch (kernel loads), then the timed pass over all images
    reconstruct.run_rfid_reconstruction(G, src, os.path.join(tmp, "warm"), 256, a.batch, rank, log=lambda *x: None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = reconstruct.run_rfid_reconstruction(G, src, out, 256, a.batch, rank, log=lambda *x: None)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res = evaluate.evaluate_image_metrics(os.path.join(out, "inputs"), os.path.join(out, "outputs"), batch_size=64,
                                          num_workers=8, log=lambda *x: None)
    print(json.dumps({"tool": "reconstruct", "images": n, "batch": a.batch, "seconds": round(dt, 3),
                      "images_per_s": round(n / dt, 2), "eval": res,
                      "note": "random-init weights: metrics show the plumbing, not reconstruction quality"}),
          flush=True)


if __name__ == "__main__":
    main()
