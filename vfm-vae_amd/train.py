"""Train VFM-VAE from a YAML config (reference train.py:55-206 surface).

  torchrun --nproc_per_node=8 train.py --config configs/vfm_vae_f16d32_siglip2_stage_0_strong_alignment.yaml

Same YAML keys, the same kwarg inheritance between sections, the same batch
split (batch_gpu = batch_size / (world * accumulate_gradients)) and auto-resume
from the newest `network-snapshot-*.pth` in run_dir.
"""
import argparse
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch
import yaml

import dnnlib
from torch_utils import distributed as dist
from training import training_loop


def to_easydict(d):
    if isinstance(d, dict):
        return dnnlib.EasyDict({k: to_easydict(v) for k, v in d.items()})
    if isinstance(d, list):
        return [to_easydict(v) for v in d]
    return d


def find_latest_network_snapshot(run_dir):
    snaps = glob.glob(os.path.join(run_dir, "network-snapshot-*.pth"))
    if not snaps:
        return None
    def kimg(p):
        m = re.search(r"network-snapshot-(\d+)\.pth$", p)
        return int(m.group(1)) if m else -1
    return max(snaps, key=kimg)


def resolve_config(cfg):
    """Apply the reference's kwarg inheritance rules (train.py:66-114)."""
    c = to_easydict(cfg)
    c.setdefault("one_epoch", c.training_set_kwargs.get("one_epoch", False))
    c.setdefault("resume_kimg", 0)
    c.setdefault("resume_path", None)
    G, L, T = c.G_kwargs, c.get("loss_kwargs", dnnlib.EasyDict()), c.training_set_kwargs
    if "resolution" not in G and "resolution" in T:
        G.img_resolution = T.get("resolution")
    if "conditional" not in G and "conditional" in T:
        G.conditional = T.get("conditional", False)
    if "label_type" not in G and "label_type" in T:
        G.label_type = T.get("label_type")
    if "use_kl_loss" not in G and "kl_loss_weight" in L:
        G.use_kl_loss = L.get("kl_loss_weight", 0.0) > 0.0
    if "use_vf_loss" not in G and "vf_loss_weight" in L:
        G.use_vf_loss = L.get("vf_loss_weight", 0.0) > 0.0
    if "use_adaptive_vf_loss" not in G and "use_adaptive_vf_loss" in L:
        G.use_adaptive_vf_loss = L.get("use_adaptive_vf_loss", False)
    if "use_equivariance_regularization" not in G and "use_equivariance_regularization" in L:
        G.use_equivariance_regularization = L.get("use_equivariance_regularization", False)
    if "use_multiscale_output" not in G and "multiscale_block_indices" in L:
        G.use_multiscale_output = len(L.get("multiscale_block_indices", [])) > 0
    if "D_kwargs" in c and "vfm_name" not in c.D_kwargs:
        c.D_kwargs.vfm_name = G.get("vfm_name")
    if "loss_kwargs" in c:
        L.setdefault("vfm_name", G.get("vfm_name"))
        if "compression_mode" not in L and "compression_mode" in G:
            L.compression_mode = G.get("compression_mode")
        L.setdefault("resume_kimg", c.get("resume_kimg", 0))
    return c


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True)
    args = ap.parse_args(argv)
    cfg = yaml.safe_load(open(args.config))
    c = resolve_config(cfg)
    dist.init()
    world = dist.get_world_size()
    c.setdefault("accumulate_gradients", 1)
    assert c.batch_size % (world * c.accumulate_gradients) == 0
    c.batch_gpu = c.batch_size // (world * c.accumulate_gradients)
    torch.manual_seed(c.get("random_seed", 42))
    if c.resume_path is None:
        snap = find_latest_network_snapshot(c.run_dir)
        if snap and os.path.getsize(snap) > 1000:
            c.resume_path = snap
            c.resume_kimg = int(re.search(r"(\d+)\.pth$", snap).group(1))
    c.train_sample_dir = os.path.join(c.run_dir, "train_samples")
    if dist.get_rank() == 0:
        os.makedirs(c.run_dir, exist_ok=True)
        os.makedirs(c.train_sample_dir, exist_ok=True)
        with open(os.path.join(c.run_dir, "training_config.yaml"), "w") as f:
            yaml.safe_dump(cfg, f, sort_keys=False)
        dnnlib.util.Logger(file_name=os.path.join(c.run_dir, "log.txt"), file_mode="a", should_flush=True)
        print(json.dumps(cfg, indent=2))
    if torch.distributed.is_initialized():
        torch.distributed.barrier()
    training_loop.training_loop(**c)


if __name__ == "__main__":
    main()
