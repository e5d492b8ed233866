"""Latent prefetch for downstream diffusion training (LightningDiT layout).

Drop-in for the reference `tools/preprocess_for_lightningdit/prefetch.py:31-349`: same CLI
(`--data-path --output-dir --vae-pth --use-config --resolution --batch-size-per-gpu
--max-images-per-gpu`), same input (WebDataset tar shards with `jpg`/`png` + `cls` members),
same ADM preprocessing (`center_crop_imagenet`: BOX halving while ≥ 2× the size, BICUBIC to the
short side, integer-floor centre crop), same encoder call (`G.encode(x)` and `G.encode(flip(x))`
in fp32), and the same output: `latents_rank{RR}_shard{NNN}.safetensors` with `latents`,
`latents_flip` (float32 `[n, 32, 16, 16]`) and `labels` (int64), flushed every ≥ 10 000 samples,
plus `latents_stats.pt` (`{'mean','std'}` over ≤ 10 000 random latents, per channel) written by
`ImgLatentDataset` on rank 0.

webdataset is not installed here: `tools/wds.py` restates the part of its pipeline the
reference uses.
"""
import os
import sys
from glob import glob

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import common  # noqa: E402
from wds import center_crop_imagenet, iter_batches  # noqa: E402,F401

SHARD_SAMPLES = 10000


# ------------------------------------------------------------------ latents dataset

class ImgLatentDataset(torch.utils.data.Dataset):
    """Reads the prefetched shards; `latent_norm` standardises with the cached stats
    (reference `prefetch.py:31-103`)."""

    def __init__(self, data_dir, latent_norm=True, latent_multiplier=1.0, log=print):
        from safetensors import safe_open
        self._open = safe_open
        self.data_dir = data_dir
        self.latent_norm = latent_norm
        self.latent_multiplier = latent_multiplier
        self.files = sorted(glob(os.path.join(data_dir, "*.safetensors")))
        self.index = []                                  # (file, idx_in_file)
        for fn in self.files:
            with safe_open(fn, framework="pt", device="cpu") as f:
                n = f.get_slice("labels").get_shape()[0]
            self.index.extend((fn, i) for i in range(n))
        log(f"[ImgLatentDataset] Found {len(self.index)} images across {len(self.files)} files in {data_dir}")
        if latent_norm:
            self._latent_mean, self._latent_std = self.get_latent_stats()

    def get_latent_stats(self):
        path = os.path.join(self.data_dir, "latents_stats.pt")
        if not os.path.exists(path):
            stats = self.compute_latent_stats()
            torch.save(stats, path)
        else:
            stats = torch.load(path, weights_only=True)
        return stats["mean"], stats["std"]

    def compute_latent_stats(self):
        n = min(SHARD_SAMPLES, len(self.index))
        picks = np.random.choice(len(self.index), n, replace=False)
        by_file = {}
        for j in picks:
            fn, i = self.index[j]
            by_file.setdefault(fn, []).append(i)
        lat = []
        for fn, rows in by_file.items():                  # one open per file, not per sample
            with self._open(fn, framework="pt", device="cpu") as f:
                t = f.get_tensor("latents")
            lat.append(t[torch.tensor(rows)])
        lat = torch.cat(lat, 0)
        return {"mean": lat.mean(dim=[0, 2, 3], keepdim=True), "std": lat.std(dim=[0, 2, 3], keepdim=True)}

    def __len__(self):
        return len(self.index)

    def __getitem__(self, idx):
        fn, i = self.index[idx]
        with self._open(fn, framework="pt", device="cpu") as f:
            key = "latents" if np.random.uniform(0, 1) > 0.5 else "latents_flip"
            feat = f.get_slice(key)[i:i + 1]
            label = f.get_slice("labels")[i:i + 1]
        if self.latent_norm:
            feat = (feat - self._latent_mean) / self._latent_std
        feat = feat * self.latent_multiplier
        return feat.squeeze(0), label.squeeze(0)


# ------------------------------------------------------------------ extraction

def _save(output_dir, rank, shard, lat, lat_f, lab, log):
    from safetensors.torch import save_file
    path = os.path.join(output_dir, f"latents_rank{rank:02d}_shard{shard:03d}.safetensors")
    save_file({"latents": torch.cat(lat).contiguous(), "latents_flip": torch.cat(lat_f).contiguous(),
               "labels": torch.cat(lab).contiguous()}, path)
    if rank == 0:
        log(f"Saved {path}")


@torch.no_grad()
def run_latent_extraction_wds(vae, data_path, output_dir, rank: common.Rank, resolution, batch_size_per_gpu,
                              max_images_per_gpu=None, log=print):
    os.makedirs(output_dir, exist_ok=True)
    urls = sorted(glob(os.path.join(data_path, "*.tar"))) if os.path.isdir(data_path) else [data_path]
    log(f"Rank {rank.rank}: Found {len(urls)} tar files")
    lat, lat_f, lab = [], [], []
    saved, seen = 0, 0
    for arr, labels, _ in iter_batches(urls, resolution, batch_size_per_gpu, rank.rank, rank.world_size, log):
        if max_images_per_gpu is not None:
            remain = max_images_per_gpu - seen
            if remain <= 0:
                break
            arr, labels = arr[:remain], labels[:remain]
        x = common.batch_to_device(list(arr), rank.device)
        z1 = vae.encode(x)
        z2 = vae.encode(torch.flip(x, dims=[-1]))
        lat.append(z1.float().cpu())
        lat_f.append(z2.float().cpu())
        lab.append(torch.tensor(labels, dtype=torch.long))
        seen += x.shape[0]
        if sum(t.shape[0] for t in lat) >= SHARD_SAMPLES:
            _save(output_dir, rank.rank, saved, lat, lat_f, lab, log)
            lat, lat_f, lab = [], [], []
            saved += 1
    if lat:
        _save(output_dir, rank.rank, saved, lat, lat_f, lab, log)
    rank.barrier()
    return seen


def main(argv=None):
    import argparse
    p = argparse.ArgumentParser()
    p.add_argument('--data-path', type=str, required=True, help='Path to WebDataset tar files')
    p.add_argument('--output-dir', type=str, required=True, help='Directory to save extracted latents')
    p.add_argument('--vae-pth', type=str, required=True, help='Path to the VAE checkpoint (.pth)')
    p.add_argument('--use-config', type=str, required=True, help='Path to YAML config')
    p.add_argument('--resolution', type=int, default=256, help='Image resolution for preprocessing')
    p.add_argument('--batch-size-per-gpu', type=int, default=64, help='Batch size per GPU')
    p.add_argument('--max-images-per-gpu', type=int, default=None, help='Optional image limit per GPU')
    p.add_argument('--device', type=str, default=None, help='override (default cuda:LOCAL_RANK, else cpu)')
    args = p.parse_args(argv)

    rank = common.Rank(args.device)
    print(f"Rank {rank.rank} of {rank.world_size} initialized.")
    vae = common.build_vae(args.use_config, args.resolution, rank.device)
    print(f"Loading checkpoint: {args.vae_pth}")
    common.load_vae_weights(vae, args.vae_pth, rank.device)
    n = run_latent_extraction_wds(vae, args.data_path, args.output_dir, rank, args.resolution,
                                  args.batch_size_per_gpu, args.max_images_per_gpu)
    print(f"Rank {rank.rank} processed {n} images.")
    if rank.rank == 0:
        ImgLatentDataset(args.output_dir, latent_norm=True)
        print("Latent stats saved at", os.path.join(args.output_dir, "latents_stats.pt"))
    rank.close()


if __name__ == "__main__":
    main()
