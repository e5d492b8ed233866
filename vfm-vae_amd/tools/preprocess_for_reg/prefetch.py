"""Image + latent extraction for REG / SiT-style diffusion training.

Drop-in for the reference `tools/preprocess_for_reg/prefetch.py:30-382`: same CLI
(`--data-path --output-dir --vae-pth --use-config --resolution --batch-size-per-gpu
--max-images-per-gpu --no-images --images-folder-name --vae-folder-name`; `generator_kwargs` or
`G_kwargs` in the YAML), same input pipeline (WebDataset shards, ADM centre crop; `tools/wds.py`),
same outputs:
  * `<vae>/<key.split('_')[0]>/<key>.npy` = float32 `[2·z, h, w]`: posterior mean ‖ std from
    `G.encode(x, return_z_before_quantize=True)` (mean ‖ logvar → logvar clamped to [-30, 20],
    std = exp(logvar / 2));
  * `<images>/<subfolder>/<key>.png` (unless `--no-images`);
  * per-rank `dataset_rank{r}.json` (`{"labels": [["sub/key.ext", label], ...]}` in the
    reference's quote-fixed text form), merged into `dataset.json` on rank 0;
  * `<vae>/latents_stats.pt` = per-channel mean/std over ≤ 10 000 sampled latents
    (mean + std·ε) on rank 0.
"""
import json
import os
import random
import sys
from glob import glob

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import common  # noqa: E402
from wds import iter_batches  # noqa: E402


def mean_logvar_to_mean_std(moments):
    mean, logvar = torch.chunk(moments, 2, dim=1)
    logvar = torch.clamp(logvar, -30.0, 20.0)
    return torch.cat([mean, torch.exp(0.5 * logvar)], dim=1)


def save_json(records, path):
    with open(path, "w") as f:
        f.write('{"labels": [\n')
        for i, (name, label) in enumerate(records):
            f.write(f'  ["{name}", {label}]' + (",\n" if i < len(records) - 1 else "\n"))
        f.write("]}\n")


def _save_npy(feat, path):
    np.save(path, feat.astype(np.float32))


def compute_vae_stats_sampled(vae_dir, num_samples=10000, log=print):
    files = [os.path.join(r, f) for r, _, fs in os.walk(vae_dir) for f in fs if f.endswith(".npy")]
    if not files:
        log(f"[WARN] No latent files found in {vae_dir}")
        return
    feats = []
    for fp in random.sample(files, min(num_samples, len(files))):
        z = torch.from_numpy(np.load(fp))
        mean, std = torch.chunk(z, 2, dim=0)
        feats.append((mean + std * torch.randn_like(mean)).unsqueeze(0))
    feats = torch.cat(feats, 0)
    torch.save({"mean": feats.mean(dim=[0, 2, 3], keepdim=True), "std": feats.std(dim=[0, 2, 3], keepdim=True)},
               os.path.join(vae_dir, "latents_stats.pt"))
    log(f"Saved VAE stats to {vae_dir}/latents_stats.pt")


@torch.no_grad()
def run_extraction(vae, data_path, output_dir, rank: common.Rank, resolution, batch_size_per_gpu,
                   process_images=True, images_folder_name="images_png", vae_folder_name="vae_latents",
                   max_images_per_gpu=None, log=print):
    images_dir = os.path.join(output_dir, images_folder_name)
    vae_dir = os.path.join(output_dir, vae_folder_name)
    os.makedirs(images_dir, exist_ok=True)
    os.makedirs(vae_dir, exist_ok=True)
    urls = sorted(glob(os.path.join(data_path, "*.tar"))) if os.path.isdir(data_path) else [data_path]
    log(f"Rank {rank.rank}: Found {len(urls)} shards")
    writer = common.Writer()
    rec_img, rec_lat = [], []
    total = 0
    for arr, labels, keys in iter_batches(urls, resolution, batch_size_per_gpu, rank.rank, rank.world_size, log):
        if max_images_per_gpu:
            remain = max_images_per_gpu - total
            if remain <= 0:
                break
            arr, labels, keys = arr[:remain], labels[:remain], keys[:remain]
        x = common.batch_to_device(list(arr), rank.device)
        lat = mean_logvar_to_mean_std(vae.encode(x, return_z_before_quantize=True).float()).cpu().numpy()
        for i, (key, label) in enumerate(zip(keys, labels)):
            sub = key.split("_")[0]
            if process_images:
                os.makedirs(os.path.join(images_dir, sub), exist_ok=True)
                writer.put(arr[i], os.path.join(images_dir, sub, f"{key}.png"))
                rec_img.append((f"{sub}/{key}.png", int(label)))
            os.makedirs(os.path.join(vae_dir, sub), exist_ok=True)
            writer.pending.append(writer.pool.submit(_save_npy, lat[i], os.path.join(vae_dir, sub, f"{key}.npy")))
            rec_lat.append((f"{sub}/{key}.npy", int(label)))
        total += len(labels)
    writer.drain()
    save_json(rec_lat, os.path.join(vae_dir, f"dataset_rank{rank.rank}.json"))
    if process_images:
        save_json(rec_img, os.path.join(images_dir, f"dataset_rank{rank.rank}.json"))
    rank.barrier()
    if rank.rank == 0:
        def merge(folder):
            recs = []
            for f in sorted(os.listdir(folder)):
                if f.startswith("dataset_rank") and f.endswith(".json"):
                    with open(os.path.join(folder, f)) as jf:
                        recs.extend(json.load(jf).get("labels", []))
            save_json(recs, os.path.join(folder, "dataset.json"))
        merge(vae_dir)
        if process_images:
            merge(images_dir)
        compute_vae_stats_sampled(vae_dir, log=log)
    return total


def main(argv=None):
    import argparse
    p = argparse.ArgumentParser(description="Extract images and VAE latents using WebDataset (.pth)")
    p.add_argument("--data-path", type=str, required=True, help="Path to WebDataset .tar files or folder")
    p.add_argument("--output-dir", type=str, required=True, help="Output directory for extracted data")
    p.add_argument("--vae-pth", type=str, required=True, help="Path to pretrained VAE checkpoint (.pth)")
    p.add_argument("--use-config", type=str, required=True, help="Path to YAML config defining model")
    p.add_argument("--resolution", type=int, default=256)
    p.add_argument("--batch-size-per-gpu", type=int, default=64)
    p.add_argument("--max-images-per-gpu", type=int, default=None)
    p.add_argument("--no-images", action="store_true", help="Skip PNG saving")
    p.add_argument("--images-folder-name", type=str, default="images")
    p.add_argument("--vae-folder-name", type=str, default="vae_latents")
    p.add_argument('--device', type=str, default=None, help='override (default cuda:LOCAL_RANK, else cpu)')
    args = p.parse_args(argv)

    rank = common.Rank(args.device)
    print(f"[Init] Rank {rank.rank}/{rank.world_size} ready on device {rank.device}.")
    vae = common.build_vae(args.use_config, args.resolution, rank.device, keys=("generator_kwargs", "G_kwargs"))
    print(f"[Rank {rank.rank}] Loading checkpoint: {args.vae_pth}")
    common.load_vae_weights(vae, args.vae_pth, rank.device)
    total = run_extraction(vae, args.data_path, args.output_dir, rank, args.resolution, args.batch_size_per_gpu,
                           process_images=not args.no_images, images_folder_name=args.images_folder_name,
                           vae_folder_name=args.vae_folder_name, max_images_per_gpu=args.max_images_per_gpu)
    print(f"[Rank {rank.rank}] Processed {total} samples.")
    rank.close()


if __name__ == "__main__":
    main()
