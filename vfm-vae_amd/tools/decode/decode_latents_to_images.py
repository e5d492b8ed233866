"""Multi-GPU image decoding of `.safetensors` latents with a VFM-VAE checkpoint.

Drop-in for the reference `tools/decode/decode_latents_to_images.py:27-183`: same CLI
(`--input-dir --output-dir --vae-pth --use-config --batch-size-per-gpu --max-images-per-gpu`),
same file split (`sorted(*.safetensors)[rank::world_size]`), keys `latents` (required) and
`labels` (optional; one-hot for a `cls2id` conditional decoder), `G.decode(z, c)` in fp32,
images written as `rank{RR}_{index:06d}.png` with the per-rank running index, and the
reference's skip-and-warn on unreadable files or files without `latents`.

MI355X design: one process per GPU, the file's latents moved to HBM once, decoded in
micro-batches, quantised to uint8 on the device, PNGs encoded on a thread pool.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import common  # noqa: E402


@torch.no_grad()
def run_latent_decoding(vae, input_dir, output_dir, batch_size_per_gpu, rank: common.Rank,
                        max_images_per_gpu=None, log=print):
    from safetensors.torch import load_file
    os.makedirs(output_dir, exist_ok=True)
    all_files = sorted(f for f in os.listdir(input_dir) if f.endswith(".safetensors"))
    assert all_files, f"No .safetensors files found in {input_dir}"
    files = rank.shard(all_files)
    log(f"[Rank {rank.rank}] Processing {len(files)} of {len(all_files)} files...")
    dev = rank.device
    writer = common.Writer()
    global_index = 0
    saved = 0
    for file in files:
        if max_images_per_gpu is not None and saved >= max_images_per_gpu:
            break
        try:
            data = load_file(os.path.join(input_dir, file))
        except Exception as e:  # reference: warn and skip
            log(f"Failed to load {file}: {e}")
            continue
        if "latents" not in data:
            log(f"Missing 'latents' in {file}")
            continue
        latents = data["latents"].to(dev)
        labels = data["labels"].to(dev) if "labels" in data else torch.zeros(latents.size(0), device=dev)
        if getattr(vae, "conditional", False) and getattr(vae, "label_type", None) == "cls2id":
            labels = F.one_hot(labels.long(), num_classes=vae.c_dim).float()
        for start in range(0, latents.size(0), batch_size_per_gpu):
            if max_images_per_gpu is not None and saved >= max_images_per_gpu:
                break
            end = min(start + batch_size_per_gpu, latents.size(0))
            images = vae.decode(latents[start:end].float(), labels[start:end])
            u8 = common.to_uint8(((images.float() + 1) / 2)).cpu().numpy()
            for i in range(u8.shape[0]):
                if max_images_per_gpu is not None and saved >= max_images_per_gpu:
                    break
                writer.put(u8[i], os.path.join(output_dir, f"rank{rank.rank:02d}_{global_index + i:06d}.png"))
                saved += 1
            global_index += u8.shape[0]
    writer.drain()
    rank.barrier()
    log(f"[Rank {rank.rank}] Done. Saved {saved} images.")
    return saved


def main(argv=None):
    import argparse
    p = argparse.ArgumentParser(description="Decode latent .safetensors files using .pth VAE model weights.")
    p.add_argument("--input-dir", type=str, required=True, help="Directory containing .safetensors latent files.")
    p.add_argument("--output-dir", type=str, required=True, help="Directory to save decoded images.")
    p.add_argument("--vae-pth", type=str, required=True, help="Path to pretrained VAE checkpoint (.pth).")
    p.add_argument("--use-config", type=str, required=True, help="Path to model config (YAML).")
    p.add_argument("--batch-size-per-gpu", type=int, default=32, help="Batch size per GPU for decoding.")
    p.add_argument("--max-images-per-gpu", type=int, default=None, help="Maximum number of images to decode per GPU.")
    p.add_argument('--device', type=str, default=None, help='override (default cuda:LOCAL_RANK, else cpu)')
    args = p.parse_args(argv)

    rank = common.Rank(args.device)
    vae = common.build_vae(args.use_config, 256, rank.device)
    print(f"Loading checkpoint: {args.vae_pth}")
    inc = common.load_vae_weights(vae, args.vae_pth, rank.device)
    common.report_incompatible_keys("vae", inc)
    run_latent_decoding(vae, args.input_dir, args.output_dir, args.batch_size_per_gpu, rank,
                        max_images_per_gpu=args.max_images_per_gpu)
    rank.close()


if __name__ == "__main__":
    main()
