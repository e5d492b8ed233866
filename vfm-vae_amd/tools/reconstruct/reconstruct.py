"""Multi-GPU image reconstruction (rFID inputs/outputs) for VFM-VAE.

Drop-in for the reference `tools/reconstruct/reconstruct.py:85-162`: same CLI
(`--input-dir --output-dir --vae-pth --use-config --resolution --batch-size-per-gpu`), same
model overrides (`num_fp16_res = 0`, KL/VF off, unconditional), same outputs
(`<out>/inputs/<name>.png` = the resized/cropped real image, `<out>/outputs/<name>.png` = the
reconstruction mapped from [-1,1] to [0,1]), generator called as
`G(images, names, validation=True)` in fp32.

Launch: `torchrun --nproc-per-node N tools/reconstruct/reconstruct.py ...` (one process per
GPU; RCCL only for the closing barrier) or plain `python` for one process. Files are sorted and
dealt round-robin over ranks (the reference's DistributedSampler pads the last round with
repeats that overwrite the same files; the set of written files is identical).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import common  # noqa: E402


@torch.no_grad()
def run_rfid_reconstruction(vae, input_dir, output_dir, resolution, batch_size_per_gpu, rank: common.Rank,
                            log=print):
    in_dir = os.path.join(output_dir, "inputs")
    out_dir = os.path.join(output_dir, "outputs")
    os.makedirs(in_dir, exist_ok=True)
    os.makedirs(out_dir, exist_ok=True)
    names = rank.shard(common.list_images(input_dir))
    batches = [names[i:i + batch_size_per_gpu] for i in range(0, len(names), batch_size_per_gpu)]
    writer = common.Writer()
    loader = writer.pool

    def load(batch):
        return [common.load_image(os.path.join(input_dir, n), resolution) for n in batch]

    fut = loader.submit(load, batches[0]) if batches else None
    for bi, batch in enumerate(batches):
        arrays = fut.result()
        if bi + 1 < len(batches):                      # decode the next batch while this one runs
            fut = loader.submit(load, batches[bi + 1])
        images = common.batch_to_device(arrays, rank.device)
        out = vae(images, list(batch), validation=True)
        gen = out.gen_img.float().add(1).div(2)
        real_u8 = common.to_uint8(images).cpu().numpy()
        gen_u8 = common.to_uint8(gen).cpu().numpy()
        for i, name in enumerate(batch):
            base, _ = os.path.splitext(name)
            writer.put(real_u8[i], os.path.join(in_dir, f"{base}.png"))
            writer.put(gen_u8[i], os.path.join(out_dir, f"{base}.png"))
        log(f"[Rank {rank.rank}] Reconstruction {bi + 1}/{len(batches)}")
    writer.drain()
    return len(names)


def main(argv=None):
    import argparse
    p = argparse.ArgumentParser()
    p.add_argument('--input-dir', type=str, required=True, help='Path to input image folder')
    p.add_argument('--output-dir', type=str, required=True, help='Path to output folder')
    p.add_argument('--vae-pth', type=str, required=True, help='Path to VAE model (.pth)')
    p.add_argument('--use-config', type=str, required=True, help='Path to YAML config file')
    p.add_argument('--resolution', type=int, default=256, help='Input image resolution')
    p.add_argument('--batch-size-per-gpu', type=int, default=32, help='Batch size per GPU')
    p.add_argument('--device', type=str, default=None, help='override (default cuda:LOCAL_RANK, else cpu)')
    args = p.parse_args(argv)

    rank = common.Rank(args.device)
    vae = common.build_vae(args.use_config, args.resolution, rank.device)
    print(f"Loading checkpoint: {args.vae_pth}")
    common.load_vae_weights(vae, args.vae_pth, rank.device)
    n = run_rfid_reconstruction(vae, args.input_dir, args.output_dir, args.resolution,
                                args.batch_size_per_gpu, rank)
    rank.barrier()
    print(f"[Rank {rank.rank}] Done. Reconstructed {n} images.")
    rank.close()


if __name__ == "__main__":
    main()
