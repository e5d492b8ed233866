"""LPIPS / PSNR / SSIM between paired image folders (reconstruction quality).

Drop-in for the reference `tools/reconstruct/evaluate.py:22-139`: same CLI
(`--ref-dir --pred-dir --batch-size --num-workers`), pairs = the sorted intersection of the
two folders' file names, images mapped to [-1, 1], and the same reductions:
  * LPIPS (`training.lpips.LPIPS`): batch mean, weighted by batch size;
  * SSIM: torchmetrics `StructuralSimilarityIndexMeasure(data_range=2)` restated in
    `training.loss.SSIM` (11×11 Gaussian σ=1.5, reflect pad, border cropped), batch mean;
  * PSNR: per image `10·log10(2² / mse)` (torchmetrics `PeakSignalNoiseRatio(data_range=2)`
    called one image at a time, as the reference does), averaged.
torchmetrics is not installed here, so SSIM/PSNR parity rests on the restatement (unpinned).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import common  # noqa: E402


def psnr_per_image(pred, ref, data_range=2.0):
    mse = (pred.double() - ref.double()).pow(2).flatten(1).mean(1)
    return 10.0 * torch.log10(data_range ** 2 / mse)


@torch.no_grad()
def evaluate_image_metrics(ref_dir, pred_dir, batch_size=64, num_workers=8, device=None, log=print):
    from training.lpips import LPIPS
    from training.loss import SSIM
    device = torch.device(device or ("cuda:0" if torch.cuda.is_available() else "cpu"))
    log(f"Using device: {device}")
    names = sorted(set(os.listdir(ref_dir)) & set(os.listdir(pred_dir)))
    if not names:
        raise ValueError(f"No overlapping files found between {ref_dir} and {pred_dir}")
    lpips_metric = LPIPS().to(device).eval()
    ssim_metric = SSIM(data_range=2.0)
    pool = common.Writer(workers=max(1, num_workers)).pool

    def load(batch):
        ref = [common.load_png_uint8(os.path.join(ref_dir, n)) for n in batch]
        prd = [common.load_png_uint8(os.path.join(pred_dir, n)) for n in batch]
        return ref, prd

    batches = [names[i:i + batch_size] for i in range(0, len(names), batch_size)]
    lp_sum = ps_sum = ss_sum = 0.0
    total = 0
    fut = pool.submit(load, batches[0])
    for bi in range(len(batches)):
        ref_a, prd_a = fut.result()
        if bi + 1 < len(batches):
            fut = pool.submit(load, batches[bi + 1])
        ref = common.batch_to_device(ref_a, device).sub_(0.5).div_(0.5)
        prd = common.batch_to_device(prd_a, device).sub_(0.5).div_(0.5)
        bs = ref.shape[0]
        lp = lpips_metric(prd, ref).mean()
        ss = ssim_metric(prd, ref)
        pn = psnr_per_image(prd, ref).mean()
        lp_sum += float(lp) * bs
        ss_sum += float(ss) * bs
        ps_sum += float(pn) * bs
        total += bs
    pool.shutdown(wait=True)
    res = {"total": total, "lpips": lp_sum / total, "psnr": ps_sum / total, "ssim": ss_sum / total}
    log("\n===== Evaluation Results =====")
    log(f"Total Images : {total}")
    log(f"Average LPIPS: {res['lpips']:.4f}")
    log(f"Average PSNR : {res['psnr']:.4f}")
    log(f"Average SSIM : {res['ssim']:.4f}")
    return res


if __name__ == "__main__":
    import argparse
    p = argparse.ArgumentParser(description="Evaluate LPIPS / PSNR / SSIM between image pairs.")
    p.add_argument("--ref-dir", type=str, required=True, help="Path to reference images.")
    p.add_argument("--pred-dir", type=str, required=True, help="Path to predicted images.")
    p.add_argument("--batch-size", type=int, default=64, help="Batch size for GPU inference.")
    p.add_argument("--num-workers", type=int, default=8, help="Number of loader threads.")
    a = p.parse_args()
    evaluate_image_metrics(a.ref_dir, a.pred_dir, batch_size=a.batch_size, num_workers=a.num_workers)
