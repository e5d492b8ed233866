"""Real-data path on the GPU: the training iteration fed by training/data_wds.py WdsWrapper from
WebDataset tar shards of JPEG images (ImageNet-like sizes, written here: no dataset download),
against the same iteration fed from a resident synthetic pool, in one process (reference
training/data_wds.py:235-353 + training/training_loop.py fetch / preprocess). Reports the data
path's own decode rate and the share of each step the loop waited for a batch."""
import io
import os
import sys
import tarfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vfm-vae_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def make_shards(root, n_shards=16, per_shard=64, seed=0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    os.makedirs(root, exist_ok=True)
    for s in range(n_shards):
        with tarfile.open(os.path.join(root, f"{s:05d}.tar"), "w") as tf:
            for i in range(per_shard):
                w, h = int(rng.integers(400, 640)), int(rng.integers(300, 480))
                # smooth random field + noise: JPEG sizes / decode cost like natural images
                base = rng.random((h // 16 + 1, w // 16 + 1, 3)) * 255
                img = np.kron(base, np.ones((16, 16, 1)))[:h, :w] + rng.normal(0, 12, (h, w, 3))
                buf = io.BytesIO()
                Image.fromarray(np.clip(img, 0, 255).astype(np.uint8)).save(buf, format="JPEG", quality=90)
                for ext, data in (("jpg", buf.getvalue()), ("cls", str(int(rng.integers(0, 1000))).encode())):
                    ti = tarfile.TarInfo(f"s{s:03d}_{i:04d}.{ext}")
                    ti.size = len(data)
                    tf.addfile(ti, io.BytesIO(data))


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    root = "/tmp/wds_bench"
    t0 = time.time()
    make_shards(root)
    print(f"shards written in {time.time() - t0:.1f}s", flush=True)
    from training.data_wds import WdsWrapper
    from training.training_loop import fetch_data
    B = 32
    workers = int(os.environ.get("WDS_WORKERS", "12"))
    ds = WdsWrapper(root, 256, label_type="cls2text", workers=workers, sample_shuffle_size=256)
    it = iter(ds.iterate(batch_size=B, seed=0))
    next(it)
    t0 = time.time()
    for _ in range(8):
        next(it)
    print(f"data path alone: {8 * B / (time.time() - t0):.1f} img/s ({workers} decode {'processes' if ds.processes else 'threads'})", flush=True)

    c, step = bench.build(bench.CONFIG, B, dev, 1)
    from training.data_synthetic import SyntheticDataset
    pool = SyntheticDataset(resolution=c.training_set_kwargs.resolution, seed=0).make_pool(B, dev)
    labels = ['a photo'] * B
    nimg = 0
    for i in range(3):                           # warm-up (all shapes), resident pool
        step([pool[i % len(pool)].float() / 255.], [labels], nimg)
        nimg += B
    for mode in ("resident", "wds", "resident", "wds"):
        torch.cuda.synchronize()
        waited = 0.0
        t0 = time.time()
        n = 8
        for i in range(n):
            if mode == "wds":
                tw = time.time()
                imgs, cs = fetch_data(it, dev, B)
                waited += time.time() - tw
                step(imgs, cs, nimg)
            else:
                step([pool[i % len(pool)].float() / 255.], [labels], nimg)
            nimg += B
        torch.cuda.synchronize()
        dt = time.time() - t0
        print(f"{mode:8s}: {n * B / dt:6.1f} img/s, {1e3 * dt / n:6.1f} ms/step, waited for data "
              f"{1e3 * waited / n:5.1f} ms/step", flush=True)


if __name__ == "__main__":
    main()
