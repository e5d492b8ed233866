"""WebDataset tar-shard input as the reference's preprocessing tools use it (webdataset is not
installed here): `SimpleShardList` → `split_by_node` (`urls[rank::world]`) →
`tarfile_to_samples` (members grouped by the key before the first '.', tar order) →
`decode("pilrgb")` → `rename(image="jpg;png", label="cls", key="__key__")` → ADM centre crop
(`tools/preprocess_for_*/prefetch.py` `center_crop_imagenet`), decode errors logged and skipped
as `log_and_continue`."""
import io
import os
import tarfile

import numpy as np

def center_crop_imagenet(image_size, arr):
    """ADM centre crop (reference `prefetch.py:113-127`)."""
    from PIL import Image
    im = Image.fromarray(arr)
    while min(*im.size) >= 2 * image_size:
        im = im.resize(tuple(x // 2 for x in im.size), resample=Image.Resampling.BOX)
    scale = image_size / min(*im.size)
    im = im.resize(tuple(round(x * scale) for x in im.size), resample=Image.Resampling.BICUBIC)
    a = np.array(im)
    cy = (a.shape[0] - image_size) // 2
    cx = (a.shape[1] - image_size) // 2
    return a[cy:cy + image_size, cx:cx + image_size]


def iter_wds_samples(urls, rank=0, world=1, log=print):
    """(image HWC uint8 RGB, label int, key) in shard/tar order for this rank's shards."""
    from PIL import Image
    for url in list(urls)[rank::world]:
        with tarfile.open(url, "r") as tf:
            cur_key, cur = None, {}

            def flush(key, members):
                if key is None:
                    return None
                img = members.get("jpg", members.get("png"))
                if img is None or "cls" not in members:
                    return None
                try:
                    with Image.open(io.BytesIO(img)) as im:
                        arr = np.asarray(im.convert("RGB"), dtype=np.uint8).copy()
                    return arr, int(members["cls"].decode().strip()), os.path.basename(key)
                except Exception as e:  # log_and_continue
                    log(f"Handling webdataset error ({type(e).__name__}): {e}")
                    return None

            for m in tf:
                if not m.isfile():
                    continue
                base = os.path.basename(m.name)
                dirn = os.path.dirname(m.name)
                if "." not in base:
                    continue
                key, ext = base.split(".", 1)
                key = os.path.join(dirn, key)
                if key != cur_key:
                    s = flush(cur_key, cur)
                    if s is not None:
                        yield s
                    cur_key, cur = key, {}
                cur[ext.lower()] = tf.extractfile(m).read()
            s = flush(cur_key, cur)
            if s is not None:
                yield s


def iter_batches(urls, resolution, batch_size, rank, world, log=print):
    """Batches of (uint8 [n,H,W,3] array, labels, keys); decode + crop of the next batch runs on a
    worker thread while the current one is encoded on the GPU."""
    from concurrent.futures import ThreadPoolExecutor
    it = iter_wds_samples(urls, rank, world, log)

    def take():
        imgs, labels, keys = [], [], []
        for arr, lab, key in it:
            imgs.append(center_crop_imagenet(resolution, arr))
            labels.append(lab)
            keys.append(key)
            if len(imgs) == batch_size:
                break
        return (np.stack(imgs), labels, keys) if imgs else None

    with ThreadPoolExecutor(max_workers=1) as pool:
        fut = pool.submit(take)
        while True:
            b = fut.result()
            if b is None:
                return
            fut = pool.submit(take)
            yield b
