"""Shared plumbing of the inference tools (reconstruct / decode / evaluate).

Mirrors what the reference tools do around the model call
(`tools/reconstruct/reconstruct.py:93-149`, `tools/decode/decode_latents_to_images.py:126-183`):
YAML `G_kwargs` + the tool overrides (label_dim 1000, unconditional, cls2text, KL/VF off,
`num_fp16_res = 0`), checkpoint `G_ema` (or a bare state dict) loaded with strict=False, and
torchvision's image conversions restated on PIL + numpy (torchvision is not in the image):

  * `load_image`   = Resize(res) (shorter side, PIL bilinear) → CenterCrop(res) → ToTensor
  * `to_uint8`     = `to_pil_image(t.clamp(0, 1))`, i.e. `t.mul(255).byte()` (truncation),
                     done on the device so only uint8 crosses PCIe.

MI355X design: one process per GPU (torchrun env vars; RCCL process group only for the final
barrier — the work is sharded by file, there is no data-path collective), host decode of the
next batch and PNG encoding of the previous one overlap the GPU work on a thread pool, and
host→device copies come from pinned memory.
"""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch
import yaml

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if PKG not in sys.path:
    sys.path.insert(0, PKG)

import dnnlib  # noqa: E402


class Rank:
    """Process placement: torchrun env vars when present, a single process otherwise."""

    def __init__(self, device=None):
        self.world_size = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        if device is None:
            device = f"cuda:{local}" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        self.pg = False
        if self.world_size > 1 and not torch.distributed.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            backend = "nccl" if self.device.type == "cuda" else "gloo"
            kw = {"device_id": self.device} if backend == "nccl" else {}
            torch.distributed.init_process_group(backend=backend, init_method="env://", **kw)
            self.pg = True

    def shard(self, items):
        """Files are dealt round-robin over ranks (reference decode: `all_files[rank::world_size]`)."""
        return list(items)[self.rank::self.world_size]

    def barrier(self):
        if torch.distributed.is_initialized():
            torch.distributed.barrier()

    def close(self):
        if self.pg:
            torch.distributed.destroy_process_group()


def vae_kwargs_from_config(path, resolution=256, keys=("G_kwargs",)):
    with open(path, "r") as f:
        cfg = yaml.safe_load(f)
    kw = {}
    for k in keys:                                     # first key present wins
        if k in cfg:
            kw = dict(cfg[k])
            break
    kw["label_dim"] = 1000
    kw["img_resolution"] = resolution
    kw["conditional"] = False
    kw["label_type"] = "cls2text"
    kw["use_kl_loss"] = False
    kw["use_vf_loss"] = False
    kw["num_fp16_res"] = 0
    return kw


def build_vae(config_path, resolution, device, vae_kwargs_override=None, keys=("G_kwargs",)):
    kw = vae_kwargs_from_config(config_path, resolution, keys)
    if vae_kwargs_override:
        kw.update(vae_kwargs_override)
    vae = dnnlib.util.construct_class_by_name(**kw).to(device)
    vae.requires_grad_(False)
    return vae


def load_vae_weights(vae, path, device, log=print):
    """`G_ema` of a training snapshot, else the whole dict as a state dict. Loaded with
    `weights_only=True` (no unpickling of arbitrary objects)."""
    ckpt = torch.load(path, map_location=device, weights_only=True)
    if isinstance(ckpt, dict) and "G_ema" in ckpt:
        log("Found 'G_ema' in checkpoint, loading its weights...")
        sd = ckpt["G_ema"]
    elif isinstance(ckpt, dict):
        log("No 'G_ema' found, loading full state dict.")
        sd = ckpt
    else:
        raise TypeError(f"Unexpected checkpoint type: {type(ckpt)}")
    incompatible = vae.load_state_dict(sd, strict=False)
    vae.eval()
    return incompatible


def report_incompatible_keys(name, incompatible, log=print):
    if incompatible.missing_keys:
        log(f"[{name}] Missing keys ({len(incompatible.missing_keys)}):")
        for k in incompatible.missing_keys:
            log(f"  - {k}")
    if incompatible.unexpected_keys:
        log(f"[{name}] Unexpected keys ({len(incompatible.unexpected_keys)}):")
        for k in incompatible.unexpected_keys:
            log(f"  - {k}")
    if not incompatible.missing_keys and not incompatible.unexpected_keys:
        log(f"[{name}] All keys matched successfully.")


# ------------------------------------------------------------------ images

IMAGE_EXTS = (".jpg", ".jpeg", ".png")


def list_images(root, exts=IMAGE_EXTS):
    files = sorted(f for f in os.listdir(root) if f.lower().endswith(exts))
    if not files:
        raise FileNotFoundError(f"No images found in {root}")
    return files


def load_image(path, resolution):
    """torchvision Resize(resolution) + CenterCrop(resolution) + ToTensor on a PIL image →
    uint8 HWC array (the /255 happens on the device)."""
    from PIL import Image
    with Image.open(path) as im:
        im = im.convert("RGB")
        w, h = im.size
        if min(w, h) != resolution:
            # Resize(int): shorter side → resolution, longer side int(res * long / short)
            if w <= h:
                nw, nh = resolution, int(resolution * h / w)
            else:
                nw, nh = int(resolution * w / h), resolution
            im = im.resize((nw, nh), Image.BILINEAR)
            w, h = nw, nh
        # CenterCrop: offsets int(round((size - crop) / 2))
        top = int(round((h - resolution) / 2.0))
        left = int(round((w - resolution) / 2.0))
        im = im.crop((left, top, left + resolution, top + resolution))
        return np.asarray(im, dtype=np.uint8).copy()


def load_png_uint8(path):
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"), dtype=np.uint8).copy()


def to_uint8(img01):
    """[B,3,H,W] float in [0,1] → [B,H,W,3] uint8 with torchvision's `mul(255).byte()`
    truncation (to_pil_image of a float tensor)."""
    return img01.clamp(0, 1).mul(255).to(torch.uint8).permute(0, 2, 3, 1).contiguous()


def save_png(arr_hwc, path):
    from PIL import Image
    Image.fromarray(arr_hwc).save(path)


def batch_to_device(arrays, device):
    """list of HWC uint8 → [B,3,H,W] float32 in [0,1] on `device` (pinned, async H2D)."""
    x = torch.from_numpy(np.stack(arrays))
    if device.type == "cuda":
        x = x.pin_memory().to(device, non_blocking=True)
    return x.permute(0, 3, 1, 2).float().div_(255.0)


class Writer:
    """PNG encoding off the critical path: a small thread pool; `drain()` waits for all."""

    def __init__(self, workers=8):
        self.pool = ThreadPoolExecutor(max_workers=workers)
        self.pending = []

    def put(self, arr, path):
        self.pending.append(self.pool.submit(save_png, arr, path))
        if len(self.pending) > 1024:
            self._reap()

    def _reap(self):
        done = [f for f in self.pending if f.done()]
        for f in done:
            f.result()
        self.pending = [f for f in self.pending if not f.done()]

    def drain(self):
        for f in self.pending:
            f.result()
        self.pending = []
        self.pool.shutdown(wait=True)
