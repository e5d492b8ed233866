"""WebDataset (tar shard) training input, restated without the `webdataset` package.

Same class name, constructor keywords and dataset surface as the reference
`training/data_wds.py` (`WdsWrapper` :356-472, pipeline `wds_dataloader` :235-353), which every
stage YAML names (`training_set_kwargs.class_name: training.data_wds.WdsWrapper`):

  shards    sorted `path/**/*.tar` (label types cls2text / cls2id) or the tars next to
            `*_stats.json` files (text); endless random resampling of shards per rank and
            worker (`ResampledShards`), or -- `one_epoch` -- one shuffled pass split over
            ranks and workers (`SimpleShardList` + `split_by_node` + `split_by_worker`) whose
            consumed shards are logged per rank (`ShardTracker`, :70-115) and skipped on
            resume (`get_all_processed_tars`, :123-144);
  samples   tar members grouped by key (`tarfile_to_samples`), a shuffle buffer of
            `sample_shuffle_size` raw samples, the optional key filter, decode to RGB;
            errors are logged and skipped (`log_and_continue`);
  images    cls2text/cls2id: `transform_image` (:195-217) -- crop side = min(h, w) * U(0.5, 1)
            at a random offset (centre crop of the short side without augmentation), LANCZOS
            resize to `resolution`, horizontal flip with p = 0.5; text: images already at
            `resolution` (`preprocess_img`, :150-157);
  labels    cls2text: class index -> text (`cls_to_text_path` JSON); cls2id: one-hot over
            the classes; text: the stripped caption.

MI355X-side design: decode and augmentation run in `workers` host processes (`processes=True`,
the default on a GPU host: the training loop's own Python thread issues ~10k kernel launches per
iteration and held the GIL long enough that decode threads fell behind -- 53 ms of every
~420 ms step waiting for a batch in `tools_dev/wdsbench.py` with 12 threads that decode 440 img/s
on an idle host), each owning its shard stream and emitting whole batches, like the reference's
WebLoader workers; or on threads (`processes=False`: the one-epoch shard log and CPU runs). Batches
land in pinned uint8 [B, 3, R, R] tensors, so the training loop's host->device copy is
asynchronous (`training_loop.fetch_data`, `non_blocking=True`) and overlaps the previous
iteration. The key filter file (reference: a pickled key set) is read with a loader that
accepts only plain containers and strings (nothing in the file is executed); JSON or text
(one key per line) files work too.
"""
import glob
import io
import json
import logging
import os
import pickle
import queue
import random
import tarfile
import threading
from pathlib import Path

import numpy as np
import torch

from torch_utils import distributed as dist

DEFAULT_SEED = 42
_IMAGE_EXTS = ("jpg", "jpeg", "png", "webp")


# ----------------------------------------------------------------------------- helpers

class _PlainUnpickler(pickle.Unpickler):
    """Unpickles builtin containers / strings / numbers only (the key-filter sets)."""
    _OK = {("builtins", n) for n in ("set", "frozenset", "list", "tuple", "dict", "str", "int")}

    def find_class(self, module, name):
        if (module, name) in self._OK:
            return getattr(__import__(module), name)
        raise pickle.UnpicklingError(f"key filter file refers to {module}.{name}; only plain containers are read")


def load_key_filter(path):
    """Set of sample keys to keep, from a pickled set/list, a JSON list or a text file."""
    if not path or not os.path.isfile(path):
        return None
    if path.endswith(".json"):
        return set(json.load(open(path)))
    if path.endswith(".txt"):
        return {line.strip() for line in open(path) if line.strip()}
    with open(path, "rb") as f:
        return set(_PlainUnpickler(f).load())


def get_tail(p):
    """'…/capsfusion_120m_09/00304.tar' -> 'capsfusion_120m_09/00304.tar' (reference :147-148)."""
    return os.path.join(os.path.basename(os.path.dirname(p)), os.path.basename(p))


def get_all_processed_tars(processed_tar_read_dir, workers):
    """Shard tails recorded by earlier one-epoch runs; the last `workers` lines of every log may
    belong to shards still in flight when that run stopped, so they are not skipped."""
    done = set()
    if processed_tar_read_dir and os.path.isdir(processed_tar_read_dir):
        for txt in glob.glob(os.path.join(processed_tar_read_dir, "processed_tars_*.txt")):
            lines = [ln.strip() for ln in open(txt)]
            lines = lines[:-workers] if workers > 0 else lines
            done.update(get_tail(ln) for ln in lines if ln)
    return sorted(done)


class ShardTracker:
    """Appends each newly seen shard URL to processed_tars_rank{rank:02d}.txt (one-epoch mode)."""

    def __init__(self, log_dir, rank):
        os.makedirs(log_dir, exist_ok=True)
        self.log_path = os.path.join(log_dir, f"processed_tars_rank{rank:02d}.txt")
        self.seen = set()
        if os.path.isfile(self.log_path):
            self.seen = {ln.strip() for ln in open(self.log_path) if ln.strip()}
        self._lock = threading.Lock()

    def __call__(self, url):
        with self._lock:
            if url not in self.seen:
                self.seen.add(url)
                with open(self.log_path, "a") as f:
                    f.write(url + "\n")


def transform_image(img, resolution, augment, rng):
    """Reference transform_image (:195-217) with an explicit random.Random."""
    from PIL import Image
    a = np.asarray(img)
    if a.ndim == 2:
        a = np.repeat(a[:, :, None], 3, axis=2)
    h, w = a.shape[:2]
    ratio = rng.uniform(0.5, 1.0) if augment else 1.0
    side = max(1, int(min(h, w) * ratio))
    top = rng.randint(0, h - side) if augment else max((h - side) // 2, 0)
    left = rng.randint(0, w - side) if augment else max((w - side) // 2, 0)
    a = a[top:top + side, left:left + side]
    a = np.asarray(Image.fromarray(a, "RGB").resize((resolution, resolution), Image.LANCZOS))
    if augment and rng.random() < 0.5:
        a = a[:, ::-1]
    return np.ascontiguousarray(a.transpose(2, 0, 1), dtype=np.uint8)


def preprocess_img(img, resolution):
    a = np.asarray(img)
    if a.ndim == 2:
        a = np.repeat(a[:, :, None], 3, axis=2)
    a = a.transpose(2, 0, 1)
    if a.shape[-1] != resolution:
        raise ValueError(f"image width {a.shape[-1]} does not match resolution {resolution}")
    return np.ascontiguousarray(a, dtype=np.uint8)


def iter_tar_samples(url, log=logging.warning):
    """{'__key__', '__url__', ext: bytes} per key, in tar order (tarfile_to_samples)."""
    try:
        tf = tarfile.open(url, "r")
    except Exception as e:  # log_and_continue
        log(f"Webdataset error ({e!r}). Ignoring.")
        return
    with tf:
        cur_key, cur = None, None
        for m in tf:
            if not m.isfile():
                continue
            d, base = os.path.split(m.name)
            if "." not in base:
                continue
            key, ext = base.split(".", 1)
            key = os.path.join(d, key) if d else key
            if key != cur_key:
                if cur is not None:
                    yield cur
                cur_key, cur = key, {"__key__": key, "__url__": url}
            try:
                cur[ext.lower()] = tf.extractfile(m).read()
            except Exception as e:
                log(f"Webdataset error ({e!r}). Ignoring.")
        if cur is not None:
            yield cur


# ----------------------------------------------------------------------------- dataset

class _WorkerError:
    def __init__(self, exc):
        self.exc = exc


class _Leftover:
    """A worker's last partial batch (fewer than batch_size samples)."""

    def __init__(self, arr, labels):
        self.arr, self.labels = arr, labels


def _batch_worker(ds, rank, world, seed, w, batch_size, out_q, stop):
    """Process entry of WdsWrapper._iterate_processes: worker w's shard stream -> whole batches
    (uint8 [B, 3, R, R] numpy, labels); the same per-worker seeds as the thread workers."""
    try:
        shards, _ = ds._shard_plan(rank, world, seed)
        keep = load_key_filter(ds.filter_keys_path) if ds.label_type != "text" else None
        rng = random.Random((seed + rank * 1000 + w) * 7919 + 1)
        R = ds.resolution
        arr, labels = np.empty([batch_size, 3, R, R], dtype=np.uint8), []
        for img, lab in ds._samples(shards[w], None, rng, keep, stop):
            arr[len(labels)] = img
            labels.append(lab)
            if len(labels) == batch_size:
                out_q.put((arr, labels))
                arr, labels = np.empty([batch_size, 3, R, R], dtype=np.uint8), []
        if labels and not stop.is_set():
            # this worker's leftover samples: the parent pools the leftovers of all workers into whole
            # batches, so only the final remainder of the epoch is dropped (as with threads / wds.batched)
            out_q.put(_Leftover(arr[:len(labels)].copy(), labels))
    except Exception as e:                            # surfaced in iterate(), not swallowed
        out_q.put(_WorkerError(e))
    finally:
        out_q.put(None)


class WdsWrapper:
    def __init__(self, path, resolution, label_type="text", filter_keys_path=None, cls_to_text_path=None,
                 data_augmentation=False, one_epoch=False, processed_tar_read_dir=None,
                 processed_tar_write_dir=None, workers=3, shard_shuffle_size=50_000, sample_shuffle_size=50_000,
                 processes=None, **_unused):
        self._root = Path(path)
        self.resolution = int(resolution)
        self.label_type = label_type
        if label_type not in ("text", "cls2text", "cls2id"):
            raise ValueError(f"Unsupported label_type: {label_type}")
        self.filter_keys_path = filter_keys_path
        self.cls_to_text_path = cls_to_text_path
        self.data_augmentation = bool(data_augmentation)
        self.one_epoch = bool(one_epoch)
        self.processed_tar_read_dir = processed_tar_read_dir
        self.processed_tar_write_dir = processed_tar_write_dir
        self.workers = max(1, int(workers))
        self.shard_shuffle_size = int(shard_shuffle_size)
        self.sample_shuffle_size = max(1, int(sample_shuffle_size))
        self._cls2text = json.load(open(cls_to_text_path, encoding="utf-8")) \
            if cls_to_text_path and os.path.isfile(cls_to_text_path) else None
        self.num_classes = len(self._cls2text) if self._cls2text else 0
        self.urls = self._get_urls(str(path))
        # decode in processes on a GPU host (see the module docstring); threads for the one-epoch
        # shard log (a per-rank file the workers append to) and by request
        self.processes = bool(torch.cuda.is_available() if processes is None else processes)
        self.worker_poll_s = 5.0             # watchdog period of the process workers (dead-worker check)

    def _get_urls(self, path):
        if self.label_type in ("cls2text", "cls2id"):
            return sorted(glob.glob(f"{path}/**/*.tar", recursive=True))
        return sorted(p.replace("_stats.json", ".tar") for p in glob.glob(f"{path}/**/*.json", recursive=True))

    # reference dataset surface ------------------------------------------------------
    def __len__(self):
        if self.label_type in ("cls2text", "cls2id"):
            keys = load_key_filter(self.filter_keys_path)
            return len(keys) if keys is not None else 1281167      # ImageNet-1k
        return len(self.urls) * 10000

    @property
    def image_shape(self):
        return [3, self.resolution, self.resolution]

    @property
    def label_shape(self):
        return [self.num_classes] if self.label_type in ("cls2text", "cls2id") else [1]

    @property
    def label_dim(self):
        return self.label_shape[0]

    @property
    def name(self):
        return self._root.name

    # sample decoding -------------------------------------------------------------------
    def _label(self, sample):
        if self.label_type == "text":
            txt = sample.get("txt")
            if txt is None:
                return None
            txt = txt.decode("utf-8", errors="ignore").strip()
            return txt or None
        raw = sample.get("cls")
        if raw is None:
            return None
        cls = int(raw.decode().strip())
        if self.label_type == "cls2id" and not 0 <= cls < self.num_classes:
            raise ValueError(f"class {cls} outside the {self.num_classes} classes of cls_to_text_path "
                             f"({self.cls_to_text_path}); cls2id one-hot labels need the class list")
        if self.label_type == "cls2text":
            return self._cls2text[str(cls)] if self._cls2text is not None else str(cls)
        one_hot = np.zeros(self.num_classes, dtype=np.float32)
        one_hot[cls] = 1.0
        return one_hot

    def _decode(self, sample, rng):
        from PIL import Image
        data = next((sample[e] for e in _IMAGE_EXTS if e in sample), None)
        label = self._label(sample)
        if data is None or label is None:
            return None
        try:
            with Image.open(io.BytesIO(data)) as im:
                im = im.convert("RGB")
                if self.label_type == "text":
                    return preprocess_img(im, self.resolution), label
                return transform_image(im, self.resolution, self.data_augmentation, rng), label
        except Exception as e:  # log_and_continue
            logging.warning(f"Webdataset error ({e!r}). Ignoring.")
            return None

    # shard streams -------------------------------------------------------------------
    def _shard_plan(self, rank, world, seed):
        """Per-worker shard iterables for this rank."""
        urls = list(self.urls)
        if not urls:
            raise FileNotFoundError(f"no WebDataset shards under {self._root}")
        if not self.one_epoch:
            def resampled(w):
                r = random.Random((seed * 1_000_003 + rank) * 131 + w)
                while True:
                    yield r.choice(urls)
            return [resampled(w) for w in range(self.workers)], None
        tracker = None
        if self.processed_tar_read_dir:
            skip = set(get_all_processed_tars(self.processed_tar_read_dir, self.workers))
            done = [u for u in urls if get_tail(u) in skip]
            urls = [u for u in urls if get_tail(u) not in skip]
            dist.print0(f"[one-epoch] skipped {len(done)} shards, {len(urls)} remain")
            if self.processed_tar_write_dir and done:
                os.makedirs(self.processed_tar_write_dir, exist_ok=True)
                with open(os.path.join(self.processed_tar_write_dir, f"processed_tars_rank{rank:02d}.txt"), "a") as f:
                    f.writelines(u + "\n" for u in done)
        if self.processed_tar_write_dir:
            tracker = ShardTracker(self.processed_tar_write_dir, rank)
        random.Random(seed).shuffle(urls)            # same order on every rank, then split
        mine = urls[rank::world]
        return [iter(mine[w::self.workers]) for w in range(self.workers)], tracker

    def _worker(self, shards, tracker, rng, keep, out_q, stop):
        try:
            for item in self._samples(shards, tracker, rng, keep, stop):
                out_q.put(item)
        except Exception as e:                        # surfaced in iterate(), not swallowed
            out_q.put(_WorkerError(e))
        finally:
            out_q.put(None)                           # this worker is exhausted

    def _samples(self, shards, tracker, rng, keep, stop):
        """Decoded (image, label) items of one worker's shard stream through its shuffle buffer."""
        buf = []
        for url in shards:
            if stop.is_set():
                return
            for sample in iter_tar_samples(url):
                if tracker is not None:
                    tracker(sample["__url__"])
                if keep is not None and os.path.basename(sample["__key__"]) not in keep \
                        and sample["__key__"] not in keep:
                    continue
                buf.append(sample)
                if len(buf) >= self.sample_shuffle_size:
                    item = self._decode(buf.pop(rng.randrange(len(buf))), rng)
                    if item is not None:
                        yield item
                if stop.is_set():
                    return
        rng.shuffle(buf)
        for smp in buf:
            item = self._decode(smp, rng)
            if item is not None:
                yield item

    def _iterate_processes(self, batch_size, rank, world, seed):
        """Worker processes (spawned: no CUDA state is inherited) each decode their shard stream into
        whole batches; the parent copies each into a pinned tensor."""
        import multiprocessing as mp
        ctx = mp.get_context("spawn")
        out_q = ctx.Queue(maxsize=2 * self.workers)
        stop = ctx.Event()
        procs = [ctx.Process(target=_batch_worker, daemon=True, args=(self, rank, world, seed, w, batch_size, out_q,
                                                                           stop))
                 for w in range(self.workers)]
        for p in procs:
            p.start()
        live = len(procs)
        pin = torch.cuda.is_available()
        carry_arr, carry_lab = [], []          # pooled leftovers of finished workers
        try:
            while True:
                # watchdog: a worker killed before its finally clause (OOM kill, SIGKILL, a crash in the
                # decoder) never posts its None sentinel; without this check live never reaches 0 and
                # the loop waits forever (a normal exit is code 0, after the sentinel)
                dead = [(i, p.exitcode) for i, p in enumerate(procs) if p.exitcode not in (None, 0)]
                if dead:
                    raise RuntimeError(f"WebDataset worker process(es) died without finishing: "
                                       f"{', '.join(f'worker {i} exit code {c}' for i, c in dead)}")
                try:
                    item = out_q.get(timeout=self.worker_poll_s)
                except queue.Empty:
                    continue
                if isinstance(item, _WorkerError):
                    raise RuntimeError("WebDataset worker failed") from item.exc
                if item is None:
                    live -= 1
                    if live == 0:
                        return
                    continue
                if isinstance(item, _Leftover):
                    carry_arr.append(item.arr)
                    carry_lab.extend(item.labels)
                    if len(carry_lab) < batch_size:
                        continue
                    pooled = np.concatenate(carry_arr)
                    arr, labels = pooled[:batch_size], carry_lab[:batch_size]
                    carry_arr, carry_lab = ([pooled[batch_size:]] if len(carry_lab) > batch_size else []), \
                        carry_lab[batch_size:]
                else:
                    arr, labels = item
                imgs = torch.from_numpy(arr)
                if pin:
                    imgs = imgs.pin_memory()
                if self.label_type == "cls2id":
                    labels = torch.from_numpy(np.stack(labels))
                yield imgs, labels
        finally:
            stop.set()
            for p in procs:
                p.join(timeout=0.5)
                if p.is_alive():
                    p.terminate()

    def iterate(self, batch_size, rank=0, world=1, seed=DEFAULT_SEED):
        """Batches (pinned uint8 [batch_size, 3, R, R], labels) for this rank: endless, or one
        pass over this rank's shards in one-epoch mode (the last partial batch is dropped, as
        `wds.batched` + the loop's full-batch split)."""
        if self.processes and not (self.one_epoch and (self.processed_tar_write_dir or self.processed_tar_read_dir)):
            yield from self._iterate_processes(batch_size, rank, world, seed)
            return
        shards, tracker = self._shard_plan(rank, world, seed)
        keep = load_key_filter(self.filter_keys_path) if self.label_type != "text" else None
        out_q = queue.Queue(maxsize=4 * batch_size)
        stop = threading.Event()
        threads = [threading.Thread(target=self._worker, daemon=True,
                                    args=(shards[w], tracker, random.Random((seed + rank * 1000 + w) * 7919 + 1),
                                          keep, out_q, stop))
                   for w in range(self.workers)]
        for t in threads:
            t.start()
        live = len(threads)
        R = self.resolution
        pin = torch.cuda.is_available()
        try:
            while True:
                imgs = torch.empty([batch_size, 3, R, R], dtype=torch.uint8, pin_memory=pin)
                labels = []
                while len(labels) < batch_size:
                    item = out_q.get()
                    if isinstance(item, _WorkerError):
                        raise RuntimeError("WebDataset worker failed") from item.exc
                    if item is None:
                        live -= 1
                        if live == 0:
                            return
                        continue
                    img, lab = item
                    imgs[len(labels)].copy_(torch.from_numpy(img))
                    labels.append(lab)
                if self.label_type == "cls2id":
                    labels = torch.from_numpy(np.stack(labels))
                yield imgs, labels
        finally:
            stop.set()
            while any(t.is_alive() for t in threads):   # unblock workers waiting on a full queue
                try:
                    out_q.get_nowait()
                except queue.Empty:
                    pass
                for t in threads:
                    t.join(timeout=0.05)
