"""The reference's training entry point on this build, end to end on CPU:

  * training/data_wds.py WdsWrapper over real tar shards (the class every stage YAML names):
    sample grouping, cls->text labels, key filter, augmentation determinism per seed, rank
    split, one-epoch pass with the processed-shard log and its resume skip;
  * train.main() with a YAML config: training_loop() runs two ticks, writes
    network-snapshot-*.pth with the reference key layout {G, D, G_ema, training_set_kwargs}
    and stats.jsonl; a second train.main() on the same run_dir auto-resumes from the newest
    snapshot (kimg parsed from the file name) and starts from exactly the saved weights.
"""
import io
import json
import os
import socket
import tarfile

import numpy as np
import pytest
import torch
import yaml

import net_cases


def _write_shards(root, n_shards=2, per_shard=5, size=(80, 72), seed=0):
    from PIL import Image
    rng = np.random.default_rng(seed)
    os.makedirs(root, exist_ok=True)
    keys = []
    for s in range(n_shards):
        with tarfile.open(os.path.join(root, f"part{s}", f"{s:05d}.tar") if False else os.path.join(root, f"{s:05d}.tar"),
                          "w") as tf:
            for i in range(per_shard):
                key = f"img{s:02d}_{i:03d}"
                keys.append(key)
                arr = rng.integers(0, 256, (size[1], size[0], 3), dtype=np.uint8)
                buf = io.BytesIO()
                Image.fromarray(arr).save(buf, format="PNG")
                for ext, data in (("png", buf.getvalue()), ("cls", str((s * per_shard + i) % 3).encode())):
                    ti = tarfile.TarInfo(f"{key}.{ext}")
                    ti.size = len(data)
                    tf.addfile(ti, io.BytesIO(data))
    return keys


def test_wds_wrapper_batches_labels_and_filter(tmp_path):
    from training.data_wds import WdsWrapper
    keys = _write_shards(str(tmp_path / "wds"))
    c2t = tmp_path / "c2t.json"
    json.dump({"0": "zero", "1": "one", "2": "two"}, open(c2t, "w"))
    keep = tmp_path / "keep.json"
    json.dump(keys[:7], open(keep, "w"))
    ds = WdsWrapper(str(tmp_path / "wds"), 64, label_type="cls2text", cls_to_text_path=str(c2t),
                    filter_keys_path=str(keep), data_augmentation=True, workers=1, sample_shuffle_size=3)
    assert len(ds) == 7 and ds.label_dim == 3 and ds.image_shape == [3, 64, 64] and ds.name == "wds"
    it = ds.iterate(batch_size=4, seed=5)
    imgs, labels = next(it)
    assert imgs.shape == (4, 3, 64, 64) and imgs.dtype == torch.uint8
    assert all(lab in ("zero", "one", "two") for lab in labels)
    imgs2, labels2 = next(ds.iterate(batch_size=4, seed=5))
    assert torch.equal(imgs, imgs2) and labels == labels2           # seeded: reproducible stream


def test_wds_one_epoch_pass_log_and_resume_skip(tmp_path):
    from training.data_wds import WdsWrapper, get_all_processed_tars
    _write_shards(str(tmp_path / "wds"), n_shards=4, per_shard=3)
    log_dir = str(tmp_path / "log")
    c2t = tmp_path / "c2t.json"
    json.dump({"0": "zero", "1": "one", "2": "two"}, open(c2t, "w"))
    kw = dict(label_type="cls2id", one_epoch=True, processed_tar_write_dir=log_dir, workers=1,
              sample_shuffle_size=2, cls_to_text_path=str(c2t))
    counts = []
    for rank in range(2):
        ds = WdsWrapper(str(tmp_path / "wds"), 32, **kw)
        n = sum(b[0].shape[0] for b in ds.iterate(batch_size=1, rank=rank, world=2, seed=1))
        counts.append(n)
        labels = next(ds.iterate(batch_size=2, rank=rank, world=2, seed=1))[1]
        assert labels.shape == (2, 3) and float(labels.sum()) == 2.0   # one-hot (cls2id)
    assert counts == [6, 6]                                            # 4 shards x 3 split over 2 ranks
    logged = [ln.strip() for r in range(2) for ln in open(os.path.join(log_dir, f"processed_tars_rank{r:02d}.txt"))]
    assert sorted(set(logged)) == sorted(str(p) for p in (tmp_path / "wds").glob("*.tar"))
    assert len(get_all_processed_tars(log_dir, workers=0)) == 4
    ds = WdsWrapper(str(tmp_path / "wds"), 32, label_type="cls2id", one_epoch=True, processed_tar_read_dir=log_dir,
                    workers=1, cls_to_text_path=str(c2t))
    # the last `workers` logged shard of each rank may have been in flight: it is re-read
    # (reference get_all_processed_tars :136), the other two are skipped
    left = sum(b[0].shape[0] for b in ds.iterate(batch_size=1, rank=0, world=1, seed=1))
    assert left == 2 * 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_train_main_snapshot_and_auto_resume(tmp_path, monkeypatch):
    import train
    from training import training_loop as tl
    _write_shards(str(tmp_path / "wds"), n_shards=2, per_shard=4)
    vfm = tmp_path / net_cases.VFM_DIRNAME
    vfm.mkdir()
    json.dump(dict(net_cases.SIGLIP_CFG, layer_norm_eps=1e-6), open(vfm / "config.json", "w"))
    run_dir = tmp_path / "run"
    g_kw = dict(net_cases.g_kwargs(str(vfm)), class_name="networks.generator.Generator")
    for k in ("img_resolution", "conditional", "label_type"):
        g_kw.pop(k)
    cfg = dict(
        run_dir=str(run_dir), random_seed=3,
        training_set_kwargs=dict(class_name="training.data_wds.WdsWrapper", path=str(tmp_path / "wds"), resolution=64,
                                 conditional=False, label_type="cls2text", data_augmentation=True, one_epoch=False,
                                 workers=1, sample_shuffle_size=2),
        G_kwargs=g_kw,
        D_kwargs=dict(net_cases.D_KWARGS, class_name="networks.discriminator.ProjectedDiscriminator"),
        loss_kwargs=dict(net_cases.loss_kwargs(str(vfm)), class_name="training.loss.TotalLoss"),
        G_opt_kwargs=dict(class_name="torch.optim.Adam", lr=1e-4, betas=[0.0, 0.99], eps=1e-8),
        D_opt_kwargs=dict(class_name="torch.optim.Adam", lr=1e-4, betas=[0.0, 0.99], eps=1e-8),
        batch_size=2, accumulate_gradients=1, kimg_per_tick=0.002, image_snapshot_ticks=1, network_snapshot_ticks=1,
        total_kimg=0.004, ema_kimg=0.01, ema_rampup=0.05, metrics=[], cudnn_benchmark=False, resume_path=None,
        resume_kimg=0)
    for k in ("vfm_name", "resume_kimg"):
        cfg["loss_kwargs"].pop(k, None)
    cfg_path = tmp_path / "cfg.yaml"
    yaml.safe_dump(cfg, open(cfg_path, "w"))
    monkeypatch.setenv("MASTER_PORT", str(_free_port()))
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    train.main(["--config", str(cfg_path)])
    snaps = sorted(run_dir.glob("network-snapshot-*.pth"))
    assert snaps, list(run_dir.iterdir())
    ck = torch.load(snaps[-1], map_location="cpu", weights_only=True)
    assert set(ck) == {"G", "D", "G_ema", "training_set_kwargs"}
    assert ck["training_set_kwargs"]["class_name"] == "training.data_wds.WdsWrapper"
    stats = [json.loads(ln) for ln in open(run_dir / "stats.jsonl")]
    assert stats and "Timing/sec_per_kimg" in stats[-1]
    # second run: auto-resume from the newest snapshot; capture the weights it starts from
    seen = {}
    orig = tl.TrainingIteration.__call__

    def spy(self, *a, **k):
        if not seen:
            seen["G"] = {n: t.detach().clone() for n, t in self.G.state_dict().items()}
            seen["D"] = {n: t.detach().clone() for n, t in self.D.state_dict().items()}
        return orig(self, *a, **k)

    monkeypatch.setattr(tl.TrainingIteration, "__call__", spy)
    cfg["total_kimg"] = 0.006
    yaml.safe_dump(cfg, open(cfg_path, "w"))
    torch.distributed.destroy_process_group() if torch.distributed.is_initialized() else None
    train.main(["--config", str(cfg_path)])
    for name in ("G", "D"):
        for n, t in ck[name].items():
            assert torch.equal(seen[name][n], t), (name, n)


def test_wds_process_workers_batches(tmp_path):
    """Decode in spawned worker processes (the GPU-host default): whole batches per worker, the same
    decoded images as the thread workers (one-epoch pass, so the sample set is fixed)."""
    from training.data_wds import WdsWrapper
    _write_shards(str(tmp_path / "wds"), n_shards=4, per_shard=4)
    c2t = tmp_path / "c2t.json"
    c2t.write_text(json.dumps({"0": "zero", "1": "one", "2": "two"}))
    kw = dict(label_type="cls2text", cls_to_text_path=str(c2t), workers=2, one_epoch=True, sample_shuffle_size=2)
    got = {}
    for procs in (False, True):
        ds = WdsWrapper(str(tmp_path / "wds"), 64, processes=procs, **kw)
        batches = list(ds.iterate(batch_size=4, seed=3))
        assert all(b[0].shape == (4, 3, 64, 64) and b[0].dtype == torch.uint8 for b in batches)
        assert all(len(b[1]) == 4 and all(lab in ("zero", "one", "two") for lab in b[1]) for b in batches)
        got[procs] = sorted(bytes(x.numpy().tobytes()[:64]) for b in batches for x in b[0])
    assert len(got[True]) == 16 and got[True] == got[False]


def test_wds_process_leftovers_pooled(tmp_path):
    """One-epoch pass on worker processes: each worker's last partial batch goes to the parent, which
    pools the leftovers into whole batches (only the final remainder is dropped, as on threads)."""
    from training.data_wds import WdsWrapper
    _write_shards(str(tmp_path / "wds"), n_shards=4, per_shard=3)
    c2t = tmp_path / "c2t.json"
    c2t.write_text(json.dumps({"0": "zero", "1": "one", "2": "two"}))
    kw = dict(label_type="cls2text", cls_to_text_path=str(c2t), workers=2, one_epoch=True, sample_shuffle_size=2)
    n = {}
    for procs in (False, True):
        ds = WdsWrapper(str(tmp_path / "wds"), 64, processes=procs, **kw)
        batches = list(ds.iterate(batch_size=4, seed=3))
        assert all(b[0].shape == (4, 3, 64, 64) and len(b[1]) == 4 for b in batches)
        n[procs] = len(batches)
    assert n[True] == n[False] == 3          # 12 samples: 2 workers x (1 whole batch + 2 leftovers)


def test_wds_process_worker_death_raises(tmp_path):
    """A decode worker killed without reaching its finally clause (SIGKILL) must surface as an error
    in the training process, not as an endless wait for its end-of-stream sentinel."""
    import multiprocessing as mp
    import signal
    import time
    from training.data_wds import WdsWrapper
    _write_shards(str(tmp_path / "wds"), n_shards=2, per_shard=4)
    c2t = tmp_path / "c2t.json"
    c2t.write_text(json.dumps({"0": "zero", "1": "one", "2": "two"}))
    ds = WdsWrapper(str(tmp_path / "wds"), 64, processes=True, label_type="cls2text", cls_to_text_path=str(c2t),
                    workers=2, one_epoch=False, sample_shuffle_size=2)
    ds.worker_poll_s = 0.2
    it = ds.iterate(batch_size=2, seed=3)
    next(it)
    victims = [p for p in mp.active_children() if "Process" in p.name]
    assert victims
    os.kill(victims[0].pid, signal.SIGKILL)
    t0 = time.time()
    with pytest.raises(RuntimeError, match="died without finishing"):
        while time.time() - t0 < 60:
            next(it)
    it.close()


def test_fast_adam_step_matches_torch_fused_adam():
    """training_loop.fast_adam_step (cached tensor lists -> torch._fused_adam_) against torch.optim.Adam
    (fused=True).step() on a twin model: bit-identical parameters after every step, including a step where
    one parameter has no gradient (the cache is rebuilt) and the first step (regular path creates state)."""
    import dnnlib
    from training.training_loop import fast_adam_step

    def mk():
        torch.manual_seed(0)
        return torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Linear(16, 4))
    a, b = mk(), mk()
    kw = dict(lr=1e-2, betas=(0.0, 0.99), eps=1e-8, fused=True)
    oa, ob = torch.optim.Adam(a.parameters(), **kw), torch.optim.Adam(b.parameters(), **kw)
    phase = dnnlib.EasyDict(opt=ob)
    used = []
    g = torch.Generator().manual_seed(1)
    for i in range(4):
        x = torch.randn(5, 8, generator=g)
        for m in (a, b):
            m.zero_grad(set_to_none=True)
            m(x).square().sum().backward()
        if i == 2:
            a[1].bias.grad = None
            b[1].bias.grad = None
        oa.step()
        u = fast_adam_step(phase) is not False
        if not u:
            ob.step()
        used.append(u)
        assert all(torch.equal(p, q) for p, q in zip(a.parameters(), b.parameters())), i
    assert used == [False, True, True, True]
