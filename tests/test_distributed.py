"""Multi-process (gloo, world_size 2, CPU) tests of the data-parallel path:
FlatGradSync's bucketed hook-driven all-reduce reproduces the reference
`sync_grads` semantics (training_loop.py:281-289: sum over ranks / world, * gain,
nan_to_num(0, 1e5, -1e5)); a full TrainingIteration keeps the replicas identical."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT, PKG


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawn(fn, world=2, *args):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_entry, args=(fn, r, world, port, q, args)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, out = q.get(timeout=300)
        res[r] = out
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0, p.exitcode
    for r, out in res.items():
        if isinstance(out, str) and out.startswith("ERROR"):
            raise AssertionError(out)
    return res


def _entry(fn, rank, world, port, q, args):
    for p in (PKG, ROOT, os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
    torch.set_num_threads(2)
    try:
        from torch_utils import distributed as dist
        dist.init(backend="gloo")
        out = globals()[fn](rank, world, *args)
        # plain numpy (tensors would travel as shared-memory handles that die with this process)
        conv = lambda v: v.detach().numpy().copy() if isinstance(v, torch.Tensor) else v
        out = {k: conv(v) for k, v in out.items()} if isinstance(out, dict) else out
        q.put((rank, out))
        dist.destroy_process_group()
    except Exception as e:  # report to the parent instead of hanging it
        import traceback
        q.put((rank, "ERROR " + traceback.format_exc()))


def _toy(seed=0):
    torch.manual_seed(seed)
    m = torch.nn.Sequential(torch.nn.Linear(6, 32), torch.nn.Tanh(), torch.nn.Linear(32, 5))
    m.unused = torch.nn.Parameter(torch.ones(3))
    return m


def _toy_loss(m, rank, poison=False):
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(4, 6, generator=g)
    y = m(x)
    loss = y.square().sum() * (rank + 1)
    if poison and rank == 1:
        loss = loss + m[2].bias[0] * float("inf")
    return loss


def _flat_sync_worker(rank, world, bucket_mb, poison):
    from training.training_loop import FlatGradSync
    m = _toy()
    sync = FlatGradSync(m, bucket_mb=bucket_mb)
    sync.prepare()
    _toy_loss(m, rank, poison).backward()
    sync.finish(gain=2.0)
    return {n: (None if p.grad is None else p.grad.clone()) for n, p in m.named_parameters()}


@pytest.mark.parametrize("bucket_mb", [64.0, 1e-4])      # one bucket / one bucket per parameter
def test_flat_grad_sync_matches_reference_semantics(bucket_mb):
    res = _spawn("_flat_sync_worker", 2, bucket_mb, False)
    expect = {}
    for r in range(2):
        m = _toy()
        _toy_loss(m, r).backward()
        for n, p in m.named_parameters():
            if p.grad is not None:
                expect[n] = expect.get(n, 0) + p.grad
    for r in range(2):
        got = res[r]
        assert got["unused"] is None
        for n, e in expect.items():
            torch.testing.assert_close(torch.from_numpy(got[n]), e / 2 * 2.0, rtol=1e-6, atol=1e-6)


def test_flat_grad_sync_nan_to_num():
    res = _spawn("_flat_sync_worker", 2, 64.0, True)
    for r in range(2):
        b = torch.from_numpy(res[r]["2.bias"])
        assert torch.isfinite(b).all()
        assert float(b[0]) in (1e5, -1e5, 0.0)
    torch.testing.assert_close(torch.from_numpy(res[0]["0.weight"]), torch.from_numpy(res[1]["0.weight"]))


def _iteration_worker(rank, world):
    import copy
    import json
    import tempfile
    import net_cases
    from networks.generator import Generator
    from networks.discriminator import ProjectedDiscriminator
    from training.loss import TotalLoss
    from training.training_loop import TrainingIteration, make_optimizer
    d = os.path.join(tempfile.mkdtemp(), net_cases.VFM_DIRNAME)
    os.makedirs(d)
    json.dump(dict(net_cases.SIGLIP_CFG, layer_norm_eps=1e-6), open(os.path.join(d, "config.json"), "w"))
    torch.manual_seed(0)
    dev = torch.device("cpu")
    G = Generator(label_dim=0, **net_cases.g_kwargs(d)).train().requires_grad_(False)
    D = ProjectedDiscriminator(c_dim=0, **net_cases.D_KWARGS).train().requires_grad_(False)
    loss = TotalLoss(device=dev, G=G, D=D, **net_cases.loss_kwargs(d))
    opt = dict(class_name='torch.optim.Adam', lr=1e-3, betas=[0.0, 0.99], eps=1e-8)
    it = TrainingIteration(G, D, copy.deepcopy(G).eval(), loss, make_optimizer(G.parameters(), opt, dev),
                           make_optimizer(D.parameters(), opt, dev), batch_size=2 * world, bucket_mb=0.5)
    before = torch.cat([p.detach().flatten() for p in G.parameters()]).clone()
    g = torch.Generator().manual_seed(rank)
    img = torch.rand(2, 3, 64, 64, generator=g)
    it([img], [['x', 'x']], 0)
    after_g = torch.cat([p.detach().flatten() for p in G.parameters()])
    after_d = torch.cat([p.detach().flatten() for p in D.parameters()])
    return dict(moved=float((after_g - before).abs().max()), g=after_g, d=after_d)


def test_training_iteration_replicas_stay_identical():
    res = _spawn("_iteration_worker", 2)
    assert res[0]["moved"] > 0
    assert (res[0]["g"] == res[1]["g"]).all()
    assert (res[0]["d"] == res[1]["d"]).all()


def _tools_decode_worker(rank, world, lat_dir, out_dir, cfg, ckpt):
    """tools/decode on a 2-rank gloo group: each rank decodes sorted(files)[rank::2]."""
    import importlib.util
    tools = os.path.join(PKG, "tools")
    spec = importlib.util.spec_from_file_location("decode_tool", os.path.join(tools, "decode", "decode_latents_to_images.py"))
    dec = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(dec)
    import common
    rk = common.Rank("cpu")
    assert (rk.rank, rk.world_size) == (rank, world) and not rk.pg     # uses the existing group
    G = common.build_vae(cfg, 64, torch.device("cpu"))
    common.load_vae_weights(G, ckpt, torch.device("cpu"), log=lambda *a: None)
    n = dec.run_latent_decoding(G, lat_dir, out_dir, 2, rk, log=lambda *a: None)
    return {"n": n}


def test_tools_decode_shards_over_two_ranks(tmp_path):
    import json
    import yaml
    import net_cases
    from safetensors.torch import save_file
    vfm = tmp_path / net_cases.VFM_DIRNAME
    vfm.mkdir()
    json.dump(dict(net_cases.SIGLIP_CFG, layer_norm_eps=1e-6), open(vfm / "config.json", "w"))
    cfg = tmp_path / "tiny.yaml"
    yaml.safe_dump({"G_kwargs": dict(net_cases.g_kwargs(str(vfm)), class_name="networks.generator.Generator")},
                   open(cfg, "w"))
    sys.path.insert(0, os.path.join(PKG, "tools"))
    import common
    torch.manual_seed(0)
    G = common.build_vae(str(cfg), 64, torch.device("cpu"))
    ckpt = tmp_path / "snap.pth"
    torch.save({"G_ema": G.state_dict()}, ckpt)
    lat = tmp_path / "lat"
    lat.mkdir()
    g = torch.Generator().manual_seed(1)
    for i, n in enumerate([3, 2, 1]):                          # files 0, 2 -> rank 0; file 1 -> rank 1
        save_file({"latents": torch.randn(n, 32, 4, 4, generator=g)}, str(lat / f"f{i}.safetensors"))
    out = tmp_path / "dec"
    res = _spawn("_tools_decode_worker", 2, str(lat), str(out), str(cfg), str(ckpt))
    assert res[0]["n"] == 4 and res[1]["n"] == 2
    files = sorted(os.listdir(out))
    assert files == [f"rank00_{i:06d}.png" for i in range(4)] + [f"rank01_{i:06d}.png" for i in range(2)]


def _disagree_worker(rank, world):
    from training.training_loop import FlatGradSync
    m = _toy()
    sync = FlatGradSync(m, bucket_mb=64.0)
    sync.prepare()
    loss = _toy_loss(m, rank)
    if rank == 1:
        loss = loss + m.unused.sum()          # a gradient only rank 1 produces
    loss.backward()
    sync.finish()
    try:
        sync.prepare()                        # the agreement check of the previous step runs here
    except RuntimeError as e:
        return {"raised": "different parameter sets" in str(e)}
    return {"raised": False}


def test_flat_grad_sync_detects_rank_disagreement():
    res = _spawn("_disagree_worker", 2)
    assert res[0]["raised"] and res[1]["raised"]


def _stats_worker(rank, world):
    from torch_utils import training_stats
    training_stats.init_multiprocessing(rank, torch.device("cpu"))
    col = training_stats.Collector(regex="Loss/.*")
    training_stats.report("Loss/a", torch.tensor([1.0, 2.0]) * (rank + 1))
    training_stats.report0("Loss/r0", 5.0)
    training_stats.report("Other/x", 1.0)
    col.update()
    return {"names": col.names(), "num": col.num("Loss/a"), "mean": col.mean("Loss/a"), "std": col.std("Loss/a"),
            "r0": (col.num("Loss/r0"), col.mean("Loss/r0"))}


def test_training_stats_reduce_over_ranks():
    res = _spawn("_stats_worker", 2)
    vals = torch.tensor([1.0, 2.0, 2.0, 4.0], dtype=torch.float64)
    for r in range(2):
        out = res[r]
        assert out["names"] == ["Loss/a", "Loss/r0"]
        assert out["num"] == 4 and abs(out["mean"] - 2.25) < 1e-12
        assert abs(out["std"] - float(vals.std(unbiased=False))) < 1e-12
        assert out["r0"] == (1.0, 5.0)



def _accum_worker(rank, world, bucket_mb):
    """Two microbatches per phase (accumulate_gradients=2); m[0] is touched only in the first,
    m.unused only in the second (the last), m[2] in both."""
    from training.training_loop import FlatGradSync
    m = _toy()
    sync = FlatGradSync(m, bucket_mb=bucket_mb, collective=world > 1)
    sync.prepare()
    g = torch.Generator().manual_seed(200 + rank)
    x = torch.randn(4, 6, generator=g)
    h = torch.tanh(m[0](x)).detach()
    sync.last_microbatch = False
    (m[2](torch.tanh(m[0](x))).square().sum() * (rank + 1)).backward()          # microbatch 0: m[0], m[2]
    sync.last_microbatch = True
    ((m[2](h).sum() + m.unused.square().sum()) * (rank + 2)).backward()          # microbatch 1: m[2], unused
    sync.finish(gain=2.0)
    return {n: (None if p.grad is None else p.grad.clone()) for n, p in m.named_parameters()}


def _accum_expect(world):
    """sum over ranks and microbatches of the plain-autograd gradients / world * gain."""
    tot = {}
    for r in range(world):
        m = _toy()
        g = torch.Generator().manual_seed(200 + r)
        x = torch.randn(4, 6, generator=g)
        h = torch.tanh(m[0](x)).detach()
        (m[2](torch.tanh(m[0](x))).square().sum() * (r + 1)).backward()
        ((m[2](h).sum() + m.unused.square().sum()) * (r + 2)).backward()
        for n, p in m.named_parameters():
            tot[n] = tot.get(n, 0) + p.grad
    return {n: v / world * 2.0 for n, v in tot.items()}


@pytest.mark.parametrize("bucket_mb", [64.0, 1e-4])
def test_flat_grad_sync_two_microbatches(bucket_mb):
    """FlatGradSync over two microbatches with parameters touched in only one of them, on the
    collective path (gloo, 2 ranks: buckets launched from the last microbatch's hooks, the rest in
    finish()) and on the world-size-1 path (stolen gradients gathered in chunks): both equal
    sum / world * gain."""
    res = _spawn("_accum_worker", 2, bucket_mb)
    expect = _accum_expect(2)
    for r in (0, 1):
        for n, v in expect.items():
            assert res[r][n] is not None, n
            assert torch.allclose(torch.from_numpy(res[r][n]), v, rtol=1e-5, atol=1e-6), (r, n)
    from training.training_loop import FlatGradSync  # noqa: F401  (world size 1, in this process)
    out = _accum_worker(0, 1, bucket_mb)
    expect1 = _accum_expect(1)
    for n, v in expect1.items():
        assert torch.allclose(out[n], v, rtol=1e-5, atol=1e-6), n


def _bench_worker(rank, world, cfg_path):
    """bench.main's world > 1 branch on a 2-rank gloo group (CPU): barrier-bracketed timed steps,
    max-over-ranks time, one JSON line from rank 0."""
    import contextlib
    import io
    import json
    import bench
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.main(["--gpus", str(world), "--steps", "2", "--warmup", "1", "--batch", "1", "--config", cfg_path,
                    "--device", "cpu", "--no-cpu-baseline", "--no-kernel-timer"])
    lines = [ln for ln in buf.getvalue().splitlines() if ln.startswith("{")]
    return {"lines": [json.loads(ln) for ln in lines]}


def test_bench_main_two_ranks_gloo(tmp_path):
    """The driver's N > 1 launch of bench.py (one process per device, WORLD_SIZE 2) on a tiny 64-px
    stage-0 config: both ranks run the same iteration; only rank 0 prints, value = images of all ranks
    / the max-over-ranks time, parallelism dp2."""
    import json
    import yaml
    import net_cases
    vfm = tmp_path / net_cases.VFM_DIRNAME
    vfm.mkdir()
    json.dump(dict(net_cases.SIGLIP_CFG, layer_norm_eps=1e-6), open(vfm / "config.json", "w"))
    gk = net_cases.g_kwargs(str(vfm))
    gk.pop("img_resolution")
    gk.update(class_name="networks.generator.Generator")
    lk = dict(net_cases.loss_kwargs(str(vfm)), class_name="training.loss.TotalLoss",
              patchgan_discriminator_loss_weight=0.0,
              feature_matching_loss_weight=0.0)
    dk = dict(net_cases.D_KWARGS, class_name="networks.discriminator.ProjectedDiscriminator",
              use_patchgan_discriminator=False, get_interm_feat=False)
    opt = dict(class_name="torch.optim.Adam", lr=1e-4, betas=[0.0, 0.99], eps=1e-8)
    cfg = dict(random_seed=42, training_set_kwargs=dict(class_name="training.data_synthetic.SyntheticDataset",
                                                        resolution=64, conditional=False, label_type="cls2text"),
               G_kwargs=gk, D_kwargs=dk, loss_kwargs=lk, G_opt_kwargs=opt, D_opt_kwargs=opt, batch_size=2,
               ema_kimg=10.0, ema_rampup=None, cudnn_benchmark=False)
    path = tmp_path / "tiny.yaml"
    path.write_text(yaml.safe_dump(cfg))
    res = _spawn("_bench_worker", 2, str(path))
    assert res[1]["lines"] == []
    (line,) = res[0]["lines"]
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "dp2" and line["steps"] == 2
    assert line["config"]["global_batch"] == 2 and line["value"] > 0
    assert abs(line["value"] - 2 * 2 / (line["ms_per_step"] * 2 / 1e3)) / line["value"] < 1e-2


def _safety_worker(rank, world):
    """TotalLoss._sync_safety at world 2: a rank's unsafe mark reaches every rank when the check ran
    (checked=True); with checked=False (no rank ran it) each rank keeps its own values with no collective."""
    from training.loss import TotalLoss
    obj = TotalLoss.__new__(TotalLoss)
    obj.device = torch.device("cpu")
    marks = [1, 1, 1]
    mine = [1, 0, 1] if rank == 1 else marks
    skip, got = obj._sync_safety(rank == 1, mine, checked=True)
    skip2, got2 = obj._sync_safety(False, marks, checked=False)
    return {"skip": skip, "marks": got, "skip2": skip2, "marks2": got2}


def test_sync_safety_agrees_only_when_checked():
    res = _spawn("_safety_worker", 2)
    for r in range(2):
        assert res[r]["skip"] is True and res[r]["marks"] == [1, 0, 1]
        assert res[r]["skip2"] is False and res[r]["marks2"] == [1, 1, 1]
