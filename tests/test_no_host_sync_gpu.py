"""No blocking host-device synchronisation inside the training iteration.

The benchmark iteration (BASELINE configs[1]: stage-0 SigLIP2-L at batch 8, every equivariance outcome once warm)
runs under torch's CUDA sync debug mode ("warn"): every call that blocks the host on the GPU -- a pageable
host-to-device copy such as torch.tensor(..., device=cuda), .item() / .tolist() / .cpu() of a device tensor, an
index_put_ with device indices, a stream synchronisation -- warns. A blocking call drains the GPU queue before the
host can issue more work (37 of them per iteration cost ~4 % of the step, profiles/r6_bv_host_syncs.txt), so the
list must stay empty. The loss-safety checks that read losses on the host are scheduled after
safe_loss_checking_start_nimg and are not part of this window (cur_nimg stays below it here)."""
import os
import traceback
import warnings

import pytest
import torch
import yaml

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


class _sync_watch:
    """Collects the call sites of the synchronising calls torch's sync debug mode reports inside the block."""

    def __enter__(self):
        self.hits = []
        self._cw = warnings.catch_warnings()
        self._cw.__enter__()
        warnings.simplefilter("always")
        warnings.showwarning = self._hook
        torch.cuda.set_sync_debug_mode("warn")
        return self.hits

    def _hook(self, message, category, filename, lineno, file=None, line=None):
        if "synchroniz" not in str(message).lower() or "prototype" in str(message):
            return
        frames = [f"{os.path.relpath(f.filename, ROOT)}:{f.lineno}" for f in traceback.extract_stack()
                  if ROOT in f.filename and "tests" not in f.filename]
        self.hits.append(" < ".join(frames[-3:][::-1]) or "(test)")

    def __exit__(self, *exc):
        torch.cuda.set_sync_debug_mode("default")
        self._cw.__exit__(*exc)
        return False


def test_sync_watch_sees_a_blocking_copy():
    """The detector itself: a pageable host-to-device copy and a device .item() are reported."""
    with _sync_watch() as hits:
        torch.tensor(1.0, device=DEV)
        float(torch.ones((), device=DEV).item())
    assert len(hits) >= 2, hits


def test_stage0_iteration_has_no_host_sync():
    from train import resolve_config
    from training.training_loop import configure_backends, construct_networks, construct_iteration
    c = resolve_config(yaml.safe_load(open(os.path.join(PKG, "configs", "vfm_vae_f16d32_siglip2_stage_0_synthetic.yaml"))))
    configure_backends(c.get("cudnn_benchmark", True))
    torch.manual_seed(0)
    batch = 8
    G, G_ema, D = construct_networks(c.G_kwargs, c.D_kwargs, DEV)
    step = construct_iteration(G, D, G_ema, DEV, c.loss_kwargs, c.G_opt_kwargs, c.D_opt_kwargs, batch_size=batch,
                               ema_kimg=c.ema_kimg, ema_rampup=c.ema_rampup)
    g = torch.Generator().manual_seed(0)
    img = (torch.randint(0, 256, (batch, 3, 256, 256), dtype=torch.uint8, generator=g).float() / 255.).to(DEV)
    labels = ["a photo"] * batch
    eqt = step.G.equivariance_transform
    for i, v in enumerate(eqt.variants()):          # every shape class and the optimizer state created first
        eqt.forced = v
        step([img], [labels], i * batch)
    eqt.forced = None
    for i in range(2):
        step([img], [labels], (10 + i) * batch)
    torch.cuda.synchronize()
    with _sync_watch() as hits:
        for i in range(3):
            step([img], [labels], (20 + i) * batch)
    torch.cuda.synchronize()
    assert not hits, "blocking host-device synchronisations in the iteration:\n" + "\n".join(sorted(set(hits)))
