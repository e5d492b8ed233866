"""Main training loop.

Same entry point and keyword surface as the reference
`training/training_loop.py:training_loop(**c)` (:462-881): phase loop D then G,
gradient accumulation, gradient synchronisation with mean/gain/nan_to_num
semantics (reference sync_grads :281-289), Adam per phase, G_ema update
(:734-742), ticks, stats.jsonl, snapshots `network-snapshot-{kimg:08d}.pth`
with keys {G, D, G_ema, training_set_kwargs} (:782-801) and auto-resume.

MI355X-specific execution (`TrainingIteration`, shared with bench.py):
  * gradients of each phase live in ONE flat fp32 buffer (parameter .grad are
    views), so the reduction, /world, *gain and nan_to_num are single passes;
    on one GPU without a collective (the bench) the gradients stay the tensors
    autograd allocated and the fused Adam kernel applies *gain and nan_to_num
    as it reads them (FlatGradSync direct mode);
  * with world_size > 1 the buffer is all-reduced in buckets launched from
    post-accumulate-grad hooks on a dedicated stream, overlapping the backward
    (RCCL over xGMI); the math equals the reference's flat sharded all-reduce;
  * Adam runs fused (one multi-tensor kernel) when on a GPU;
  * the EMA update is one multi-tensor lerp over the parameters that can change
    (frozen VFM weights are bit-identical in G and G_ema, so their EMA
    p.lerp(p_ema, beta) is the identity and is not recomputed).
"""
import copy
import gc
import json
import math
import operator
import os
import random
import time
from typing import Optional

import numpy as np
import torch
import torch.nn as nn

import dnnlib
from torch_utils import misc
from torch_utils import training_stats
from torch_utils import distributed as dist
from torch_utils.ops import conv2d_gradfix


# ---------------------------------------------------------------------------
# Gradient synchronisation over a flat buffer.


class FlatGradSync:
    """Owns the .grad storage of the trainable parameters of one phase.

    Gradient accumulation: non-last microbatches leave each parameter's (stolen) gradient in place;
    the last microbatch's hooks launch the bucket all-reduces, finish() launches the buckets whose
    parameters the last microbatch did not touch (tests/test_distributed.py covers two microbatches
    with parameters seen in only one of them). The rank-agreement check on the parameter set runs
    without a host sync and therefore raises one step late, at the next prepare(): by then Adam has
    applied one step of the divergent gradients.

    Direct mode (a GPU, no collective, the native Adam: `self.direct`): no flat buffer, hooks or
    gather -- each parameter keeps the gradient tensor autograd allocated (or accumulated into,
    over microbatches), finish() only records the gain (`self.raw`), and fast_adam_step hands the
    gain and nan_to_num to the Adam kernel, which applies them as it reads the gradients
    (csrc/adam.hip vfm_adam_ema_step_raw: the same float multiply and clamp as the flat passes).
    Whatever else steps the phase calls materialize() first, which applies them in place."""

    def __init__(self, module: nn.Module, bucket_mb: float = 64.0, collective: Optional[bool] = None):
        self.module = module
        self.bucket_mb = bucket_mb
        self.world = dist.get_world_size()
        # collective=True runs the bucketed all-reduce path (comm stream, hooks, agreement check)
        # even at world size 1 (an initialised 1-rank process group): how the RCCL path is
        # exercised on a single GPU (tests/test_distributed_gpu.py)
        self.collective = self.world > 1 if collective is None else bool(collective)
        self.params = []
        self.key = None
        self.hooks = []
        self.comm_stream = None
        self.direct = False
        self.raw = None

    def _build(self, params):
        for h in self.hooks:
            h.remove()
        self.hooks = []
        self.params = params
        self.key = tuple(id(p) for p in params)
        self.direct = params[0].device.type == 'cuda' and not self.collective and HIP_ADAM and DIRECT_GRADS
        if self.direct:
            self.flat = None
            return
        order = list(reversed(params))              # gradients of late layers arrive first
        total = sum(p.numel() for p in order)
        dev = params[0].device
        self.flat = torch.zeros(total, dtype=torch.float32, device=dev)
        self.offsets = {}
        off = 0
        for p in order:
            self.offsets[id(p)] = (off, p.numel())
            off += p.numel()
        limit = max(1, int(self.bucket_mb * 2 ** 20 / 4))
        self.buckets = []                           # (start, end, n_params)
        start, n, cnt = 0, 0, 0
        self.bucket_of = {}
        self.bucket_params = [[]]
        for p in order:
            self.bucket_of[id(p)] = len(self.buckets)
            self.bucket_params[-1].append(p)
            n += p.numel()
            cnt += 1
            if n >= limit:
                self.buckets.append((start, start + n, cnt))
                self.bucket_params.append([])
                start, n, cnt = start + n, 0, 0
        if cnt:
            self.buckets.append((start, start + n, cnt))
        else:
            self.bucket_params.pop()
        self.views = {id(p): self.flat[self.offsets[id(p)][0]:self.offsets[id(p)][0] + p.numel()].view_as(p)
                      for p in params}
        if dev.type == 'cuda' and self.collective:
            self.comm_stream = torch.cuda.Stream(device=dev)
        for p in params:
            self.hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    def prepare(self):
        """Call after requires_grad is set for the phase, before the first backward."""
        # the module's parameter list is walked once (module.parameters() recurses through every
        # submodule: ~2-3 ms of host time per call with the GPU queue at its shortest, r4k gap profile)
        allp = self.__dict__.get('_all_params')
        if allp is None:
            allp = self._all_params = list(self.module.parameters())
        params = [p for p in allp if p.requires_grad and p.dtype == torch.float32]
        if not params:
            self.params = []
            return
        if tuple(id(p) for p in params) != self.key:
            self._build(params)
        self.raw = None
        if self.direct:
            for p in self.params:
                p.grad = None
            return
        self.flat.zero_()
        # grads start as None: the autograd engine then hands each parameter its gradient tensor
        # without a kernel (AccumulateGrad "steals" it), and the grads move into the flat buffer
        # with one multi-tensor copy per bucket (or per phase at world size 1) instead of one
        # accumulate kernel per parameter
        for p in self.params:
            p.grad = None
        self.seen = set()
        self.staged = []
        self.ready = [0] * len(self.buckets)
        self.pending = {}
        self.last_microbatch = True
        self.late = False
        self._check_agreement()

    def _check_agreement(self):
        """Verify (one phase late, without a host sync on the step) that every rank produced
        gradients for the same parameter set in the previous step of this phase. A parameter
        whose grad is None on some ranks only would be stepped by Adam on those ranks alone
        and the replicas would drift silently (the reference fails with mismatched
        all-reduce sizes instead)."""
        chk = getattr(self, '_agree', None)
        self._agree = None
        if chk is None:
            return
        host, event = chk
        if event is not None:
            event.synchronize()
        if int(host[0]) != 0:
            raise RuntimeError("FlatGradSync: ranks produced gradients for different parameter sets in the "
                               "previous step (replicas would diverge)")

    def _launch_agreement(self):
        mask = torch.tensor([id(p) in self.seen for p in self.params], dtype=torch.int32)
        dev = self.flat.device
        mask = mask.pin_memory().to(dev, non_blocking=True) if dev.type == 'cuda' else mask
        tot = mask.clone()
        torch.distributed.all_reduce(tot)
        bad = ((tot != 0) & (tot != self.world)).any().to(torch.int32).reshape(1)
        if dev.type == 'cuda':
            host = torch.empty(1, dtype=torch.int32, pin_memory=True)
            host.copy_(bad, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._agree = (host, ev)
        else:
            self._agree = (bad, None)

    def _on_grad(self, p):
        self.seen.add(id(p))
        if not self.collective:
            # world size 1: gather in chunks while the backward is still running (host work and the
            # multi-tensor copies overlap the GPU instead of trailing it in finish())
            self.staged.append(p)
            if len(self.staged) >= 64:
                self._gather(self.staged)
                self.staged = []
            return
        if not self.last_microbatch:
            return
        bi = self.bucket_of[id(p)]
        if bi in self.pending:              # a second backward touched a bucket already in flight
            self.late = True
            return
        self.ready[bi] += 1
        if self.ready[bi] == self.buckets[bi][2]:
            self._launch(bi)

    def _gather(self, plist):
        """Move the stolen gradients of `plist` into their flat-buffer views (one multi-tensor copy)
        and point .grad at the views."""
        dst, src = [], []
        for p in plist:
            g, v = p.grad, self.views[id(p)]
            if g is None or g.data_ptr() == v.data_ptr():
                continue
            dst.append(v)
            src.append(g)
        if dst:
            torch._foreach_copy_(dst, src)
            for p in plist:
                if p.grad is not None:
                    p.grad = self.views[id(p)]

    def _launch(self, bi):
        self._gather(self.bucket_params[bi])
        s, e, _ = self.buckets[bi]
        view = self.flat[s:e]
        if self.comm_stream is not None:
            self.comm_stream.wait_stream(torch.cuda.current_stream(self.flat.device))
            with torch.cuda.stream(self.comm_stream):
                self.pending[bi] = torch.distributed.all_reduce(view, async_op=True)
        else:
            self.pending[bi] = torch.distributed.all_reduce(view, async_op=True)

    def finish(self, gain: Optional[float] = None):
        """Complete the reduction: flat = nan_to_num(sum_ranks / world * gain) (direct mode: deferred to the
        optimizer step, see materialize())."""
        if not self.params:
            return
        if self.direct:
            self.raw = 1.0 if gain is None else float(gain)
            return
        if self.collective:
            for bi in range(len(self.buckets)):
                if bi not in self.pending:
                    self._launch(bi)
            for bi in sorted(self.pending):
                self.pending[bi].wait()
            if self.late:
                raise RuntimeError("FlatGradSync: more than one backward pass in the last microbatch of a phase "
                                   "(gradients changed under an in-flight all-reduce)")
            if self.comm_stream is not None:
                torch.cuda.current_stream(self.flat.device).wait_stream(self.comm_stream)
            self._launch_agreement()
            self.flat.mul_(1.0 / self.world)
        else:
            self._gather(self.staged)
            self.staged = []
        if gain is not None and gain != 1:
            self.flat.mul_(gain)
        torch.nan_to_num_(self.flat, nan=0, posinf=1e5, neginf=-1e5)
        for p in self.params:   # parameters that produced no gradient keep grad=None (Adam skips them)
            if id(p) not in self.seen:
                p.grad = None

    def materialize(self):
        """Direct mode: apply the pending gain and nan_to_num to the gradients in place (for an optimizer step
        other than the native fused one)."""
        if self.raw is None:
            return
        gain, self.raw = self.raw, None
        grads = [p.grad for p in self.params if p.grad is not None]
        with torch.no_grad():
            if grads and gain != 1:
                torch._foreach_mul_(grads, gain)
            for g in grads:
                torch.nan_to_num_(g, nan=0, posinf=1e5, neginf=-1e5)


_VERSION = operator.attrgetter('_version')
HIP_ADAM = os.environ.get("VFM_ADAM", "hip") == "hip"      # VFM_ADAM=torch: torch's fused Adam + foreach lerp (A/B)
DIRECT_GRADS = os.environ.get("VFM_DIRECT_GRADS", "1") == "1"  # 0: flat-buffer gradients at world size 1 too (A/B)


def fast_adam_step(phase, ema=None):
    """torch.optim.Adam(fused=True).step() without its per-step Python bookkeeping: after one regular
    step has created the state, the tensor lists of the parameters that have gradients are cached per
    parameter set. On ROCm the step is one launch of csrc/adam.hip over device tables built once per set
    (torch_utils/ops/adam_hip.py: torch's fused arithmetic), which also applies the G_ema lerp to the
    parameters `ema` = (pairs, weight) maps (pairs: {id(p): p_ema}); elsewhere (or VFM_ADAM=torch) the same
    two calls torch's fused path makes (`_foreach_add_` on the step counters, `_fused_adam_`). Returns False
    (nothing done: the caller runs opt.step()) for anything but a single fp32 group of plain fused Adam with
    float hyper-parameters, or on the first step of a parameter set (the regular path creates state); else
    the set of ids of the parameters whose EMA it applied. The regular step loops over every parameter
    checking grads, state and dtypes: ~2-4 ms of host time per phase with the GPU idle (r4k gap profile).
    With the phase's FlatGradSync in direct mode (gradients pending gain / nan_to_num, `sync.raw`) the native
    step applies them; every other outcome materializes them first (the caller's opt.step() included)."""
    sync = getattr(phase, 'sync', None)
    gain = getattr(sync, 'raw', None)
    opt = phase.opt
    if type(opt) is not torch.optim.Adam or len(opt.param_groups) != 1:
        return _materialized(sync, False)
    g = opt.param_groups[0]
    if not g.get('fused') or g.get('amsgrad') or g.get('capturable') or g.get('differentiable') or \
            g.get('maximize') or g.get('foreach') or g.get('decoupled_weight_decay') or \
            isinstance(g['lr'], torch.Tensor) or \
            any(isinstance(b, torch.Tensor) for b in g['betas']):
        return _materialized(sync, False)
    plist = getattr(phase, 'adam_params', None)     # (phases are EasyDicts: attributes are items)
    if plist is None:
        plist = phase.adam_params = list(g['params'])
    now = [p.grad for p in plist]                       # the one Python pass over the parameters
    raw = gain is not None
    # cache key: the gradient tensors themselves (flat-buffer views persist across steps), or with raw
    # gradients (new tensors every step) which parameters have one
    key = [gr is None for gr in now] if raw else now
    pairs = ema[0] if ema is not None else None
    cache = getattr(phase, 'adam_cache', None)
    st = opt.state
    if (cache is not None and cache[6] is pairs and cache[8] == raw
            and (key == cache[0] if raw else all(map(operator.is_, now, cache[0])))
            and st[cache[1][0]]['exp_avg'] is cache[3][0] and st[cache[1][-1]]['exp_avg_sq'] is cache[4][-1]):
        _, params, grads, m1, m2, steps, _, plan, _ = cache
    else:
        phase.adam_rebuilds = getattr(phase, 'adam_rebuilds', 0) + 1       # (tools_dev/adam_cache_debug.py)
        with_grad = [p for p, gr in zip(plist, now) if gr is not None]
        if not with_grad:
            return _materialized(sync, set())
        dev = with_grad[0].device
        if any(p not in st or p.dtype != torch.float32 or p.device != dev or p.grad.dtype != torch.float32
               for p in with_grad):
            phase.adam_cache = None
            return _materialized(sync, False)   # first step of these parameters: the regular path creates state
        params, grads = with_grad, [p.grad for p in with_grad]
        m1, m2 = [st[p]['exp_avg'] for p in with_grad], [st[p]['exp_avg_sq'] for p in with_grad]
        steps = [st[p]['step'] for p in with_grad]
        plan = None
        if HIP_ADAM and dev.type == 'cuda':
            counts = torch.stack([s.reshape(()) for s in steps]).cpu()
            if bool((counts == counts[0]).all()):
                from torch_utils.ops import adam_hip
                emas = [pairs.get(id(p)) if pairs is not None else None for p in with_grad]
                plan = [adam_hip.AdamEmaPlan(params, None if raw else grads, m1, m2, emas, steps), float(counts[0]),
                        {id(p) for p, e in zip(with_grad, emas) if e is not None}]
        phase.adam_cache = (key, params, grads, m1, m2, steps, pairs, plan, raw)
    if raw:
        grads = [gr for gr in now if gr is not None]
        if plan is not None and not all(map(torch.Tensor.is_contiguous, grads)):
            # (autograd hands contiguous gradients; an assigned .grad may not be): torch's step this time, and the
            # cached plan dropped -- its host step count would fall behind the counters torch advances
            plan = None
            phase.adam_cache = None
        if plan is None:
            sync.materialize()
    beta1, beta2 = g['betas']
    with torch.no_grad():
        if plan is None or not plan[0].owns_steps:
            torch._foreach_add_(steps, 1)
        if plan is not None:                      # (the launch advances the step counters it owns)
            plan[1] += 1.0
            plan[0].step(g['lr'], beta1, beta2, g['weight_decay'], g['eps'], plan[1],
                         ema[1] if ema is not None else 0.0, raw=grads if raw else None,
                         gscale=gain if raw else 1.0)
            if raw:
                sync.raw = None
            return plan[2]
        torch._fused_adam_(params, grads, m1, m2, [], steps, amsgrad=False, lr=g['lr'], beta1=beta1, beta2=beta2,
                           weight_decay=g['weight_decay'], eps=g['eps'], maximize=False, grad_scale=None,
                           found_inf=None)
    return set()


def _materialized(sync, result):
    """fast_adam_step's exits that leave the step to something else: the pending direct-mode gain and
    nan_to_num applied to the gradients first."""
    if sync is not None and getattr(sync, 'raw', None) is not None:
        sync.materialize()
    return result


class TrainingIteration:
    """One optimisation iteration: D phase, G phase, EMA (reference :708-742)."""

    def __init__(self, G, D, G_ema, loss, G_opt, D_opt, batch_size, n_batch_acc=1, ema_kimg=10.0,
                 ema_rampup=0.05, bucket_mb=64.0):
        self.G, self.D, self.G_ema, self.loss = G, D, G_ema, loss
        self.phases = [dnnlib.EasyDict(name='D', module=D, opt=D_opt, sync=FlatGradSync(D, bucket_mb)),
                       dnnlib.EasyDict(name='G', module=G, opt=G_opt, sync=FlatGradSync(G, bucket_mb))]
        self.batch_size = batch_size
        self.n_batch_acc = n_batch_acc
        self.ema_kimg = ema_kimg
        self.ema_rampup = ema_rampup
        self._ema_pairs = None
        self.trace = None          # callable(msg) -> per-phase wall times (synchronising; diagnostics only)

    @staticmethod
    def partial_freeze(phase):
        """Reference :446-459."""
        if phase.name == 'D':
            if 'dino' in phase.module._modules:
                phase.module.dino.requires_grad_(False)
        else:
            phase.module.requires_grad_(False)
            layers = phase.module.trainable_layers
            for name, layer in phase.module.named_modules():
                layer.requires_grad_(any(t in name for t in layers))

    def _apply_freeze(self, phase):
        """partial_freeze() semantics, evaluated once per (phase, trainable_layers) and then
        applied as a flat list of per-parameter flags (the module walk costs milliseconds of
        host time per phase)."""
        key = (phase.name, tuple(getattr(phase.module, 'trainable_layers', ()) or ()))
        cache = phase.setdefault('freeze_cache', {})
        flags = cache.get(key)
        if flags is None:
            phase.module.requires_grad_(True)
            self.partial_freeze(phase)
            flags = [(p, p.requires_grad) for p in phase.module.parameters()]
            cache[key] = flags
        else:
            # the trainable ones were switched off at the end of the phase's last run; the frozen ones only
            # need a call when something switched them on since (attribute reads are ~10x cheaper than the call)
            for p, f in flags:
                if f:
                    p.requires_grad_(True)
                elif p.requires_grad:
                    p.requires_grad_(False)
        phase.active_flags = flags

    def run_phase(self, phase, real_imgs, real_cs, cur_nimg, ema=None):
        """One phase (reference :708-732); `ema` = (pairs, weight) hands the G_ema update of the phase's
        parameters to the fused optimizer step (fast_adam_step). Returns the ids of the parameters whose EMA
        was applied."""
        self._apply_freeze(phase)
        phase.sync.prepare()
        enc = getattr(self.G, 'vfm_encoder', None)
        reuse = enc is not None and getattr(enc, 'reuse_features', False)
        if reuse and phase.name == 'D':
            enc.clear_features()                 # the D phase offers each microbatch's tower features
        n = len(real_imgs)
        for i, (img, c) in enumerate(zip(real_imgs, real_cs)):
            phase.sync.last_microbatch = (i == n - 1)
            self.loss.accumulate_gradients(phase=phase.name, real_img=img, real_c=c, cur_nimg=cur_nimg)
        if reuse and phase.name == 'G':
            enc.clear_features()                 # entries the G phase did not take (other draws) freed
        flags = phase.active_flags
        if phase.sync.params or any(p.grad is not None for p, _ in flags):
            phase.sync.finish(gain=self.n_batch_acc)
        done = fast_adam_step(phase, ema)
        if done is False:
            phase.opt.step()
            done = set()
        # requires_grad_(False) over the flag list of _apply_freeze (a module walk costs ms of host time at the
        # point where the GPU queue is shortest), after the optimizer launch so that it overlaps it
        for p, f in flags:
            if f:
                p.requires_grad_(False)
        phase.opt.zero_grad(set_to_none=True)
        return done

    def _phase_ema(self, phase, cur_nimg):
        """(pairs, lerp weight) for the G phase's fused optimizer step, None otherwise: the EMA of G's stepped
        parameters then rides on that step (the D phase does not change G, so after the G phase's update the
        parameters are the values the reference's end-of-iteration lerp reads)."""
        if phase.name != 'G' or not HIP_ADAM:
            return None
        return self._ema_pair_map(), 1.0 - self._ema_beta(cur_nimg)

    def _ema_beta(self, cur_nimg):
        ema_nimg = self.ema_kimg * 1000
        if self.ema_rampup is not None:
            ema_nimg = min(ema_nimg, cur_nimg * self.ema_rampup)
        return 0.5 ** (self.batch_size / max(ema_nimg, 1e-8))

    def _ema_pair_map(self):
        """{id(p): p_ema} of the current EMA pair list (the same dict object while the list is unchanged)."""
        pairs = self._current_ema_pairs()
        if self.__dict__.get('_ema_map_src') is not pairs:
            self._ema_map = {id(p): pe for pe, p in zip(pairs[1], pairs[2])}
            self._ema_map_src = pairs
        return self._ema_map

    def _current_ema_pairs(self):
        # frozen tensors equal in G and G_ema are left out of the lerp; the pair list is rebuilt when the
        # trainable set changes or any left-out tensor was written since (a checkpoint loaded into one
        # side bumps its version counter), so a frozen tensor that comes to differ is averaged again
        pairs = self._ema_pairs
        # (the version check runs twice a step over the ~400 left-out tensors: one C-level map, not a generator)
        if pairs is not None and (pairs[0] != tuple(self.G.trainable_layers)
                                  or list(map(_VERSION, pairs[4])) != pairs[5]):
            pairs = None
        if pairs is None:
            names = self.G.trainable_layers
            dst, src, same = [], [], []
            for (n, pe), (_, p) in zip(self.G_ema.named_parameters(), self.G.named_parameters()):
                mod = n.rsplit('.', 1)[0]
                if any(t in mod for t in names) or not torch.equal(pe, p):
                    dst.append(pe)
                    src.append(p)
                else:
                    same.append((pe, p, pe._version, p._version))
            flat = [t for pe, p, _, _ in same for t in (pe, p)]
            pairs = self._ema_pairs = (tuple(names), dst, src, same, flat, list(map(_VERSION, flat)))
        return pairs

    @torch.no_grad()
    def update_ema(self, cur_nimg, done=()):
        """G_ema <- lerp toward G (reference :734-742) for the pairs not in `done` (ids of G parameters whose
        EMA the fused G-phase optimizer step already applied), then the changed buffers."""
        beta = self._ema_beta(cur_nimg)
        _, dst, src = self._current_ema_pairs()[:3]
        if done:
            keep = [(d, s_) for d, s_ in zip(dst, src) if id(s_) not in done]
            dst, src = [d for d, _ in keep], [s_ for _, s_ in keep]
        if dst:
            # p_ema <- p.lerp(p_ema, beta) == p_ema + (1 - beta) * (p - p_ema)
            torch._foreach_lerp_(dst, src, 1.0 - beta)
        # buffers are copied only when the source changed since the last copy (version counter):
        # the generator's buffers are constants (noise planes, filters), and copying ~60 of them
        # every step was ~60 launches of nothing
        seen = self.__dict__.setdefault('_ema_buf_versions', {})
        pairs_b = self.__dict__.get('_ema_buf_pairs')
        if pairs_b is None:         # module walks once (they cost ~1 ms each at the end of the step)
            pairs_b = self._ema_buf_pairs = list(zip(self.G_ema.buffers(), self.G.buffers()))
        bufs = []
        for be, b in pairs_b:
            if be.data_ptr() == b.data_ptr():
                continue
            key = (be.data_ptr(), b.data_ptr())
            if seen.get(key) != (b._version, be._version):
                bufs.append((be, b))
        if bufs:
            torch._foreach_copy_([be for be, _ in bufs], [b for _, b in bufs])
            for be, b in bufs:
                seen[(be.data_ptr(), b.data_ptr())] = (b._version, be._version)

    def __call__(self, phase_real_img, phase_real_c, cur_nimg):
        if self.trace is None:
            done = set()
            for phase in self.phases:
                done |= self.run_phase(phase, phase_real_img, phase_real_c, cur_nimg, ema=self._phase_ema(phase, cur_nimg))
            self.update_ema(cur_nimg, done)
            return
        import time
        for phase in self.phases:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            self.loss.trace = self.trace
            self.run_phase(phase, phase_real_img, phase_real_c, cur_nimg)
            self.loss.trace = None
            torch.cuda.synchronize()
            self.trace(f"phase {phase.name}: {time.perf_counter() - t0:.3f}s")
        t0 = time.perf_counter()
        self.update_ema(cur_nimg)
        torch.cuda.synchronize()
        self.trace(f"ema: {time.perf_counter() - t0:.3f}s")


# ---------------------------------------------------------------------------
# Data helpers.


def split(arr, chunk_size, dim=0):
    if isinstance(arr, list):
        return [arr[i:i + chunk_size] for i in range(0, len(arr), chunk_size)]
    return list(torch.split(arr, chunk_size, dim)) if isinstance(arr, torch.Tensor) else \
        np.array_split(arr, int(np.ceil(len(arr) / chunk_size)), dim)


def preprocess_image(image, device):
    return image.to(device, non_blocking=True).to(torch.float32) / 255.


def _sync_all_done(local_done, device):
    """True once any rank's one-epoch stream is exhausted (all ranks stop together)."""
    if dist.get_world_size() == 1:
        return bool(local_done)
    flag = torch.tensor([int(local_done)], dtype=torch.int32, device=device)
    torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MAX)
    return bool(flag.item())


def fetch_data(iterator, device, batch_gpu):
    real_img, real_cs = next(iterator)
    real_img = preprocess_image(real_img, device)
    real_cs = real_cs if isinstance(real_cs[0], str) else real_cs.to(device)
    return split(real_img, batch_gpu), split(real_cs, batch_gpu)


def load_state_dict_with_report(model, state_dict, name="model", strict=False, max_items=10):
    res = model.load_state_dict(state_dict, strict=strict)
    missing, unexpected = list(res.missing_keys), list(res.unexpected_keys)
    dist.print0(f"[resume:{name}] loaded; missing={len(missing)} unexpected={len(unexpected)}")
    for k in missing[:max_items]:
        dist.print0(f"      missing {k}")
    for k in unexpected[:max_items]:
        dist.print0(f"      unexpected {k}")
    return res


def make_optimizer(params, opt_kwargs, device):
    kw = dict(opt_kwargs)
    if device.type == 'cuda' and kw.get('class_name') == 'torch.optim.Adam' and 'fused' not in kw:
        kw['fused'] = True
    params = [p for p in params]
    return dnnlib.util.construct_class_by_name(params=params, **kw)


def configure_backends(cudnn_benchmark=True):
    """Backend switches shared by training_loop() and bench.py (reference :503-506).

    TF32 stays off (gfx950 has no xf32 anyway). `cudnn_benchmark` selects MIOpen's
    exhaustive per-shape convolution search on ROCm; its find-db does not persist between
    fresh boxes and the search takes > 10 minutes for the LPIPS/PatchGAN shapes, so it is
    honoured only with VFM_CUDNN_BENCHMARK=1 (immediate-mode solutions otherwise)."""
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    if torch.version.hip is not None:
        cudnn_benchmark = bool(cudnn_benchmark) and os.environ.get("VFM_CUDNN_BENCHMARK", "0") == "1"
        os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
    torch.backends.cudnn.benchmark = bool(cudnn_benchmark)
    conv2d_gradfix.enabled = True


def construct_networks(G_kwargs, D_kwargs, device, label_dim=0):
    """G (train mode, frozen until a phase unfreezes it), G_ema = deepcopy(G), D (reference :573-575)."""
    G = dnnlib.util.construct_class_by_name(label_dim=label_dim, **G_kwargs)
    G = G.train().requires_grad_(False).to(device)
    G_ema = copy.deepcopy(G).eval()
    D = dnnlib.util.construct_class_by_name(c_dim=G.c_dim, **D_kwargs).train().requires_grad_(False).to(device)
    return G, G_ema, D


def construct_iteration(G, D, G_ema, device, loss_kwargs, G_opt_kwargs, D_opt_kwargs, batch_size,
                        accumulate_gradients=1, ema_kimg=10.0, ema_rampup=0.05, graph_nograd_forward=False,
                        bucket_mb=64.0):
    """TotalLoss + optimisers + the TrainingIteration that train.py and bench.py both run.
    graph_nograd_forward: replay the D phase's no-grad generator forward from HIP graphs
    (training/graphed_forward.py). OFF by default: at the full C1 configuration a replay that
    follows an eager forward run after a decoder weight update reads stale memory
    (tools_dev/graph_c1_debug*.py), so the D phase runs eagerly."""
    loss = dnnlib.util.construct_class_by_name(device=device, G=G, D=D, **loss_kwargs)
    if graph_nograd_forward and device.type == 'cuda':
        loss.enable_graphed_nograd_forward()
    G_opt = make_optimizer(G.parameters(), G_opt_kwargs, device)
    D_opt = make_optimizer(D.parameters(), D_opt_kwargs, device)
    return TrainingIteration(G, D, G_ema, loss, G_opt, D_opt, batch_size=batch_size,
                             n_batch_acc=accumulate_gradients, ema_kimg=ema_kimg, ema_rampup=ema_rampup,
                             bucket_mb=bucket_mb)


def save_snapshot(path, G, D, G_ema, training_set_kwargs):
    torch.save({"G": G.state_dict(), "D": D.state_dict(), "G_ema": G_ema.state_dict(),
                "training_set_kwargs": dict(training_set_kwargs)}, path)


# ---------------------------------------------------------------------------


def training_loop(run_dir='.', training_set_kwargs={}, validation_set_kwargs={}, data_loader_kwargs={},
                  G_kwargs={}, D_kwargs={}, G_opt_kwargs={}, D_opt_kwargs={}, loss_kwargs={}, metrics=[],
                  random_seed=0, batch_size=4, batch_gpu=4, accumulate_gradients=1, ema_kimg=10, ema_rampup=0.05,
                  total_kimg=25000, kimg_per_tick=4, image_snapshot_ticks=50, network_snapshot_ticks=50,
                  resume_path=None, resume_kimg=0, resume_discriminator=True, cudnn_benchmark=True, abort_fn=None,
                  progress_fn=None, one_epoch=False, device=None, train_sample_dir=None, wandb_project_name=None,
                  wandb_run_name=None, max_iterations=None, graph_nograd_forward=False, **_unused):
    device = device or (torch.device('cuda') if torch.cuda.is_available() else torch.device('cpu'))
    start_time = time.time()
    base_seed = random_seed * dist.get_world_size() + dist.get_rank()
    np.random.seed(base_seed)
    torch.manual_seed(base_seed)
    random.seed(base_seed)
    configure_backends(cudnn_benchmark)
    if metrics:
        raise NotImplementedError(f"metrics {metrics}: the FID/IS detectors need URL downloads (reference "
                                  "metrics/), which this offline build does not fetch; set `metrics: []`")

    dist.print0('Loading training set...')
    training_set = dnnlib.util.construct_class_by_name(**training_set_kwargs)
    iterator = iter(training_set.iterate(batch_size=batch_size // dist.get_world_size(), rank=dist.get_rank(),
                                         world=dist.get_world_size(), seed=base_seed))

    dist.print0('Constructing networks...')
    G, G_ema, D = construct_networks(G_kwargs, D_kwargs, device, getattr(training_set, 'label_dim', 0))

    if resume_path is not None and dist.get_rank() == 0:
        ckpt = torch.load(resume_path, map_location=device, weights_only=True)
        if resume_discriminator and "D" in ckpt:
            load_state_dict_with_report(D, ckpt["D"], name="D")
        for key, net in (("G", G), ("G_ema", G_ema)):
            if key in ckpt:
                load_state_dict_with_report(net, ckpt[key], name=key)
    if dist.get_world_size() > 1:
        for module in (G, D, G_ema):
            for t in misc.params_and_buffers(module):
                torch.distributed.broadcast(t, src=0)

    step = construct_iteration(G, D, G_ema, device, loss_kwargs, G_opt_kwargs, D_opt_kwargs, batch_size,
                               accumulate_gradients, ema_kimg, ema_rampup, graph_nograd_forward)
    loss = step.loss

    stats_collector = training_stats.Collector(regex='.*')
    stats_jsonl = open(os.path.join(run_dir, 'stats.jsonl'), 'at') if dist.get_rank() == 0 else None
    cur_nimg = resume_kimg * 1000
    cur_tick = 0
    tick_start_nimg = cur_nimg
    tick_start_time = time.time()
    maintenance_time = tick_start_time - start_time
    batch_idx = 0
    dist.print0(f'Training started at {resume_kimg} kimg.')
    while True:
        try:
            phase_real_img, phase_real_c = fetch_data(iterator, device, batch_gpu)
            exhausted = False
        except StopIteration:
            if not one_epoch:
                raise
            exhausted = True
        if one_epoch and _sync_all_done(exhausted, device):      # reference _sync_all_done :349-353
            dist.print0(f'[one-epoch] data exhausted at {cur_nimg / 1e3:.1f} kimg')
            if dist.get_rank() == 0 and network_snapshot_ticks is not None:
                save_snapshot(os.path.join(run_dir, f'network-snapshot-{cur_nimg // 1000:08d}.pth'), G, D, G_ema,
                              training_set_kwargs)
            break
        step(phase_real_img, phase_real_c, cur_nimg)
        cur_nimg += batch_size
        batch_idx += 1
        if batch_idx == 1:
            gc.collect()
            gc.freeze()          # keep full collections over the long-lived objects out of the step
        done = (cur_nimg >= total_kimg * 1000) or (max_iterations is not None and batch_idx >= max_iterations)
        if not done and cur_tick != 0 and cur_nimg < tick_start_nimg + kimg_per_tick * 1000:
            continue
        tick_end_time = time.time()
        if device.type == 'cuda':
            torch.cuda.synchronize(device)
        tick_time = time.time() - tick_start_time
        sec_per_kimg = tick_time / max(cur_nimg - tick_start_nimg, 1) * 1e3
        training_stats.report0('Timing/total_sec', tick_end_time - start_time)
        training_stats.report0('Timing/sec_per_tick', tick_time)
        training_stats.report0('Timing/sec_per_kimg', sec_per_kimg)
        training_stats.report0('Timing/images_per_sec', 1e3 / max(sec_per_kimg, 1e-9))
        training_stats.report0('Timing/maintenance_sec', maintenance_time)
        dist.print0(f"tick {cur_tick:<5d} kimg {cur_nimg / 1e3:<8.1f} sec/kimg {sec_per_kimg:<7.2f} "
                    f"img/s {1e3 / max(sec_per_kimg, 1e-9):<8.1f} maintenance {maintenance_time:<6.1f}")
        if (network_snapshot_ticks is not None) and (done or cur_tick % network_snapshot_ticks == 0) and cur_tick > 0:
            if dist.get_rank() == 0:
                save_snapshot(os.path.join(run_dir, f'network-snapshot-{cur_nimg // 1000:08d}.pth'), G, D, G_ema,
                              training_set_kwargs)
        stats_collector.update()
        if stats_jsonl is not None:
            stats_jsonl.write(json.dumps(dict(stats_collector.as_dict(), timestamp=time.time())) + '\n')
            stats_jsonl.flush()
        cur_tick += 1
        tick_start_nimg = cur_nimg
        tick_start_time = time.time()
        maintenance_time = tick_start_time - tick_end_time
        if done:
            break
    if stats_jsonl is not None:
        stats_jsonl.close()
    dist.print0('Exiting...')
    return dict(G=G, D=D, G_ema=G_ema, cur_nimg=cur_nimg)
