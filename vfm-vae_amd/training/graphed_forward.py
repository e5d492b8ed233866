"""The D phase's no-grad generator forward replayed from HIP graphs.

The reference runs `with torch.no_grad(): self.run_G(real_img, real_c)` eagerly
(training/loss.py:254-256 of the reference; here `TotalLoss.accumulate_gradients`,
phase 'D'). On MI355X that pass (SigLIP2 tower + LDM adapter + decoder) issues a few
thousand launches, and at the low-resolution decoder blocks the host cannot issue them
as fast as the GPU retires them. This runner captures the whole pass once per
equivariance outcome (scale, quarter turns, is_prior) and input shape, then replays it:
one hipGraphLaunch instead of thousands of Python-side launches.

What stays identical to the eager pass:
  * python `random` draws of the equivariance transform are made here, before the
    replay, in the same order (`EquivarianceTransform.forward`);
  * the posterior noise is still drawn with `torch.randn` on the CPU (the order and
    shapes the eager `DiagonalGaussianDistribution.sample()` uses) and copied into the
    graph's static noise buffers through a pinned staging tensor;
  * parameters are read live by the captured kernels, and weight casts are recomputed
    inside the graph (`decoder_hip._cast_cached` does not cache while a capture is in
    progress), so optimizer steps between replays are seen;
  * module buffers mutated by the forward (mapping `x_avg`) are updated in the graph.
The eager warm-up run that precedes each capture has its buffer side effects undone.

All outcomes are captured at the first call, so no capture lands in a later (timed)
step. An outcome whose eager forward raises (e.g. a 1/4-scale latent too small for the
decoder's unshuffle at a toy resolution) is left uncaptured and runs eagerly if drawn,
raising exactly as the eager pass would. Outputs (`gen_img` and the loss terms) live in
the graphs' shared memory pool and are valid until the next replay, which is all the D
phase needs. A failed capture turns the runner off (eager from then on), with the
reason kept in `self.disabled`. Generators with a vector quantiser (discrete latent,
config 4) always run eagerly (`_has_host_state`).
"""
import torch

from networks.utils import kl_utils
from torch_utils.ops import kernel_timer

_UNAVAILABLE = object()


class GraphedNoGradForward:
    def __init__(self, G):
        self.G = G
        self.graphs = {}        # (outcome, img shape, img dtype, training) -> _Entry | _UNAVAILABLE
        self.pool = None
        self.disabled = None    # reason string once capture has been given up
        self.replays = 0

    def eligible(self, img, c):
        return (self.disabled is None and img.is_cuda and getattr(self.G, 'c_dim', 0) == 0
                and not torch.is_grad_enabled() and not self._has_host_state())

    def _has_host_state(self):
        """Modules whose forward branches on Python-side state that changes between calls
        (VectorQuantizer.vocab_usage_record_times selects the usage-EMA rate) or issues a
        collective (the usage bincount all_reduce under DDP) must stay eager: a replay would
        freeze the branch taken at capture time and re-run a captured collective."""
        cached = getattr(self, '_host_state', None)
        if cached is None:
            from networks.utils.quant_utils import VectorQuantizer
            cached = any(isinstance(m, VectorQuantizer) for m in self.G.modules())
            self._host_state = cached
        return cached

    def _key(self, outcome, img):
        return (tuple(outcome), tuple(img.shape), img.dtype, self.G.training)

    def __call__(self, img, c):
        if not self.eligible(img, c):
            return self.G(img, c)
        G = self.G
        outcome = G.equivariance_transform(validation=False)      # same python-random draws as forward()
        key = self._key(outcome, img)
        if key not in self.graphs:
            try:
                for o in G.equivariance_transform.outcomes():
                    k = self._key(o, img)
                    if k not in self.graphs:
                        self.graphs[k] = self._capture(o, img, c)
            except Exception as e:  # noqa: BLE001 - a failed capture means "run eagerly from now on"
                self.disabled = f"{type(e).__name__}: {e}"
                self.graphs.clear()
                torch.cuda.synchronize()
        ent = self.graphs.get(key, _UNAVAILABLE)
        if ent is _UNAVAILABLE:
            return self._eager(outcome, img, c)
        return ent.replay(img)

    def _eager(self, outcome, img, c):
        et = self.G.equivariance_transform
        prev, et.forced = et.forced, tuple(outcome)
        try:
            return self.G(img, c)
        finally:
            et.forced = prev

    def _warm(self, outcome, img, c):
        """One eager run on a side stream (library handles, kernel loads, caches); buffers
        restored afterwards. Returns the noise shapes drawn, or None if the outcome raises."""
        G = self.G
        shapes = []

        def source(shape):
            shapes.append(tuple(shape))
            return torch.zeros(shape)

        saved = {n: b.detach().clone() for n, b in G.named_buffers()}
        dev = img.device
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        prev_src = kl_utils._noise_source
        kl_utils.set_noise_source(source)
        try:
            with torch.cuda.stream(side):
                self._eager(outcome, img, c)
        except RuntimeError:
            shapes = None
        finally:
            kl_utils.set_noise_source(prev_src)
            torch.cuda.current_stream(dev).wait_stream(side)
            torch.cuda.synchronize(dev)
            with torch.no_grad():
                for n, b in G.named_buffers():
                    b.copy_(saved[n])
        return shapes

    def _capture(self, outcome, img, c):
        G = self.G
        served = []

        def source(shape):
            b = bufs[len(served)]
            if tuple(b.shape) != tuple(shape):
                raise RuntimeError("noise draws differ between warm-up and capture")
            served.append(b)
            return b

        static_img = img.detach().clone()
        with kernel_timer.suspended():
            shapes = self._warm(outcome, static_img, c)
            if shapes is None:
                return _UNAVAILABLE
            # static noise inputs are allocated outside the capture: memory of the graph's own
            # pool is recycled between its nodes and would be overwritten during the replay
            bufs = [torch.empty(s, device=img.device) for s in shapes]
            if self.pool is None:
                self.pool = torch.cuda.graph_pool_handle()
            graph = torch.cuda.CUDAGraph()
            et = G.equivariance_transform
            prev_forced, et.forced = et.forced, tuple(outcome)
            prev_src = kl_utils._noise_source
            kl_utils.set_noise_source(source)
            try:
                with torch.cuda.graph(graph, pool=self.pool):
                    out = G(static_img, c)
            finally:
                kl_utils.set_noise_source(prev_src)
                et.forced = prev_forced
        if len(served) != len(bufs):
            raise RuntimeError("noise draws differ between warm-up and capture")
        vfm = getattr(G.vfm_encoder, 'last_features', None) if G.vfm_encoder.reuse_features else None
        return _Entry(graph, static_img, bufs, out, self, vfm)


class _Entry:
    def __init__(self, graph, static_img, bufs, out, owner, vfm=None):
        self.graph, self.static_img, self.bufs, self.out, self.owner = graph, static_img, bufs, out, owner
        self.vfm = vfm          # (input transform, features, pooled): the captured tower outputs
        self.pinned = [torch.empty(b.shape, dtype=b.dtype, pin_memory=True) for b in bufs]
        self.copied = None      # event after the last host->device noise copy

    def replay(self, img):
        if self.copied is not None:
            self.copied.synchronize()           # the pinned staging buffers are free again
        for b, p in zip(self.bufs, self.pinned):
            p.copy_(torch.randn(b.shape))       # CPU RNG, same draws as the eager sample()
            b.copy_(p, non_blocking=True)
        if self.bufs:
            self.copied = torch.cuda.Event()
            self.copied.record()
        self.static_img.copy_(img)
        self.graph.replay()
        self.owner.replays += 1
        if self.vfm is not None:
            # the captured tower outputs are static buffers that the next replay overwrites: hand out
            # copies, so features offered for one microbatch (VFMEncoder.offer_features keeps one entry
            # per microbatch) are not replaced by a later microbatch's replay
            self.owner.G.vfm_encoder.last_features = _clone_tree(self.vfm)
        return self.out


def _clone_tree(x):
    if isinstance(x, torch.Tensor):
        return x.clone()
    if isinstance(x, (list, tuple)):
        return type(x)(_clone_tree(v) for v in x)
    return x
