"""A phase's Adam step (+ the G_ema lerp of the same parameters) as one launch of csrc/adam.hip.

Replaces, on ROCm, the reference's `phase.opt.step()` (training/training_loop.py:722-732, torch.optim.Adam) and the
G_ema update `p_ema.copy_(p.detach().lerp(p_ema, ema_beta))` (:734-742) for the parameters the phase stepped.
The moment buffers are the optimizer's own state tensors (exp_avg / exp_avg_sq) and its per-parameter `step`
tensors are advanced as torch's fused path advances them, so `opt.state_dict()`, a later regular `opt.step()` and
checkpoints see the same state either way. The tensor / chunk tables live on the device and are rebuilt only when
the parameter set or a tensor's storage changes (`AdamEmaPlan`), so a step costs one launch and a multi-tensor
add on the step counters. A plan built without gradients (`grads=None`) takes the gradient tensors per step
(`step(..., raw=grads, gscale=gain)`: FlatGradSync's direct mode, where autograd's own gradient tensors are used
without a gather into a flat buffer): their addresses are uploaded with the launch, and the kernel applies the
gain and nan_to_num that FlatGradSync.finish() applies to the flat buffer (reference training_loop.py:281-289).
"""
import numpy as np
import torch

from .. import custom_ops
from . import kernel_timer

_lib = custom_ops.get_native()


class AdamEmaPlan:
    """Device tables of one parameter set: records (p, g, m, v, ema, n, vec) and the (tensor, chunk) list."""

    def __init__(self, params, grads, m1, m2, emas, steps=None):
        """steps: the optimizer's per-parameter step tensors (fp32 scalars on the device), advanced by 1 inside
        each launch (else the caller advances them)."""
        dev = params[0].device
        self.raw = grads is None
        if grads is None:
            grads = [None] * len(params)
        ch = int(_lib.vfm_adam_chunk_elems())
        rec = np.zeros((len(params), 8), dtype=np.int64)
        chunks = []
        self.nbytes = 0
        for i, (p, g, m, v, e) in enumerate(zip(params, grads, m1, m2, emas)):
            ts = (p,) + ((g,) if g is not None else ()) + (m, v) + ((e,) if e is not None else ())
            for t in ts:
                if t.dtype != torch.float32 or not t.is_contiguous() or t.device != dev or t.numel() != p.numel():
                    raise custom_ops.NativeError("adam_hip: fp32 contiguous tensors of equal size on one device expected")
            n = p.numel()
            ptrs = [t.data_ptr() for t in ts]
            rec[i, :5] = [p.data_ptr(), g.data_ptr() if g is not None else 0, m.data_ptr(), v.data_ptr(),
                          e.data_ptr() if e is not None else 0]
            rec[i, 5] = n
            rec[i, 6] = int(n % 4 == 0 and all(q % 16 == 0 for q in ptrs))
            if steps is not None:
                s_ = steps[i]
                if s_.dtype != torch.float32 or s_.device != dev or s_.numel() != 1:
                    raise custom_ops.NativeError("adam_hip: fp32 device step counters expected")
                rec[i, 7] = s_.data_ptr()
            chunks.extend((i, c) for c in range(-(-n // ch)))
            self.nbytes += n * (28 + (8 if e is not None else 0))
        self.tensors = torch.from_numpy(rec.view(np.uint8).reshape(-1)).to(dev)
        self.chunks = torch.from_numpy(np.asarray(chunks, dtype=np.int32).reshape(-1)).to(dev)
        self.ntensors, self.nchunks = len(params), len(chunks)
        self.keep = (params, grads, m1, m2, emas, steps)   # the tables hold raw pointers into these
        self.owns_steps = steps is not None
        self._raw_ptrs, self._graw = None, None       # last uploaded raw-gradient addresses and their device array

    def step(self, lr, beta1, beta2, weight_decay, eps, step, ema_w=0.0, raw=None, gscale=1.0):
        """raw: this step's gradient tensors (plans built with grads=None; contiguous fp32 of the parameters'
        sizes on their device -- what autograd hands a parameter), used as nan_to_num(g * gscale)."""
        bc1 = 1.0 - beta1 ** step
        bc2_sqrt = (1.0 - beta2 ** step) ** 0.5
        dev = self.tensors.device
        if self.raw != (raw is not None) or (raw is not None and len(raw) != self.ntensors):
            raise custom_ops.NativeError("adam_hip: raw gradients go with plans built without gradients, one per tensor")
        gptr = 0
        if raw is not None:
            ptrs = list(map(torch.Tensor.data_ptr, raw))
            if ptrs != self._raw_ptrs:
                # pinned staging + stream-ordered copy (the caching host allocator keeps the staging buffer until
                # the copy has run); the device array is kept for later steps whose gradients land at the same
                # addresses (the caching allocator's usual pattern), which then skip the upload
                host = torch.empty(self.ntensors, dtype=torch.int64, pin_memory=True)
                host.numpy()[:] = ptrs
                self._graw = host.to(dev, non_blocking=True)
                self._raw_ptrs = ptrs
            gptr = self._graw.data_ptr()
        with kernel_timer.region("adam_ema", self.nbytes):
            custom_ops.check(_lib.vfm_adam_ema_step_raw(self.tensors.data_ptr(), self.ntensors, self.chunks.data_ptr(),
                                                        self.nchunks, gptr, float(gscale), int(raw is not None),
                                                        float(lr), float(beta1), float(beta2), float(weight_decay),
                                                        float(eps), bc1, bc2_sqrt, float(ema_w),
                                                        custom_ops.stream_ptr(dev)), "vfm_adam_ema_step_raw")
