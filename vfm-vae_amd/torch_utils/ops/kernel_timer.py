"""Per-launch timing of named kernels inside a timed region.

bench.py enables the timer around its timed steps; every native op wrapper
opens a region around its launch and reports the launch's ALGORITHMIC bytes
(unique inputs + outputs + weights at the op boundary) and flops.

Native regions (our kernels) arm a pair of HIP events in the kernel library
(`vfm_timer_arm`, include/vfmvae.h): the library then launches through
hipExtLaunchKernelGGL, which binds the events to the kernel dispatch itself, so a
region's time is the kernels' own duration -- the number rocprofv3's kernel trace
reports -- and not the host launch gaps that events recorded around a launch also
enclose when the stream runs dry. Library GEMM regions (hipBLASLt through torch)
still record events around the call on the launch stream.

`dominant_roofline()` picks the kernel with the largest total time and returns the
bench.py `roofline` object (achieved = algorithmic bytes or flops per launch /
average launch time).
"""
import contextlib
import ctypes
import os

import torch

# VFM_TIMER_SHAPES=1: GEMM regions carry their [MxNxKxz] shape (a breakdown for tuning; the
# bench line's roofline then ranks per shape)
SHAPES = os.environ.get("VFM_TIMER_SHAPES", "0") == "1"

_enabled = False
_records = {}      # name -> list of (start_event, end_event, bytes, flops, bound)
_counts = {}       # name -> launches seen while enabled (timed or not)
_flops_all = {}    # name -> algorithmic flops of every launch seen while enabled (host arithmetic)
_every = 1         # time ~1/n of each region's launches (the events cost host time per launch)


_active = True     # launches are timed only while active (bench.py: every launch of every n-th timed step)
_target = None     # set_target(): the one region counted and timed (bench.py's timed steps); None: all regions
_pos = {}          # name -> launch position within the current step (new_step resets it)
_phase = -1        # index of the current active step (new_step), -1: stepless (launch-index sampling)


def enable(flag: bool, every: int = 1):
    """Timing on / off. The start event is bound to the timed kernel's own dispatch; VFM_TIMER_PROBE=1 binds it
    to the end of an empty probe kernel launched before it instead (vfm_timer_mode, include/vfmvae.h): both read
    the same averages once the fixed per-launch interval is calibrated out (gpurun_out r6q / r6q0), and the
    probe is one more launch per timed launch."""
    if flag:
        _native().vfm_timer_mode(1 if os.environ.get("VFM_TIMER_PROBE", "0") == "1" else 0)
    _enable(flag, every)


def _enable(flag: bool, every: int = 1):
    global _enabled, _every, _active, _phase, _target
    _enabled = bool(flag)
    _active = True
    _phase = -1
    _target = None
    _pos.clear()
    _per_step.clear()
    if flag:
        _records.clear()
        _counts.clear()
        _flops_all.clear()
        _every = max(1, int(every))


_per_step = {}     # name -> launches in the previous stepped step (sets the region's sampling rate)
MIN_SAMPLES = 2    # target timed launches per step and region: rate 1 / clamp(n // MIN_SAMPLES, 1, every)


def new_step(active: bool):
    """Start of one step of the timed loop (bench.py). While stepped, a region's launch at position j of the
    k-th active step is timed when (j + k) % every == 0: STRATIFIED over the launch positions of a step, so
    every position of the step's launch sequence (a region's launches differ in shape: the LPIPS VGG conv's
    13 layers, the decoder's blocks) is timed equally often over `every` active steps. The pseudo-random
    launch-index sample of round 5 carried the shape mix's sampling error: the VGG conv read 426 us by events
    against 619 us in rocprof on the same box (What's weak 6)."""
    global _active, _phase
    _active = bool(active)
    for k, n in _pos.items():
        _per_step[k] = n
    _pos.clear()
    if active:
        _phase += 1


def set_active(flag: bool):
    """While enabled: launches keep being counted, but only those issued while active are timed.
    Timing every launch of whole steps (rather than a sample of each region's launches in every
    step) makes a region's average exact for those steps: its launches differ in shape, so a
    sampled average of them carries the shape mix's sampling error."""
    global _active
    _active = bool(flag)


def is_enabled():
    return _enabled


def set_target(name):
    """Count and time only region `name` (None: every region) until the next enable(). bench.py ranks the regions
    in untimed pre-pass steps and then times only the dominant one over its timed steps: the per-launch
    bookkeeping of every region (counts, sampling, HIP events on 1/n of ~6 k launches a step) cost ~2 % of the
    step's wall time (profiles/r6_bm_timer_overhead_ab.txt), and a bypassed region costs one string compare."""
    global _target
    _target = name


def dominant_name(s):
    """The region with the largest total time among our kernels (not library GEMMs) of a summary() dict."""
    own = [(v["total_ms"], k) for k, v in s.items() if not k.startswith("vendor_gemm<")]
    return max(own)[1] if own else None


class _Null:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False


_NULL = _Null()


class _TorchPair:
    """Events recorded around a (library) call on the launch stream; pooled like _KernelPair (creating
    two events per timed call is host work inside the timed steps)."""
    _pool = []

    def __init__(self):
        if _TorchPair._pool:
            self.s, self.e = _TorchPair._pool.pop()
        else:
            self.s = torch.cuda.Event(enable_timing=True)
            self.e = torch.cuda.Event(enable_timing=True)

    def ms(self):
        out = self.s.elapsed_time(self.e)
        _TorchPair._pool.append((self.s, self.e))
        return out


class _KernelPair:
    """Events bound to our kernels' dispatches (vfm_timer_arm); pooled, since a timed region creates
    one pair per timed launch."""
    _pool = []

    def __init__(self, lib):
        self.lib = lib
        if _KernelPair._pool:
            self.s, self.e = _KernelPair._pool.pop()
        else:
            s, e = ctypes.c_void_p(), ctypes.c_void_p()
            if lib.vfm_event_create(ctypes.byref(s)) or lib.vfm_event_create(ctypes.byref(e)):
                raise RuntimeError("vfm_event_create failed")
            self.s, self.e = s.value, e.value
        self.launched = False

    def ms(self):
        if not self.launched:
            return None
        out = ctypes.c_float()
        rc = self.lib.vfm_event_elapsed(self.s, self.e, ctypes.byref(out))
        _KernelPair._pool.append((self.s, self.e))
        return float(out.value) if rc == 0 else None


_lib = None


def _native():
    global _lib
    if _lib is None:
        from torch_utils import custom_ops
        _lib = custom_ops.get_native()
    return _lib


class _Timed:
    """One sampled launch: native regions arm the kernel library's dispatch events around the launch,
    library regions record torch events on the current stream. A plain context-manager class (a
    generator-based one costs a few microseconds of host time per timed launch)."""
    __slots__ = ("name", "nbytes", "flops", "bound", "native", "pair", "first")

    def __init__(self, name, nbytes, flops, bound, native, first=False):
        # nbytes may be lazy (decoder_hip._LazyBytes): evaluated for sampled launches only
        self.name, self.nbytes, self.flops, self.bound, self.native = name, int(nbytes), flops, bound, native
        self.first = first

    def __enter__(self):
        if self.native:
            lib = _native()
            self.pair = _KernelPair(lib)
            (lib.vfm_timer_arm_first if self.first else lib.vfm_timer_arm)(self.pair.s, self.pair.e)
        else:
            self.pair = _TorchPair()
            self.pair.s.record(torch.cuda.current_stream())
        return None

    def __exit__(self, *exc):
        pair = self.pair
        if self.native:
            pair.launched = pair.lib.vfm_timer_arm(None, None) > 0
            if not pair.launched:
                _KernelPair._pool.append((pair.s, pair.e))
        else:
            pair.e.record(torch.cuda.current_stream())
        _records.setdefault(self.name, []).append((pair, self.nbytes, self.flops, self.bound))
        return False


@contextlib.contextmanager
def suspended():
    """No timing inside (HIP-graph capture: events cannot be recorded into a capture and the
    replayed kernels are not launched through the wrappers)."""
    global _enabled
    prev, _enabled = _enabled, False
    try:
        yield
    finally:
        _enabled = prev


def _sampled(c):
    """Launch index c of a region is timed: (c * 40503) mod 2^16 is a permutation of each block of
    2^16 indices, so exactly 1/_every of them fall below the threshold, spread pseudo-randomly over a
    step's launch positions (a plain stride aliases with the region's launches per step: every 4th of
    10 per step = even ones only). Three integer operations on the host path of every launch."""
    return ((c * 40503) & 0xFFFF) < 65536 // _every


def region(name, nbytes=0, flops=0, bound="hbm", native=True, first_only=False):
    """Context manager around one launch (native = our kernel library, timed by the kernel dispatch;
    otherwise events around the call); a shared no-op object when timing is off or the launch is not
    sampled (this is on every launch's host path). first_only: only the call's first kernel is timed (a GEMM
    whose split-K combine pass follows as a kernel of its own: the region then covers exactly the launches of
    the GEMM kernel instantiation rocprofv3 names)."""
    if not _enabled or (_target is not None and name != _target):
        return _NULL
    c = _counts.get(name, 0)
    _counts[name] = c + 1
    if flops:
        _flops_all[name] = _flops_all.get(name, 0.0) + flops
    if not _active:
        return _NULL
    if _every > 1:
        if _phase >= 0:
            j = _pos.get(name, 0)
            _pos[name] = j + 1
            # a region with few launches per step is sampled more densely (all of them below 2 x MIN_SAMPLES):
            # the decoder's b5 MLP runs 5 times a step, in shapes that follow each step's equivariance draw, and
            # 1/20 of them over 20 steps were 5 samples from 5 particular steps
            ev = max(1, min(_every, _per_step.get(name, _every * MIN_SAMPLES) // MIN_SAMPLES))
            if (j + _phase) % ev:
                return _NULL
        elif not _sampled(c):
            return _NULL
    return _Timed(name, nbytes, flops, bound, native, first_only)


def vendor_gemm(tag, M, N, K, z=1, esize=2):
    """Region around a library GEMM (hipBLASLt through torch.matmul / bmm / addmm) with its
    algorithmic FLOPs and bytes (A, B, C once each), so the bench can rank the vendor kernels next
    to ours; names start with `vendor_gemm<`."""
    if not _enabled:
        return _NULL
    return region(f"vendor_gemm<{tag}>", esize * z * (M * K + K * N + M * N), 2.0 * z * M * N * K, "mfma",
                  native=False)


_calib_ms = 0.0    # fixed interval of one timed launch of an empty kernel (calibrate()), subtracted per launch


def calibrate(n=64):
    """Median interval of `n` timed empty-kernel launches on the current stream (vfm_timer_null_launch): the
    dispatch gap and empty-kernel time every timed native launch carries (round 6: +5-12 us on the decoder's
    10-40 us kernels against rocprofv3's trace of the same run, gpurun_out r6r). summary() subtracts it from
    each timed native launch. Call with the GPU idle (before the timed steps)."""
    global _calib_ms
    lib = _native()
    from torch_utils import custom_ops
    st = custom_ops.stream_ptr()
    pairs = []
    torch.cuda.synchronize()
    for _ in range(n):
        pair = _KernelPair(lib)
        lib.vfm_timer_arm(pair.s, pair.e)
        custom_ops.check(lib.vfm_timer_null_launch(st), "vfm_timer_null_launch")
        pair.launched = lib.vfm_timer_arm(None, None) > 0
        pairs.append(pair)
    vals = sorted(v for v in (p.ms() for p in pairs) if v is not None)
    _calib_ms = vals[len(vals) // 2] if vals else 0.0
    return _calib_ms


def summary():
    torch.cuda.synchronize()
    out = {}
    for name, recs in _records.items():
        timed = [(p.ms(), b, f, bd) for p, b, f, bd in recs]
        timed = [t for t in timed if t[0] is not None]      # a region that launched nothing has no time
        if _calib_ms and recs and isinstance(recs[0][0], _KernelPair):
            timed = [(max(t[0] - _calib_ms, 0.0),) + t[1:] for t in timed]
        if not timed:
            continue
        ms = sum(t[0] for t in timed)
        n = _counts.get(name, len(timed))
        scale = n / len(timed)              # every n-th launch timed: totals extrapolated to all launches
        out[name] = dict(launches=n, timed_launches=len(timed), total_ms=ms * scale,
                         bytes=sum(t[1] for t in timed) * scale, flops=sum(t[2] for t in timed) * scale,
                         flops_all=_flops_all.get(name, 0.0), bound=timed[0][3])
    return out


# region name (op<dtype[,taps]>) -> the kernel instantiation(s) it launches, as rocprofv3 prints
# them (anonymous namespace and call arguments stripped); used to match the HIP-event timing
# against the rocprof summary and the PMC traffic of the same kernel.
_ROC = {
    "scale_bias_gelu_fwd": "gelu_fwd<{T}>", "scale_bias_gelu_bwd": "gelu_bwd<{T}>",
    "layer_scale_residual_fwd": "lsr_fwd<{T}, ", "layer_scale_residual_bwd": "lsr_bwd<{T}, ",
    "group_norm_fwd": "gn_fwd<{T}, ", "group_norm_bwd": "gn_bwd<{T}, ", "group_norm_fwd_stats": "gn_apply<{T}, ",
    "dwconv2d_fwd": "dwr_fwd<{T}, {K}>", "dwconv2d_bwd_data": "dwr_fwd<{T}, {K}>",
    "dwconv2d_bwd_weight": "dwr_bwd_w<{T}, {K}>",
    "dwconv2d_mfma_fwd": "dwm_fwd<{K}, ", "dwconv2d_mfma_bwd_data": "dwm_fwd<{K}, ",
    "dwconv2d_mfma_bwd_weight": "dwm_bwd_w<{K}, ",
    "shuffle_blur_fwd": "blur_fwd<{T}, 2, {K}>", "shuffle_blur_bwd": "blur_bwd<{T}, 2, {K}>",
    "residual_layer_norm": "ln_rows<", "codebook_argmax": "codebook_argmax_kernel<",
    "convnext_mlp_fwd": "mlp_fwd<", "pw_gemm_gelu_bwd": "pw_gemm_gelu<1, ",
    "attention_fwd": "attn_fwd_d64",
}
_NP = {"f32x6": 3, "f32x3": 2, "bf16": 1}
_TNAME = {"f32": "float", "bf16": "__hip_bfloat16", "f16": "__half", "f64": "double"}


def roc_match(pattern, kernel_name):
    """A rocprof kernel name (anonymous namespace / `void` / call arguments stripped or not) against a
    rocprof_name() pattern: a prefix, '*' matching any run of characters."""
    import fnmatch
    n = kernel_name.replace("void ", "").replace("(anonymous namespace)::", "")
    return fnmatch.fnmatchcase(n, pattern + "*")


def rocprof_name(region):
    """'scale_bias_gelu_bwd<bf16>' -> 'gelu_bwd<__hip_bfloat16>' (a prefix of the rocprof name)."""
    region = region.split("[", 1)[0]
    base, _, args = region.partition("<")
    args = args.rstrip(">").split(",") if args else []
    if base == "gemm8" and len(args) == 4:                     # <tag, AK, BK, OUTF32> (default schedule, EPI 0)
        return f"gemm8_kernel<{args[1]}, {args[2]}, {args[3]}, false, 0>"
    if base == "gemm9" and len(args) == 4:                     # persistent gemm9p_kernel<AK, BK, OUTF32, EPI, NP>
        # EPI 0-3 (plain / bias / GELU epilogues); 4 and 5 are the ConvNeXt-MLP forms of the gemm9_gelu regions
        return f"gemm9p_kernel<{args[1]}, {args[2]}, {args[3]}, [0-3], {_NP.get(args[0], 1)}>"
    if base == "gemm9_gelu" and len(args) == 1:                # GELU epilogue forms (mode 1 / 2: EPI 4 / 5)
        return f"gemm9p_kernel<true, false, false, {3 + int(args[0])}>"
    if base == "gemm8_gelu" and len(args) == 1:                # GELU epilogue forms (mode 1 / 2)
        return f"gemm8_kernel<true, false, false, false, {args[0]}>"
    if base == "gemm_fold" and len(args) == 3:                 # batch-folded: gemm_kernel<AK, false, NP, OUTF32, NW>
        np_ = _NP.get(args[0], 1)
        nw = 8 if (np_ == 3 and os.environ.get("VFM_GEMM128_WAVES", "8") != "4") else 4
        return f"gemm_kernel<{args[1]}, false, {np_}, {args[2]}, {nw}>"
    if base == "sgemm" and len(args) == 5:                     # exact-fp32 sgemm_kernel<AK, BK, BM, BN, KW>
        return f"sgemm_kernel<{args[0]}, {args[1]}, {args[2]}, {args[3]}, {args[4]}>"
    if base == "gemm" and len(args) == 4:                      # gemm_kernel<AK, BK, NP, OUTF32, NW>
        np_ = _NP.get(args[0], 1)
        nw = 8 if (np_ == 3 and os.environ.get("VFM_GEMM128_WAVES", "8") != "4") else 4
        return f"gemm_kernel<{args[1]}, {args[2]}, {np_}, {args[3]}, {nw}>"
    if base == "conv3x3_nhwc" and len(args) == 2:              # conv3x3_kernel<BM, BN, NP>
        np_ = _NP.get(args[0], 3)
        wide64 = os.environ.get("VFM_CONV_N64", "128") == "256"
        bm = 256 if (np_ == 3 and (args[1] == "128" or wide64)) else 128
        return f"conv3x3_kernel<{bm}, {args[1]}, {np_}>"
    if base in ("attention_fwd", "attention_bwd") and args and args[0] in ("f32x6", "f32x3"):
        np_ = _NP[args[0]]
        if base == "attention_fwd":
            occ = 2 if (np_ == 3 and os.environ.get("VFM_ATTN32_OCC", "2") != "1") else 1
            return f"attn32_fwd<{np_}, {occ}>"
        occ = 2 if (np_ == 3 and os.environ.get("VFM_ATTN32_DKDV_OCC", "2") != "1") else 1
        return f"attn32_dkdv<{np_}, {occ}>"
    if base == "convnext_mlp_fwd" and len(args) == 3:          # mlp_fwd<C, SAVE>
        return f"mlp_fwd<{args[1]}, {args[2]}>"
    pat = _ROC.get(base)
    if pat is None:
        return None
    T = _TNAME.get(args[0], args[0]) if args else ""
    K = args[1] if len(args) > 1 else ""
    return pat.format(T=T, K=K)


def _roof(name, r, hbm_peak_gbs, mfma_peak_tflops):
    t = r["total_ms"] / 1e3
    note = None
    if r["bound"] == "mfma":
        achieved = r["flops"] / t / 1e12
        peak, unit = mfma_peak_tflops, "TFLOP/s"
        if "f32x6" in name:
            # fp32-equivalent products as 6 bf16 MFMAs over exact 3-piece splits: the fp32 rate this
            # path can reach is the dense bf16 peak / 6 (the fp32 MFMA peak is 157.3 TF/s)
            peak = round(mfma_peak_tflops / 6, 1)
            note = "achieved = fp32 FLOPs of the op / time; peak = dense bf16 MFMA peak / 6 (f32x6 split)"
        elif "f32x3" in name:
            peak = round(mfma_peak_tflops / 3, 1)
            note = "achieved = fp32 FLOPs of the op / time; peak = dense bf16 MFMA peak / 3 (opt-in f32x3 split)"
        elif "<f32" in name or name.startswith("sgemm<"):
            peak = 157.3
            note = "exact fp32 MFMA peak"
    else:
        achieved = r["bytes"] / t / 1e9
        peak, unit = hbm_peak_gbs, "GB/s"
    return achieved, peak, unit, note


def dominant_roofline(hbm_peak_gbs, mfma_peak_tflops, traffic_table=None, steps=None, prepass=None):
    """The roofline object of the bench line: our kernel (timer region) with the largest total
    time, plus `vendor_top`, the library GEMM region with the largest total time (ranked the same
    way; hipBLASLt kernels are not ours, so they never become the roofline kernel itself).
    prepass = (summary of untimed pre-pass steps, scale): the current records hold only the target region
    (set_target); the ranking, runner-up, vendor_top and all_kernels come from the pre-pass summary, its
    totals multiplied by `scale` (timed steps / pre-pass steps)."""
    s = summary()
    if not s:
        return None
    timed = s
    if prepass is not None:
        pre, scale = prepass
        s = {k: dict(v, total_ms=v["total_ms"] * scale, bytes=v["bytes"] * scale, flops=v["flops"] * scale,
                     launches=max(1, round(v["launches"] * scale))) for k, v in pre.items()}
        s.update(timed)
    own = {k: v for k, v in s.items() if not k.startswith("vendor_gemm<")}
    vend = {k: v for k, v in s.items() if k.startswith("vendor_gemm<")}
    ranked = sorted(own.items(), key=lambda kv: -kv[1]["total_ms"])
    if prepass is not None:
        # the timed region's own record leads (it was the pre-pass's dominant region)
        ranked = [kv for kv in ranked if kv[0] in timed] + [kv for kv in ranked if kv[0] not in timed]

    def entry(name, r):
        achieved, peak, unit, note = _roof(name, r, hbm_peak_gbs, mfma_peak_tflops)
        roc = rocprof_name(name)
        traffic = None
        if traffic_table and roc:
            hits = [(v["dispatches_fetch_pass"], v["traffic_bytes_per_launch"]) for k, v in traffic_table.items()
                    if roc_match(roc, k) and v.get("traffic_bytes_per_launch")]
            n = sum(h[0] for h in hits)
            if n:
                traffic = int(sum(c * t for c, t in hits) / n)
        bpl = int(r["bytes"] / r["launches"])
        return {"bound": r["bound"], "achieved": round(achieved, 1), "peak": peak, "unit": unit,
                "frac": round(achieved / peak, 4), "traffic": traffic, "kernel": name, "rocprof_kernel": roc,
                "peak_note": note,
                "launches": r["launches"], "timed_launches": r["timed_launches"],
                "avg_us": round(r["total_ms"] * 1e3 / r["launches"], 2),
                "ms_total": round(r["total_ms"], 3),
                "bytes_per_launch": bpl,
                "flops_per_launch": int(r["flops"] / r["launches"]),
                # every launch's flops (host arithmetic over all launches, timed or not): the timed
                # launches' mean above should agree with it
                "flops_per_launch_all": int(r["flops_all"] / r["launches"]) if r["flops_all"] else None,
                "traffic_over_algorithmic": round(traffic / bpl, 3) if traffic and bpl else None}

    out = entry(*ranked[0])
    # the two largest of our kernels within 5 % of each other: which one leads depends on the run, so the
    # line names both (the roofline object itself stays the larger one)
    if len(ranked) > 1 and ranked[1][1]["total_ms"] >= 0.95 * ranked[0][1]["total_ms"]:
        out["runner_up"] = entry(*ranked[1])
    if vend:
        vn, vr = max(vend.items(), key=lambda kv: kv[1]["total_ms"])
        va, vp, vu, vnote = _roof(vn, vr, hbm_peak_gbs, mfma_peak_tflops)
        out["vendor_top"] = {"kernel": vn, "achieved": round(va, 1), "peak": vp, "unit": vu, "frac": round(va / vp, 4),
                             "ms_total": round(vr["total_ms"], 3), "launches": vr["launches"],
                             "avg_us": round(vr["total_ms"] * 1e3 / vr["launches"], 2)}
        out["vendor_gemm_ms_total"] = round(sum(v["total_ms"] for v in vend.values()), 3)
    out["all_kernels"] = {}
    for k, v in sorted(s.items(), key=lambda kv: -kv[1]["total_ms"]):
        gbps = v["bytes"] / max(v["total_ms"], 1e-9) / 1e6
        row = {"ms": round(v["total_ms"], 3), "launches": v["launches"], "GBps": round(gbps, 1),
               "TFps": round(v["flops"] / max(v["total_ms"], 1e-9) / 1e9, 1)}
        if gbps > hbm_peak_gbs:
            # algorithmic bytes faster than HBM can deliver: operands (partly) served from L2 / MALL
            row["cache_served"] = True
        out["all_kernels"][k] = row
    return out
