"""Per-launch HIP-event timing of named kernels inside a timed region.

bench.py enables the timer around its timed steps; every native op wrapper
brackets its launch with a pair of events recorded on the stream the kernel is
launched on, and reports the launch's ALGORITHMIC bytes (unique inputs +
outputs + weights at the op boundary) and flops. `dominant_roofline()` picks
the kernel with the largest total time and returns the bench.py `roofline`
object (achieved = algorithmic bytes or flops per launch / average launch time).
"""
import contextlib

import torch

_enabled = False
_records = {}      # name -> list of (start_event, end_event, bytes, flops, bound)


def enable(flag: bool):
    global _enabled
    _enabled = bool(flag)
    if flag:
        _records.clear()


def is_enabled():
    return _enabled


@contextlib.contextmanager
def region(name, nbytes=0, flops=0, bound="hbm"):
    if not _enabled:
        yield
        return
    st = torch.cuda.current_stream()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record(st)
    try:
        yield
    finally:
        e.record(st)
        _records.setdefault(name, []).append((s, e, nbytes, flops, bound))


def summary():
    torch.cuda.synchronize()
    out = {}
    for name, recs in _records.items():
        ms = sum(s.elapsed_time(e) for s, e, *_ in recs)
        out[name] = dict(launches=len(recs), total_ms=ms, bytes=sum(r[2] for r in recs),
                         flops=sum(r[3] for r in recs), bound=recs[0][4])
    return out


def dominant_roofline(hbm_peak_gbs, mfma_peak_tflops):
    s = summary()
    if not s:
        return None
    name, r = max(s.items(), key=lambda kv: kv[1]["total_ms"])
    t = r["total_ms"] / 1e3
    if r["bound"] == "mfma":
        achieved = r["flops"] / t / 1e12
        peak, unit = mfma_peak_tflops, "TFLOP/s"
    else:
        achieved = r["bytes"] / t / 1e9
        peak, unit = hbm_peak_gbs, "GB/s"
    return {"bound": r["bound"], "achieved": round(achieved, 1), "peak": peak, "unit": unit,
            "frac": round(achieved / peak, 4), "traffic": None, "kernel": name, "launches": r["launches"],
            "avg_us": round(r["total_ms"] * 1e3 / r["launches"], 2),
            "bytes_per_launch": int(r["bytes"] / r["launches"]),
            "all_kernels": {k: {"ms": round(v["total_ms"], 3), "launches": v["launches"],
                                "GBps": round(v["bytes"] / max(v["total_ms"], 1e-9) / 1e6, 1)}
                            for k, v in sorted(s.items(), key=lambda kv: -kv[1]["total_ms"])}}
