"""Compare the bench line's per-kernel averages (roofline.all_kernels + region -> rocprof kernel names) with the
rocprofv3 kernel-trace stats of the SAME process (bench.py run under `rocprofv3 --kernel-trace --stats`).

  python tools_dev/timer_vs_rocprof.py <bench.log> <run_kernel_trace.csv>

Prints, for every own kernel region with a rocprof counterpart, the event-timed average, rocprof's average over
the launches of the matching instantiation(s) inside the timed window (the last `timed N steps: T s` of the log,
so warm-up launches with another shape mix do not enter), and the ratio.
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "vfm-vae_amd")]


def main(bench_log, trace_csv):
    import re
    from torch_utils.ops import kernel_timer
    text = open(bench_log).read()
    line = next(json.loads(x) for x in text.splitlines() if x.startswith("{"))
    window = float(re.search(r"timed \d+ steps: ([0-9.]+)s", text).group(1))
    ak = line["roofline"]["all_kernels"]
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(trace_csv))]
    tend = max(r[1] for r in rows)
    agg = {}
    for s0, e0, n in rows:
        if s0 > tend - window * 1e9:
            a = agg.setdefault(n, [0, 0.0])
            a[0] += 1
            a[1] += e0 - s0
    stats = [(n, c, t) for n, (c, t) in agg.items()]
    out = []
    for reg, v in ak.items():
        if reg.startswith("vendor_gemm<"):
            continue
        roc = kernel_timer.rocprof_name(reg)
        if not roc:
            continue
        # regions that launch two kernels per call: their per-call time is the sum of both kernels' averages
        extra = {"attention_bwd": "attn32_dq<"}.get(reg.split("<")[0])
        hits = [(c, t) for n, c, t in stats if kernel_timer.roc_match(roc, n)]
        if not hits:
            continue
        calls, tot = sum(h[0] for h in hits), sum(h[1] for h in hits)
        ev_us = v["ms"] * 1e3 / v["launches"]
        rp_us = tot / calls / 1e3
        if extra:
            h2 = [(c, t) for n, c, t in stats if kernel_timer.roc_match(extra, n)]
            if h2:
                rp_us += sum(h[1] for h in h2) / sum(h[0] for h in h2) / 1e3
        out.append((v["ms"], reg, roc, ev_us, rp_us, ev_us / rp_us))
    out.sort(key=lambda r: -r[0])
    print(f"{'region':44s} {'events us':>10s} {'rocprof us':>10s} {'ratio':>6s}  ms (timed region)")
    for ms, reg, roc, e, r, q in out:
        print(f"{reg[:44]:44s} {e:10.1f} {r:10.1f} {q:6.3f}  {ms:.1f}")
    within = [q for *_, q in out if abs(q - 1) <= 0.05]
    print(f"{len(within)} of {len(out)} kernels within 5 %")


if __name__ == "__main__":
    main(*sys.argv[1:3])
