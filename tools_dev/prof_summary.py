"""Summarise a rocprofv3 kernel trace: per-step busy time of the last N steps, top kernels.
  python tools_dev/prof_summary.py <run_kernel_trace.csv> [steps=3] [seconds_window]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rows = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'])
            for r in csv.DictReader(open(path))]
    rows.sort()
    window = float(sys.argv[3]) if len(sys.argv) > 3 else None
    tend = rows[-1][1]
    sel = [r for r in rows if window is None or r[0] > tend - window * 1e9]
    busy = sum(e - s for s, e, _ in sel)
    print(f"kernels {len(sel)}  busy {busy / 1e6:.1f} ms  span {(sel[-1][1] - sel[0][0]) / 1e6:.1f} ms  "
          f"per step busy {busy / steps / 1e6:.1f} ms")
    agg = collections.defaultdict(lambda: [0, 0])
    for s, e, n in sel:
        k = n.replace('void ', '').replace('(anonymous namespace)::', '')
        k = k.split('(')[0][:110]
        agg[k][0] += e - s
        agg[k][1] += 1
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0])[:45]:
        print(f"{v[0] / steps / 1e6:8.2f} ms/step {v[1] / steps:7.1f}/step {v[0] / v[1] / 1e3:8.1f} us  {k}")
    # idle time on the GPU (launch-bound stretches): gap before each kernel, by kernel name
    gaps = collections.defaultdict(lambda: [0, 0])
    idle = 0
    end = sel[0][1]
    for s_, e_, n in sel[1:]:
        g = s_ - end
        if g > 0:
            idle += g
            k = n.replace('void ', '').replace('(anonymous namespace)::', '').split('(')[0][:110]
            gaps[k][0] += g
            gaps[k][1] += 1
        end = max(end, e_)
    print(f"\nGPU idle {idle / steps / 1e6:.1f} ms/step; largest idle before:")
    for k, v in sorted(gaps.items(), key=lambda kv: -kv[1][0])[:25]:
        print(f"{v[0] / steps / 1e6:8.2f} ms/step {v[1] / steps:7.1f}/step  {k}")


if __name__ == "__main__":
    main()
