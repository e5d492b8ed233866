"""HBM traffic per kernel launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

  python tools_dev/pmc_traffic.py <fetch_pass_dir> <write_pass_dir> > traffic.json

Correction per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced streaming read, so bytes read = 2 x FETCH_SIZE;
WRITE_SIZE is exact for 16-B-per-lane stores. Both counters are in KiB. Output: per kernel
name (template arguments kept, call arguments stripped) the dispatch count and the average
per-dispatch FETCH_SIZE, WRITE_SIZE and corrected traffic in bytes.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no *counter_collection.csv under {d}")
    for f in files:
        yield from csv.DictReader(open(f))


def _short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    depth, out = 0, []
    for ch in name:                       # drop the call-argument list, keep template args
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out).strip()


def per_kernel(d, counter):
    vals = defaultdict(dict)              # kernel -> dispatch -> value
    for r in _rows(d):
        if r.get("Counter_Name") != counter:
            continue
        k = _short(r.get("Kernel_Name", ""))
        disp = r.get("Dispatch_Id") or r.get("Correlation_Id") or str(len(vals[k]))
        vals[k][disp] = vals[k].get(disp, 0.0) + float(r["Counter_Value"])
    return {k: (len(v), sum(v.values()) / max(len(v), 1)) for k, v in vals.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        nf, f = fetch.get(k, (0, 0.0))
        nw, w = write.get(k, (0, 0.0))
        out[k] = {"dispatches_fetch_pass": nf, "dispatches_write_pass": nw, "fetch_kib_avg": round(f, 3),
                  "write_kib_avg": round(w, 3),
                  "traffic_bytes_per_launch": int(round((2.0 * f + w) * 1024)) if nf and nw else None}
    json.dump({"correction": "bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE counts half "
                             "of wide coalesced reads; MI355X_MICROARCH.md HBM section)", "kernels": out},
              sys.stdout, indent=1)


if __name__ == "__main__":
    main()
