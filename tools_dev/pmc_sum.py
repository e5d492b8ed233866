"""Average per-dispatch value of every counter in one or more rocprofv3 --pmc pass directories, per kernel.

  python tools_dev/pmc_sum.py <pass_dir>... [--re REGEX]

Prints one JSON object {kernel: {"dispatches": n, counter: mean, ...}} (kernel names with template arguments,
call arguments stripped); kernels that match --re only."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    depth, out = 0, []
    for ch in name:
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out).strip()


def main():
    args = sys.argv[1:]
    pat = None
    if "--re" in args:
        i = args.index("--re")
        pat = re.compile(args[i + 1])
        args = args[:i] + args[i + 2:]
    acc = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(set))
    for d in args:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = short(r.get("Kernel_Name", r.get("Kernel-Name", "")))
                if pat and not pat.search(k):
                    continue
                c = r.get("Counter_Name", r.get("Counter-Name"))
                acc[k][c] += float(r.get("Counter_Value", r.get("Counter-Value", 0)))
                cnt[k][c].add((d, r.get("Dispatch_Id", r.get("Dispatch-Id"))))
    out = {}
    for k, cs in acc.items():
        o = {}
        for c, v in cs.items():
            n = max(1, len(cnt[k][c]))
            o[c] = round(v / n, 1)
            o["dispatches"] = n
        out[k] = o
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
