"""Per-kernel ms/step difference of two bench.py JSON lines (the roofline object's all_kernels table):
python tools_dev/bench_diff.py A.log B.log [N]"""
import json
import sys


def load(f):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    return d, d["roofline"]["all_kernels"]


(da, a), (db, b) = load(sys.argv[1]), load(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 25


def ms(t, k):
    """ms per timed step (all_kernels holds the total over the timed steps)."""
    v = t.get(k)
    return 0.0 if v is None else float(v["ms"]) / (da["steps"] if t is a else db["steps"])


print(f"A {da['value']} img/s {da['ms_per_step']} ms   B {db['value']} img/s {db['ms_per_step']} ms")
rows = sorted(((ms(a, k) - ms(b, k), k, ms(a, k), ms(b, k)) for k in set(a) | set(b)), key=lambda r: -abs(r[0]))
for r in rows[:n]:
    print("%8.2f  %-70s %8.2f %8.2f" % r)
print("sum A %.1f  B %.1f" % (sum(ms(a, k) for k in a), sum(ms(b, k) for k in b)))
