#!/bin/bash
# Same-box A/B of the D phase's HIP-graph generator forward: eager, graphs, eager, graphs (bench.py).
out=gpurun_out/$1; mkdir -p $out
for i in 1 2 3; do
  timeout -k 10 600 python bench.py --no-cpu-baseline --graphs off > $out/eager$i.log 2>&1 || exit $?
  timeout -k 10 600 python bench.py --no-cpu-baseline --graphs on > $out/graphs$i.log 2>&1 || exit $?
done
