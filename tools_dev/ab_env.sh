#!/bin/bash
# Same-box A/B of an env switch: ab_env.sh <tag> <VAR> <valA> <valB>; A,B,A,B bench runs.
out=gpurun_out/$1; mkdir -p $out
for i in 1 2; do
  env $2=$3 timeout -k 10 600 python bench.py --no-cpu-baseline > $out/a$i.log 2>&1 || exit $?
  env $2=$4 timeout -k 10 600 python bench.py --no-cpu-baseline > $out/b$i.log 2>&1 || exit $?
done
