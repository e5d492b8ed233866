#!/bin/bash
# A/B of the GEMM solution table on one box: off, use, off, use (each its own time limit).
out=gpurun_out/$1; mkdir -p $out
for i in 1 2; do
  timeout -k 10 600 python bench.py --no-cpu-baseline --tunableop off > $out/off$i.log 2>&1 || exit $?
  timeout -k 10 600 python bench.py --no-cpu-baseline --tunableop use > $out/use$i.log 2>&1 || exit $?
done
