#!/bin/bash
# Same-box A/B/C of bench.py arguments: ab3_args.sh <tag> "<args A>" "<args B>" "<args C>"; A,B,C twice.
out=gpurun_out/$1; mkdir -p $out
for i in 1 2; do
  timeout -k 10 600 python bench.py --no-cpu-baseline $2 > $out/a$i.log 2>&1 || exit $?
  timeout -k 10 600 python bench.py --no-cpu-baseline $3 > $out/b$i.log 2>&1 || exit $?
  timeout -k 10 600 python bench.py --no-cpu-baseline $4 > $out/c$i.log 2>&1 || exit $?
done
