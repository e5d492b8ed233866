#!/bin/bash
# Same-box A/B of the opt-in im2col rows form + planar split kernel (both on vs both off), A B A B.
out=gpurun_out/$1; mkdir -p $out
for i in 1 2; do
  timeout -k 10 600 python bench.py --no-cpu-baseline > $out/a$i.log 2>&1 || exit $?
  VFM_IM2COL_ROWS=1 VFM_SPLIT_PLANAR8=1 timeout -k 10 600 python bench.py --no-cpu-baseline > $out/b$i.log 2>&1 || exit $?
done
