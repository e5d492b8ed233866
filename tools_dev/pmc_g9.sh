#!/bin/bash
# rocprofv3 --pmc passes over one bf16 GEMM shape (G8_M/G8_N/G8_K env) on gemm9 and on hipBLASLt (tools_dev/g8one.py),
# and over the style kernels (tools_dev/stylebench.py). Usage: tools_dev/pmc_g9.sh <tag>
out=gpurun_out/$1; mkdir -p $out
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
for kd in g9 blas; do
  G8_KIND=$kd timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/kt_$kd -o run --output-format csv -- python3 tools_dev/g8one.py > $out/kt_$kd.log 2>&1 || exit 1
  G8_KIND=$kd timeout -s KILL 120 rocprofv3 --pmc $P1 -d $out/p1_$kd -o run --output-format csv -- python3 tools_dev/g8one.py > $out/p1_$kd.log 2>&1 || exit 1
  G8_KIND=$kd timeout -s KILL 120 rocprofv3 --pmc $P2 -d $out/p2_$kd -o run --output-format csv -- python3 tools_dev/g8one.py > $out/p2_$kd.log 2>&1 || exit 1
  python3 tools_dev/pmc_sum.py $out/p1_$kd $out/p2_$kd > $out/pmc_$kd.json || exit 1
done
