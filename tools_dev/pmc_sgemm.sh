# PMC passes over tools_dev/sgemm_prof.py (one counter group per run; SGP selects the shapes)
export TMPDIR=/tmp; o=gpurun_out/${1:-r6i}; mkdir -p $o
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $o/kt -o run --output-format csv -- python3 tools_dev/sgemm_prof.py > $o/kt.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex sgemm_kernel -d $o/p1 -o run --output-format csv -- python3 tools_dev/sgemm_prof.py > $o/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --kernel-include-regex sgemm_kernel -d $o/p2 -o run --output-format csv -- python3 tools_dev/sgemm_prof.py > $o/p2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_IFETCH SQ_LEVEL_WAVES SQ_ACCUM_PREV_HIRES --kernel-include-regex sgemm_kernel -d $o/p3 -o run --output-format csv -- python3 tools_dev/sgemm_prof.py > $o/p3.log 2>&1
