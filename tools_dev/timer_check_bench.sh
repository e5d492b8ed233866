# The bench under rocprofv3's kernel trace; the bench line's event timings against the trace's timed window
# (tools_dev/timer_vs_rocprof.py). Usage: bash tools_dev/timer_check_bench.sh <tag>
export TMPDIR=/tmp; o=gpurun_out/${1:-timer}; mkdir -p $o
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > $o/prof.log 2>&1 \
  && tr=$(find $o/prof -name '*kernel_trace.csv' | head -1) \
  && python tools_dev/prof_summary.py $tr 20 $(sed -n "s/.*timed 20 steps: \([0-9.]*\)s.*/\1/p" $o/prof.log) > $o/prof_summary.txt \
  && python tools_dev/timer_vs_rocprof.py $o/prof.log $tr > $o/timer_vs_rocprof.txt \
  && find $o/prof -name '*kernel_trace.csv' -delete
