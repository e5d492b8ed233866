#!/bin/bash
# Runs a sequence of GPU steps; each under its own timeout; stops at the first
# failure (no retries). Usage: tools_dev/gpu_run.sh <tag> <step>...
# step names: tests | bench | prof | opbench
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
for s in "$@"; do
  echo "=== step $s $(date +%T)" | tee -a $out/steps.log
  case $s in
    tests)   timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 ;;
    testsk)  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 ;;
    bench)   timeout -k 10 900 python bench.py > $out/bench.log 2>&1 ;;
    benchshape) VFM_TIMER_SHAPES=1 timeout -k 10 600 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > $out/benchshape.log 2>&1 ;;
    benchres) VFM_RESIDUAL_FUSION=0 timeout -k 10 600 python bench.py --no-cpu-baseline > $out/bench_r0.log 2>&1 && VFM_RESIDUAL_FUSION=1 timeout -k 10 600 python bench.py --no-cpu-baseline > $out/bench_r1.log 2>&1 && VFM_RESIDUAL_FUSION=0 timeout -k 10 600 python bench.py --no-cpu-baseline > $out/bench_r2.log 2>&1 && VFM_RESIDUAL_FUSION=1 timeout -k 10 600 python bench.py --no-cpu-baseline > $out/bench_r3.log 2>&1 ;;
    benchkt) timeout -k 10 600 python bench.py --no-cpu-baseline > $out/bench_kt1.log 2>&1 && timeout -k 10 600 python bench.py --no-cpu-baseline --no-kernel-timer > $out/bench_kt0.log 2>&1 && timeout -k 10 600 python bench.py --no-cpu-baseline > $out/bench_kt3.log 2>&1 && timeout -k 10 600 python bench.py --no-cpu-baseline --no-kernel-timer > $out/bench_kt2.log 2>&1 ;;
    benchq)  timeout -k 10 600 python bench.py --no-cpu-baseline > $out/bench.log 2>&1 ;;
    benchref) timeout -k 10 600 python bench.py --steps 4 --warmup 2 --no-cpu-baseline --force-ref-ops > $out/bench_ref.log 2>&1 ;;
    prof)    ps=${PROF_STEPS:-20}
             timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --steps $ps --warmup 2 --no-cpu-baseline > $out/prof.log 2>&1 \
               && python tools_dev/prof_summary.py $(find $out/prof -name '*kernel_trace.csv' | head -1) $ps \
                    $(sed -n "s/.*timed $ps steps: \([0-9.]*\)s.*/\1/p" $out/prof.log) > $out/prof_summary.txt \
               && find $out/prof -name '*kernel_trace.csv' -delete ;;
    pmc)     re=${PMC_RE:-gelu_bwd}
             timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$re" -d $out/pmc_f -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > $out/pmc_f.log 2>&1 \
               && timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$re" -d $out/pmc_w -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > $out/pmc_w.log 2>&1 \
               && python tools_dev/pmc_traffic.py $out/pmc_f $out/pmc_w > $out/pmc_traffic.json ;;
    gtest)   timeout -k 10 300 python -u -m pytest tests/test_graphed_forward_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $out/gtest.log 2>&1 ;;
    pwtest)  timeout -k 10 300 python -u -m pytest tests/test_pwgemm_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $out/pwtest.log 2>&1 ;;
    pwbench) timeout -k 10 300 python tools_dev/pwbench.py > $out/pwbench.log 2>&1 ;;
    pwpmc)   timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS --kernel-include-regex pw_gemm_gelu -d $out/pwpmc -o run --output-format csv -- python3 tools_dev/pwbench.py > $out/pwpmc.log 2>&1 ;;
    g8pmc) timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $out/g8kt -o run --output-format csv -- python3 tools_dev/g8prof.py > $out/g8kt.log 2>&1 && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --kernel-include-regex gemm8_kernel -d $out/g8pmc -o run --output-format csv -- python3 tools_dev/g8prof.py > $out/g8pmc.log 2>&1 && timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVES TCC_HIT_sum TCC_MISS_sum --kernel-include-regex gemm8_kernel -d $out/g8pmc2 -o run --output-format csv -- python3 tools_dev/g8prof.py > $out/g8pmc2.log 2>&1 ;;
    dwmpmc) timeout -k 10 120 python tools_dev/decbench.py --only dw > $out/dwm_bench.log 2>&1 && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --kernel-include-regex dwm_fwd -d $out/dwmpmc -o run --output-format csv -- python3 tools_dev/decbench.py --only dw > $out/dwmpmc.log 2>&1 && timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum --kernel-include-regex dwm_fwd -d $out/dwmpmc2 -o run --output-format csv -- python3 tools_dev/decbench.py --only dw > $out/dwmpmc2.log 2>&1 ;;
    r4tests) timeout -k 10 900 python -u -m pytest tests/test_gemm_gpu.py tests/test_vgg_gpu.py tests/test_style_rmsnorm_gpu.py tests/test_graphed_forward_gpu.py tests/test_fullsize_bwd_gpu.py tests/test_decoder_gpu.py tests/test_gemm_shapes_gpu.py -m gpu --maxfail=10 -v --timeout 240 --timeout-method thread > $out/r4tests.log 2>&1 ;;
    r4tests2) timeout -k 10 900 python -u -m pytest tests/test_graphed_forward_gpu.py tests/test_fullsize_bwd_gpu.py tests/test_decoder_gpu.py tests/test_gemm_shapes_gpu.py -m gpu --maxfail=10 -v -s --timeout 240 --timeout-method thread > $out/r4tests2.log 2>&1 ;;
    r4tests3) timeout -k 10 600 python -u -m pytest tests/test_gemm_shapes_gpu.py tests/test_gemm_gpu.py -m gpu --maxfail=10 -v --timeout 240 --timeout-method thread > $out/r4tests3.log 2>&1 ;;
    r4tests4) timeout -k 10 600 python -u -m pytest tests/test_vgg_gpu.py tests/test_lpips_gpu.py tests/test_gemm_shapes_gpu.py tests/test_networks_gpu.py -m gpu --maxfail=10 -v --timeout 240 --timeout-method thread > $out/r4tests4.log 2>&1 ;;
    r4tests5) timeout -k 10 600 python -u -m pytest tests/test_style_rmsnorm_gpu.py tests/test_vgg_gpu.py tests/test_lpips_gpu.py tests/test_decoder_gpu.py tests/test_networks_gpu.py -m gpu --maxfail=10 -v --timeout 240 --timeout-method thread > $out/r4tests5.log 2>&1 ;;
    r4tests6) timeout -k 10 600 python -u -m pytest tests/test_style_rmsnorm_gpu.py tests/test_decoder_gpu.py -m gpu --maxfail=10 -v --timeout 240 --timeout-method thread > $out/r4tests6.log 2>&1 ;;
    r4tests7) timeout -k 10 600 python -u -m pytest tests/test_vgg_gpu.py tests/test_lpips_gpu.py tests/test_networks_gpu.py -m gpu --maxfail=10 -v --timeout 240 --timeout-method thread > $out/r4tests7.log 2>&1 ;;
    vggbench) timeout -k 10 300 python tools_dev/vggbench.py > $out/vggbench.log 2>&1 ;;
    benchab) VFM_LPIPS_VGG=torch timeout -k 10 600 python bench.py --no-cpu-baseline > $out/bench_a.log 2>&1 && timeout -k 10 600 python bench.py --no-cpu-baseline > $out/bench_b.log 2>&1 && VFM_LPIPS_VGG=torch timeout -k 10 600 python bench.py --no-cpu-baseline > $out/bench_c.log 2>&1 ;;
    convpmc) timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS --kernel-include-regex conv3x3_kernel -d $out/convpmc -o run --output-format csv -- python3 tools_dev/vggbench.py > $out/convpmc.log 2>&1 && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --kernel-include-regex conv3x3_kernel -d $out/convpmc2 -o run --output-format csv -- python3 tools_dev/vggbench.py > $out/convpmc2.log 2>&1 ;;
    dwpmc) timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS --kernel-include-regex "dwr_fwd|blur_fwd" -d $out/dwpmc -o run --output-format csv -- python3 tools_dev/decbench.py --only dw,blur > $out/dwpmc.log 2>&1 && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM --kernel-include-regex "dwr_fwd|blur_fwd" -d $out/dwpmc2 -o run --output-format csv -- python3 tools_dev/decbench.py --only dw,blur > $out/dwpmc2.log 2>&1 ;;
    mlppmc) timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS --kernel-include-regex mlp_fwd -d $out/mlppmc -o run --output-format csv -- python3 tools_dev/pwbench.py > $out/mlppmc.log 2>&1 && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM --kernel-include-regex mlp_fwd -d $out/mlppmc2 -o run --output-format csv -- python3 tools_dev/pwbench.py > $out/mlppmc2.log 2>&1 ;;
    gdebug)  timeout -k 10 300 python tools_dev/graph_debug.py > $out/gdebug.log 2>&1 ;;
    benchfind) MIOPEN_FIND_MODE=NORMAL VFM_CUDNN_BENCHMARK=1 timeout -k 10 900 python bench.py --no-cpu-baseline > $out/benchfind.log 2>&1 ;;
    tune)    ( while sleep 30; do echo "tick $(date +%T)"; done ) & tk=$!
             timeout -k 10 1000 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --tunableop tune --tunableop-out $out/gemm_results.csv > $out/tune.log 2>&1; rc0=$?
             kill $tk; (exit $rc0) ;;
    benchtun) timeout -k 10 600 python bench.py --no-cpu-baseline --tunableop use > $out/benchtun.log 2>&1 ;;
    benchnf) VFM_NO_FUSED_MLP=1 timeout -k 10 600 python bench.py --no-cpu-baseline > $out/benchnf.log 2>&1 ;;
    benchng) timeout -k 10 600 python bench.py --no-cpu-baseline --no-graphs > $out/benchng.log 2>&1 ;;
    decbench) timeout -k 10 300 python tools_dev/decbench.py > $out/decbench.log 2>&1 ;;
    opbench) timeout -k 10 300 python tools_dev/opbench.py > $out/opbench.log 2>&1 ;;
    dtests)  timeout -k 10 600 python -m pytest tests/test_decoder_gpu.py -q -x > $out/dtests.log 2>&1 ;;
    bsmall)  timeout -k 10 900 python bench.py --batch 8 --steps 2 --warmup 2 --trace --no-cpu-baseline > $out/bsmall.log 2>&1 ;;
    btrace)  timeout -k 10 900 python bench.py --steps 3 --warmup 2 --trace --no-cpu-baseline > $out/btrace.log 2>&1 ;;
    bsteps)  timeout -k 10 900 python bench.py --steps 6 --warmup 2 --trace --no-cpu-baseline > $out/bsteps.log 2>&1 ;;
    bstepsng) timeout -k 10 900 python bench.py --steps 6 --warmup 2 --trace --no-cpu-baseline --no-gc-freeze > $out/bstepsng.log 2>&1 ;;
    wdsbench) timeout -k 10 600 python tools_dev/wdsbench.py > $out/wdsbench.log 2>&1 ;;
    torchops) timeout -k 10 600 python tools_dev/torchops.py > $out/torchops.log 2>&1 ;;
    cparents) timeout -k 10 600 python tools_dev/copy_parents.py > $out/cparents.log 2>&1 ;;
    tprof)   timeout -k 10 600 python tools_dev/torchprof.py --out $out/tp > $out/tprof.log 2>&1 ;;
    gemmbench8) timeout -k 10 300 python tools_dev/gemmbench.py > $out/gemmbench.log 2>&1 ;;
    ptests)  timeout -k 10 ${PT_TIMEOUT:-900} python -u -m pytest $PT -m gpu -v -s --timeout ${PT_CASE:-240} --timeout-method thread > $out/ptests.log 2>&1 ;;
    ptest)   timeout -k 10 ${PT_TIMEOUT:-900} python -u -m pytest $PT -m gpu -v --timeout ${PT_CASE:-240} --timeout-method thread > $out/ptest.log 2>&1 ;;
    attnbench) timeout -k 10 300 python tools_dev/attnbench.py > $out/attnbench.log 2>&1 ;;
    gemmbench) timeout -k 10 300 python tools_dev/gemmbench.py > $out/gemmbench.log 2>&1 ;;
    gemm6bench) timeout -k 10 300 python tools_dev/gemm6bench.py > $out/gemm6bench.log 2>&1 ;;
    g8sched) timeout -k 10 300 python tools_dev/g8sched.py > $out/g8sched.log 2>&1 ;;
    g8k) timeout -k 10 300 python tools_dev/g8ksweep.py > $out/g8k.log 2>&1 && G8_DEEP=0 timeout -k 10 300 python tools_dev/g8ksweep.py > $out/g8k0.log 2>&1 ;;
    g8pmc1) timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --kernel-include-regex gemm8_kernel -d $out/p1 -o run --output-format csv -- python3 tools_dev/g8one.py > $out/p1.log 2>&1 && timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum --kernel-include-regex gemm8_kernel -d $out/p2 -o run --output-format csv -- python3 tools_dev/g8one.py > $out/p2.log 2>&1 && timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex gemm8_kernel -d $out/p3 -o run --output-format csv -- python3 tools_dev/g8one.py > $out/p3.log 2>&1 ;;
    g9pmc) for kd in g9 blas; do
             G8_KIND=$kd G8_K=8192 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS -d $out/p1_$kd -o run --output-format csv -- python3 tools_dev/g8one.py > $out/p1_$kd.log 2>&1 || exit 1
             G8_KIND=$kd G8_K=8192 timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT -d $out/p2_$kd -o run --output-format csv -- python3 tools_dev/g8one.py > $out/p2_$kd.log 2>&1 || exit 1
           done ;;
    g8st) timeout -k 10 300 python tools_dev/g8stamps.py > $out/g8st.log 2>&1 ;;
    mlpbench) timeout -k 10 300 python tools_dev/mlpbench.py > $out/mlpbench.log 2>&1 ;;
    gc1) timeout -k 10 400 python tools_dev/graph_c1.py > $out/gc1.log 2>&1 && GC1_NORM=mm timeout -k 10 400 python tools_dev/graph_c1.py > $out/gc1_mm.log 2>&1 ;;
    opsites) timeout -k 10 600 python tools_dev/opsites.py > $out/opsites.log 2>&1 ;;
    opsitest) OPSITES_TIME=1 timeout -k 10 600 python tools_dev/opsites.py > $out/opsites_timed.log 2>&1 ;;
    gapprof) timeout -k 10 600 python tools_dev/gapprof.py 1 > $out/gapprof.log 2>&1 ;;
    benchg) timeout -k 10 600 python bench.py --graphs on --no-cpu-baseline > $out/benchg.log 2>&1 && timeout -k 10 600 python bench.py --no-cpu-baseline > $out/bench_e.log 2>&1 ;;
    benchst) VFM_STYLE_HIP=1 timeout -k 10 600 python bench.py --no-cpu-baseline > $out/bench_st1.log 2>&1 && timeout -k 10 600 python bench.py --no-cpu-baseline > $out/bench_st0.log 2>&1 ;;
    styleprof) timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/styleprof -o run --output-format csv -- python3 tools_dev/stylebench.py > $out/styleprof.log 2>&1 ;;
    stylebench) timeout -k 10 300 python tools_dev/stylebench.py > $out/stylebench.log 2>&1 ;;
    decgn) timeout -k 10 300 python tools_dev/decbench.py --only gn,dw > $out/decgn.log 2>&1 ;;
    g4abl) timeout -k 10 300 python tools_dev/g4abl.py > $out/g4abl.log 2>&1 ;;
    g4bench) timeout -k 10 400 python tools_dev/g4bench.py > $out/g4bench.log 2>&1 ;;
    bf16bench) timeout -k 10 300 python tools_dev/bf16bench.py > $out/bf16bench.log 2>&1 ;;
    bf16dw) BF16BENCH_DW_ONLY=1 timeout -k 10 300 python tools_dev/bf16bench.py > $out/bf16dw.log 2>&1 ;;
    attn32bench) timeout -k 10 300 python tools_dev/attn32bench.py > $out/attn32bench.log 2>&1 ;;
    dqab) for o in 1 2 1 2; do VFM_ATTN32_DQ_OCC=$o timeout -k 10 300 python tools_dev/attn32bench.py > $out/attn32_dqocc${o}_$RANDOM.log 2>&1 || exit 1; done ;;
    attn32ab) for o in 1 2 1 2; do VFM_ATTN32_OCC=$o timeout -k 10 300 python tools_dev/attn32bench.py > $out/attn32_occ${o}_$RANDOM.log 2>&1 || exit 1; done ;;
    g128ab) for w in 4 8 4 8; do VFM_GEMM128_WAVES=$w timeout -k 10 300 python tools_dev/gemm6bench.py > $out/gemm6_w${w}_$RANDOM.log 2>&1 || exit 1; done ;;
    convab) for w in 128 256 128 256; do VFM_CONV_N64=$w timeout -k 10 300 python tools_dev/vggbench.py > $out/vgg_n64_${w}_$RANDOM.log 2>&1 || exit 1; done ;;
    r4tests8) timeout -k 10 900 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_shapes_gpu.py tests/test_attention_f32_gpu.py tests/test_networks_gpu.py -m gpu --maxfail=10 -v --timeout 240 --timeout-method thread > $out/r4tests8.log 2>&1 ;;
    r4tests9) timeout -k 10 900 python -u -m pytest tests/test_networks_gpu.py tests/test_decoder_gpu.py tests/test_fullsize_bwd_gpu.py tests/test_configs_gpu.py -m gpu --maxfail=10 -v --timeout 240 --timeout-method thread > $out/r4tests9.log 2>&1 ;;
    r4tests10) timeout -k 10 900 python -u -m pytest tests/test_attention_f32_gpu.py tests/test_networks_gpu.py tests/test_fullsize_gpu.py tests/test_fullsize_bwd_gpu.py tests/test_patchgan_gpu.py -m gpu --maxfail=10 -v --timeout 240 --timeout-method thread > $out/r4tests10.log 2>&1 ;;
    r4tests11) timeout -k 10 900 python -u -m pytest tests/test_decoder_attention_gpu.py tests/test_networks_gpu.py tests/test_fullsize_gpu.py tests/test_fullsize_bwd_gpu.py tests/test_graphed_forward_gpu.py -m gpu --maxfail=10 -v --timeout 240 --timeout-method thread > $out/r4tests11.log 2>&1 ;;
    r4tests12) timeout -k 10 900 python -u -m pytest tests/test_specnorm_gpu.py tests/test_patchgan_gpu.py tests/test_networks_gpu.py tests/test_decoder_gpu.py tests/test_attention_f32_gpu.py tests/test_decoder_attention_gpu.py tests/test_gemm_gpu.py -m gpu --maxfail=10 -v --timeout 240 --timeout-method thread > $out/r4tests12.log 2>&1 ;;
    r4tests13) timeout -k 10 900 python -u -m pytest tests/test_decoder_gpu.py tests/test_networks_gpu.py tests/test_fullsize_bwd_gpu.py tests/test_fullsize_gpu.py tests/test_configs_gpu.py -m gpu --maxfail=10 -v --timeout 240 --timeout-method thread > $out/r4tests13.log 2>&1 ;;
    abtimer) bash tools_dev/ab_args.sh $tag/abtimer "" "--no-kernel-timer" ;;
    abtimer3) bash tools_dev/ab3_args.sh $tag/abtimer3 "--timer-every 16" "--timer-every 256" "--no-kernel-timer" ;;
    newpaths) VFM_IM2COL_ROWS=1 VFM_SPLIT_PLANAR8=1 timeout -k 10 900 python -u -m pytest tests/test_specnorm_gpu.py tests/test_patchgan_gpu.py tests/test_gemm_gpu.py tests/test_networks_gpu.py tests/test_fullsize_gpu.py -m gpu --maxfail=10 -v --timeout 240 --timeout-method thread > $out/newpaths.log 2>&1 ;;
    abnew) bash tools_dev/ab_env2.sh $tag/abnew ;;
    dkdvtest) VFM_ATTN32_DKDV_OCC=2 timeout -k 10 600 python -u -m pytest tests/test_attention_f32_gpu.py tests/test_decoder_attention_gpu.py -m gpu -v --timeout 120 --timeout-method thread > $out/dkdvtest.log 2>&1 ;;
    dkdvab) for o in 1 2 1 2; do VFM_ATTN32_DKDV_OCC=$o timeout -k 10 300 python tools_dev/attn32bench.py > $out/attn32_dkdvocc${o}_$RANDOM.log 2>&1 || exit 1; done ;;
    dinobench) timeout -k 10 300 python tools_dev/dinobench.py > $out/dinobench.log 2>&1 ;;
    abfold) bash tools_dev/ab_env.sh $tag/abfold VFM_DHEAD_FOLDED 0 1 ;;
    abdw) bash tools_dev/ab_env.sh $tag/abdw VFM_DW_STREAM 0 1 ;;
    attn32pmc) ATTN32_ONLY=adapter timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex attn32 -d $out/a1 -o run --output-format csv -- python3 tools_dev/attn32bench.py > $out/a1.log 2>&1 && ATTN32_ONLY=adapter timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex attn32 -d $out/a2 -o run --output-format csv -- python3 tools_dev/attn32bench.py > $out/a2.log 2>&1 ;;
    timerchk) timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $out/tchk -o run --output-format csv -- python3 tools_dev/timer_check.py > $out/timerchk.log 2>&1 ;;
    smoke)   timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  rc=$?
  echo "=== step $s rc=$rc $(date +%T)" | tee -a $out/steps.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
