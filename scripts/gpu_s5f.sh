#!/bin/bash
# Round 5, session f: register epilogue with single-instruction bf16 packing; old-vs-new A/B on one box;
# fp8 GEMM numerics (register epilogue ported); step profile.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run gemm_tests 600 python -u -m pytest tests/test_hip_kernels.py tests/test_gpu_swiglu_gemm.py tests/test_gpu_7b_shape.py -x -q --timeout 120 --timeout-method thread -k "gemm or qkv or grouped or moe or tail or swiglu or 7b or linear or fp8"
run epi_ab 400 python -u scripts/exp/gemm_epi_ab.py
run bench 400 python -u bench.py --eager-baseline off
rm -rf $OUT/prof_bench
run prof_bench 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --eager-baseline off
python scripts/step_breakdown.py $(ls $OUT/prof_bench/*/run_kernel_trace.csv $OUT/prof_bench/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step_breakdown.txt 2>&1
rm -f $OUT/prof_bench/*/*kernel_trace.csv $OUT/prof_bench/run_kernel_trace.csv 2>/dev/null
exit 0
