#!/bin/bash
# RMSNorm backward with the residual prefetched: numerics, bf16 bench + step profile.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_rms 300 python -u -m pytest tests/test_hip_kernels.py -k "rmsnorm or fp8 or gemm" -x -q --timeout 120 --timeout-method thread
run bench_bf16 300 python -u bench.py --steps 10 --warmup 3
rm -rf $OUT/prof_bench
run prof_bench 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- python bench.py --steps 3 --warmup 2
python scripts/step_breakdown.py $(ls $OUT/prof_bench/*/run_kernel_trace.csv $OUT/prof_bench/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step_breakdown.txt 2>&1
rm -f $OUT/prof_bench/*/*kernel_trace.csv $OUT/prof_bench/run_kernel_trace.csv 2>/dev/null
exit 0
