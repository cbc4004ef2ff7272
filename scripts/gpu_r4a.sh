#!/bin/bash
# AdamW unroll check: kernel numerics, step profile, bench.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_adamw 200 python -u -m pytest tests/test_hip_kernels.py -k adamw -x -v --timeout 120 --timeout-method thread
rm -rf $OUT/prof_bench
run prof_bench 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- python bench.py --steps 3 --warmup 2
run breakdown 60 python scripts/step_breakdown.py $OUT/prof_bench/run_kernel_trace.csv
run bench 480 python bench.py --steps 10 --warmup 3
rm -f $OUT/prof_bench/run_kernel_trace.csv
