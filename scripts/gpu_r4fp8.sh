#!/bin/bash
# round 4: FP8 delayed-scaling step profile on the final tree
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run bench_fp8 300 python -u bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe delayed
run prof_fp8 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_fp8 -o run -- python -u bench.py --steps 2 --warmup 2 --fp8 --fp8-recipe delayed
run sb_fp8 120 python -u scripts/step_breakdown.py "$(find $OUT/prof_fp8 -name '*kernel_trace.csv' | head -1)"
