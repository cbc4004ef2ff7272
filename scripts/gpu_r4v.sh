#!/bin/bash
# round 4: final bf16 and FP8-delayed step profiles on the final tree
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
rm -rf $OUT/prof_bench $OUT/prof_fp8
run prof_bench 420 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- python bench.py --steps 3 --warmup 2
python scripts/step_breakdown.py $(ls $OUT/prof_bench/*/run_kernel_trace.csv $OUT/prof_bench/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step_breakdown.txt 2>&1
run prof_fp8 420 rocprofv3 --kernel-trace --stats -d $OUT/prof_fp8 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --fp8 --fp8-recipe delayed
python scripts/step_breakdown.py $(ls $OUT/prof_fp8/*/run_kernel_trace.csv $OUT/prof_fp8/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/fp8_step_breakdown.txt 2>&1
