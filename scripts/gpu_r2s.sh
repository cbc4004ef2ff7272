#!/bin/bash
# Tuned library GEMMs (shipped TunableOp table): bench A/B and step profile.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run bench_tuned 600 python bench.py --steps 10 --warmup 3
LTA_TUNED_GEMMS=0 run bench_untuned 600 python bench.py --steps 10 --warmup 3
rm -rf $OUT/prof_bench
run prof_bench 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- python bench.py --steps 3 --warmup 2
python scripts/step_breakdown.py $(ls $OUT/prof_bench/*/run_kernel_trace.csv $OUT/prof_bench/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step_breakdown.txt
