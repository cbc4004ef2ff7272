#!/bin/bash
# round 3: current FP8 (delayed scaling) bench + step profile
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
rm -rf $OUT/prof_fp8b
run fp8bench 600 python -u bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe delayed
run prof_fp8b 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_fp8b -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --fp8 --fp8-recipe delayed
