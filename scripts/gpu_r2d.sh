#!/bin/bash
# Kernel profiles of the delayed-scaling and MXFP8 FP8 benches.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run prof_delayed 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_delayed -o run --output-format csv -- python -u bench.py --steps 3 --warmup 2 --fp8 --fp8-recipe delayed
run prof_mx 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_mx -o run --output-format csv -- python -u bench.py --steps 3 --warmup 2 --fp8 --fp8-recipe mxfp8
