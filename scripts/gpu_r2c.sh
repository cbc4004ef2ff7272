#!/bin/bash
# Round-2 session C: headline bench (bf16 + the three FP8 recipes) and the bf16 kernel profile.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run bench_bf16 300 python -u bench.py --steps 10 --warmup 3
run bench_fp8_current 300 python -u bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe current
run bench_fp8_delayed 300 python -u bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe delayed
run bench_fp8_mxfp8 300 python -u bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe mxfp8
run prof_bf16 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_bf16 -o run --output-format csv -- python -u bench.py --steps 5 --warmup 2
