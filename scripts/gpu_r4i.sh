#!/bin/bash
# round 4: evidence refresh on the current tree: speedup vs eager, FP8 delayed step, GPT-2 step
# profile + generated-kernel roofline
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run bench_eager 900 python -u bench.py --steps 10 --warmup 3 --eager-baseline
run bench_fp8 600 python -u bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe delayed
run roofline 400 python -u scripts/hipfuse_roofline.py
run prof_gpt2 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_gpt2 -o run --output-format csv -- python scripts/gpt2_step_profile.py
rm -rf $OUT/prof_bench
run prof_bench 900 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- python bench.py --steps 3 --warmup 2
python scripts/step_breakdown.py $(ls $OUT/prof_bench/*/run_kernel_trace.csv $OUT/prof_bench/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step_breakdown.txt 2>&1
