#!/bin/bash
# round 4: bf16 step profile on the current defaults, GPT-2 step profile + generated-kernel roofline
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
rm -rf $OUT/prof_bench $OUT/prof_gpt2
run prof_bench 420 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- python bench.py --steps 3 --warmup 2
python scripts/step_breakdown.py $(ls $OUT/prof_bench/*/run_kernel_trace.csv $OUT/prof_bench/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step_breakdown.txt 2>&1
run roofline 300 python -u scripts/hipfuse_roofline.py
run prof_gpt2 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_gpt2 -o run --output-format csv -- python scripts/gpt2_step_profile.py
