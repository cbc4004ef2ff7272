#!/bin/bash
# GPT-2 step with the wider column grid; fp8 current-scaling bench; default bench (eager baseline on)
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
rm -rf $OUT/prof_gpt2
run prof_gpt2 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_gpt2 -o run --output-format csv -- python scripts/gpt2_step_profile.py
python scripts/step_breakdown.py $(ls $OUT/prof_gpt2/*/run_kernel_trace.csv $OUT/prof_gpt2/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/gpt2_breakdown.txt 2>&1
head -24 $OUT/gpt2_breakdown.txt
run roofline 300 python -u scripts/hipfuse_roofline.py --json $OUT/hipfuse_roofline.json
grep -v amdgpu.ids $OUT/roofline.log | tail -12
run bench_fp8cur 500 python -u bench.py --steps 10 --warmup 3 --eager-baseline off --fp8
grep '"metric"' $OUT/bench_fp8cur.log | head -1
run bench 500 python -u bench.py
grep '"metric"' $OUT/bench.log | head -1
