#!/bin/bash
# Llama-2-7B bf16 step breakdown with the dQ-from-dS attention backward; FP8 current / delayed benches
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
rm -rf $OUT/prof_l7
run prof_l7 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_l7 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --eager-baseline off
python scripts/step_breakdown.py $(ls $OUT/prof_l7/*/run_kernel_trace.csv $OUT/prof_l7/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/l7_breakdown.txt 2>&1
rm -f $OUT/prof_l7/*/*kernel_trace.csv $OUT/prof_l7/run_kernel_trace.csv 2>/dev/null
head -30 $OUT/l7_breakdown.txt
run bench_fp8cur 500 python -u bench.py --steps 10 --warmup 3 --eager-baseline off --fp8
grep '"metric"' $OUT/bench_fp8cur.log | head -1
run bench_fp8del 500 python -u bench.py --steps 10 --warmup 3 --eager-baseline off --fp8 --fp8-recipe delayed
grep '"metric"' $OUT/bench_fp8del.log | head -1
