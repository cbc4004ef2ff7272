#!/bin/bash
# fp8 backward without transposed copies: tr_b8 probe, fp8 kernel tests, fp8 bench A/B
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run tr8 60 python -u scripts/exp/tr8_probe.py
run fp8_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "fp8 or splitk or tail_split" -m gpu
grep -qE "[0-9]+ failed" $OUT/fp8_tests.log && exit 1
run bench_fp8 500 python -u bench.py --steps 10 --warmup 3 --eager-baseline off --fp8 --fp8-recipe delayed
grep '"metric"' $OUT/bench_fp8.log | head -1
export LTA_FP8_TRANSPOSED=1
run bench_fp8_t 500 python -u bench.py --steps 10 --warmup 3 --eager-baseline off --fp8 --fp8-recipe delayed
grep '"metric"' $OUT/bench_fp8_t.log | head -1
unset LTA_FP8_TRANSPOSED
rm -rf $OUT/prof_fp8
run prof_fp8 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_fp8 -o run --output-format csv -- python bench.py --steps 4 --warmup 2 --eager-baseline off --fp8 --fp8-recipe delayed
python scripts/step_breakdown.py $(ls $OUT/prof_fp8/*/run_kernel_trace.csv $OUT/prof_fp8/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/fp8_step_breakdown.txt 2>&1
head -32 $OUT/fp8_step_breakdown.txt
run hipfuse_test 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hipfuse.py -m gpu
rm -rf $OUT/prof_gpt2
run prof_gpt2 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_gpt2 -o run --output-format csv -- python scripts/gpt2_step_profile.py
python scripts/step_breakdown.py $(ls $OUT/prof_gpt2/*/run_kernel_trace.csv $OUT/prof_gpt2/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/gpt2_breakdown.txt 2>&1
head -30 $OUT/gpt2_breakdown.txt
