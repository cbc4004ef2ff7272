#!/bin/bash
# 128x128 fp8 cast+transpose: numerics, micro-benchmark A/B, FP8 delayed step + profile.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_cast 300 python -u -m pytest tests/test_hip_kernels.py -k "fp8" -x -v --timeout 120 --timeout-method thread
run ct_new 200 python -u scripts/cast_transpose_bench.py
cp $OUT/cast_transpose_bench.json $OUT/ct_new.json
LTA_CAST_T64=1 run ct_old 200 python -u scripts/cast_transpose_bench.py
cp $OUT/cast_transpose_bench.json $OUT/ct_old.json
run bench_fp8d 300 python -u bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe delayed
LTA_CAST_T64=1 run bench_fp8d_old 300 python -u bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe delayed
rm -rf $OUT/prof_fp8
run prof_fp8 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_fp8 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --fp8 --fp8-recipe delayed
python scripts/step_breakdown.py $(ls $OUT/prof_fp8/*/run_kernel_trace.csv $OUT/prof_fp8/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/fp8_step_breakdown.txt 2>&1
rm -f $OUT/prof_fp8/*/*kernel_trace.csv $OUT/prof_fp8/run_kernel_trace.csv 2>/dev/null
exit 0
