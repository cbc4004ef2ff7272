#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_rope 300 python -u -m pytest tests/test_hip_kernels.py tests/test_generate.py tests/test_gpu_models.py -m gpu -x -q --timeout 120 --timeout-method thread
run bench 600 python bench.py --steps 10 --warmup 3
rm -rf $OUT/prof_bench
run prof_bench 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- python bench.py --steps 3 --warmup 2
python scripts/step_breakdown.py $OUT/prof_bench/run_kernel_trace.csv > $OUT/step_breakdown.txt
