#!/bin/bash
# round 3: D=96 dK/dV staging fix -> attention GPU tests; 1-GPU bench + its rocprof step breakdown
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
rm -rf $OUT/prof_bench3
run attn_tests2 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py tests/test_attention_ex.py -k "flash or attention or masked or dropout or sdpa"
run bench2 600 python -u bench.py --steps 10 --warmup 3
run prof_bench3 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench3 -o run --output-format csv -- python bench.py --steps 3 --warmup 2
