#!/bin/bash
# round 4: GEMM tail split: numerics (new + existing GEMM / 7B-shape tests), whole-step A/B; FP8 step after the amax-copy removal
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run gemm_tests 400 python -u -m pytest tests/test_hip_kernels.py tests/test_gpu_7b_shape.py -q -m gpu -k "gemm or 7b_shape or linear or matmul" --timeout 180 --timeout-method thread -p no:cacheprovider
run bench_split 400 python -u bench.py --steps 10 --warmup 3
export LTA_GEMM_TAIL_SPLIT=0
run bench_nosplit 400 python -u bench.py --steps 10 --warmup 3
unset LTA_GEMM_TAIL_SPLIT
run bench_fp8 400 python -u bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe delayed
