#!/bin/bash
# Round 5, session e: swapped-operand register epilogue in the production gemm4 (numerics + A/B),
# persistent-tile experiment, bench.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run gemm_tests 600 python -u -m pytest tests/test_hip_kernels.py tests/test_gpu_swiglu_gemm.py tests/test_gpu_7b_shape.py -x -q --timeout 120 --timeout-method thread -k "gemm or qkv or grouped or moe or tail or swiglu or 7b or linear"
run anatomy3 300 python -u scripts/exp/gemm_anatomy.py 0,64,8
run g5exp 400 python -u scripts/exp/gemm5_exp.py
run bench 400 python -u bench.py --eager-baseline off
exit 0
