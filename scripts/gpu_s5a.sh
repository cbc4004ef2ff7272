#!/bin/bash
# Round 5, session a: retired attention / GEMM variants -> numerics of the remaining kernels; default
# bench (now with the eager baseline).
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_k 600 python -u -m pytest tests/test_hip_kernels.py tests/test_gpu_7b_shape.py tests/test_optim_overlap.py -x -q --timeout 120 --timeout-method thread
run bench 600 python -u bench.py
exit 0
