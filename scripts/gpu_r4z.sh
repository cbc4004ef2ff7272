#!/bin/bash
# round 4: gemm4 production instantiations back to the pre-tail-split code (tail range / split as
# separate TAIL modes): edge-tile + GEMM + 7B-shape tests, old/new A/B, bench with the tail split
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run g4_ab 200 python -u scripts/g4old/ab.py
run gemm_tests 400 python -u -m pytest tests/test_hip_kernels.py tests/test_gpu_7b_shape.py -q -m gpu -k "gemm or 7b_shape or linear or matmul" --timeout 180 --timeout-method thread -p no:cacheprovider
run bench 400 python -u bench.py --steps 10 --warmup 3
