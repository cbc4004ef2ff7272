#!/bin/bash
# round 3: fp8 4-wave GEMM correctness + A/B, then the FP8 step
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run fp8test 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "fp8"
run fp8gemm 600 python -u scripts/fp8_gemm_bench.py
run bench_fp8 600 python -u bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe delayed
