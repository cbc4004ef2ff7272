#!/bin/bash
# round 3: gemm4 register-staged A/B, kernel tests after fixes
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run gemm4 600 python -u scripts/gemm4_bench.py --rounds 2 --iters 20 --variants 1,3
run kern 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_index_ops.py tests/test_hipfuse.py -k "claimed or bias_grad or column"
run fp8_fsdp 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fp8_fsdp.py
