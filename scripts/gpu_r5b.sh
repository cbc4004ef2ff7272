#!/bin/bash
# round 3: gemm4 MN-major fix A/B + masked/dropout attention + FP8xFSDP on the GPU
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run gemm4 600 python -u scripts/gemm4_bench.py --rounds 2 --iters 20
run attn_ex 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_attention_ex.py
run fp8_fsdp 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_fp8_fsdp.py
