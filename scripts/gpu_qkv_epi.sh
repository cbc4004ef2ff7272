#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_qkv 300 python -u -m pytest tests/test_hip_kernels.py tests/test_gpu_swiglu_gemm.py -x -q -k "qkv_rope" --timeout 120 --timeout-method thread
run qkv_bench 300 python -u scripts/qkv_epilogue_bench.py
run bench_bf16 420 python bench.py --steps 10 --warmup 3 --eager-baseline off
run bench_fp8 420 python bench.py --fp8 --fp8-recipe delayed --steps 10 --warmup 3 --eager-baseline off
