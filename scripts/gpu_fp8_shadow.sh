#!/bin/bash
# FP8 path fusions: weight shadows emitted by the fused AdamW, the fp8 qkv-RoPE GEMM epilogue; tests,
# the FP8 (delayed) 7B step and its kernel breakdown.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_fp8 300 python -u -m pytest tests/test_hip_kernels.py -x -q -k "shadow or qkv_rope or fp8 or adamw" --timeout 120 --timeout-method thread
run t_fp8_7b 300 python -u -m pytest tests/test_gpu_7b_shape.py -x -q -k "fp8" --timeout 200 --timeout-method thread
run bench_fp8 420 python bench.py --fp8 --fp8-recipe delayed --steps 10 --warmup 3 --eager-baseline off
rm -rf $OUT/prof_fp8
run prof_fp8 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_fp8 -o run --output-format csv -- python bench.py --fp8 --fp8-recipe delayed --steps 3 --warmup 2 --eager-baseline off
