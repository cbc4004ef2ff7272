#!/bin/bash
# v4 attention forward with the LDS-staged row-store epilogue (+ e4m3 side output): tests, bf16 / FP8 steps, breakdowns
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_attn 400 python -u -m pytest tests/test_hip_kernels.py tests/test_attention_ex.py -x -q -k "attn or attention or sdpa or fp8" --timeout 120 --timeout-method thread
run t_fp8_7b 400 python -u -m pytest tests/test_gpu_7b_shape.py -x -q -k "fp8" --timeout 300 --timeout-method thread
run bench_bf16 420 python bench.py --steps 20 --warmup 5 --eager-baseline off
run bench_fp8 420 python bench.py --fp8 --fp8-recipe delayed --steps 20 --warmup 5 --eager-baseline off
rm -rf $OUT/prof_bf16e $OUT/prof_fp8e
run prof_bf16e 500 rocprofv3 --kernel-trace -d $OUT/prof_bf16e -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --eager-baseline off
run prof_fp8e 500 rocprofv3 --kernel-trace -d $OUT/prof_fp8e -o run --output-format csv -- python bench.py --fp8 --fp8-recipe delayed --steps 3 --warmup 2 --eager-baseline off
