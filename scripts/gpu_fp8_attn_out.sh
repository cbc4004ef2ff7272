#!/bin/bash
# FP8 attention-output e4m3 epilogue: kernel + model tests, FP8 7B step + breakdown, bf16 step unchanged
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_fp8k 300 python -u -m pytest tests/test_hip_kernels.py -x -q -k "fp8 or attn or rms" --timeout 120 --timeout-method thread
run t_fp8_7b 400 python -u -m pytest tests/test_gpu_7b_shape.py -x -q -k "fp8" --timeout 300 --timeout-method thread
run bench_fp8 420 python bench.py --fp8 --fp8-recipe delayed --steps 20 --warmup 5 --eager-baseline off
rm -rf $OUT/prof_fp8
run prof_fp8 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_fp8 -o run --output-format csv -- python bench.py --fp8 --fp8-recipe delayed --steps 3 --warmup 2 --eager-baseline off
run bench_bf16 420 python bench.py --steps 20 --warmup 5 --eager-baseline off
