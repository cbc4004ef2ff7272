#!/bin/bash
# v4 forward: direct-store bf16 epilogue vs the previous build (A/B), Q8 staged epilogue in the FP8 step
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run epi_ab 300 python -u scripts/attn_epi_ab.py scripts/exp/old_fwd4.so
run t_attn 400 python -u -m pytest tests/test_hip_kernels.py tests/test_attention_ex.py tests/test_gpu_7b_shape.py -x -q -k "attn or attention or sdpa or fp8" --timeout 300 --timeout-method thread
run bench_fp8 420 python bench.py --fp8 --fp8-recipe delayed --steps 10 --warmup 3 --eager-baseline off
rm -rf $OUT/prof_fp8q
run prof_fp8q 500 rocprofv3 --kernel-trace -d $OUT/prof_fp8q -o run --output-format csv -- python bench.py --fp8 --fp8-recipe delayed --steps 3 --warmup 2 --eager-baseline off
run bench_bf16 420 python bench.py --steps 10 --warmup 3 --eager-baseline off
