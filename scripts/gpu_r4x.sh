#!/bin/bash
# round 4: edge-tile epilogue diagnostic; prefetching fp8 cast_transpose (A/B + bitwise vs the round-3
# kernels); AdamW with pinned rounding and non-temporal streaming by default; FP8 delayed step + profile
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run edge_diag 200 python -u scripts/gemm_edge_diag.py
run cast_ab 300 python -u scripts/cast_transpose_bench.py
run tests 400 python -u -m pytest tests/test_optim_overlap.py tests/test_hip_kernels.py tests/test_transforms_misc.py tests/test_fp8_fsdp.py -q -m gpu -k "adamw or overlap or fp8 or cast" --timeout 180 --timeout-method thread -p no:cacheprovider
run adamw_ab 200 python -u scripts/adamw_nt_ab.py
run bench_fp8 400 python -u bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe delayed
run prof_fp8 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_fp8 -o run -- python -u bench.py --steps 2 --warmup 2 --fp8 --fp8-recipe delayed
run sb_fp8 120 python -u scripts/step_breakdown.py $OUT/prof_fp8/run_kernel_trace.csv
