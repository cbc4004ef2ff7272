#!/bin/bash
# qkv-RoPE epilogue (pair form): numerics, bench, step profile; then the 2-rank same-GPU gloo rehearsal.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_fused 400 python -u -m pytest tests/test_gpu_swiglu_gemm.py tests/test_gpu_7b_shape.py -x -v --timeout 200 --timeout-method thread
run bench_bf16 300 python -u bench.py --steps 10 --warmup 3
rm -rf $OUT/prof_bench
run prof_bench 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- python bench.py --steps 3 --warmup 2
python scripts/step_breakdown.py $(ls $OUT/prof_bench/*/run_kernel_trace.csv $OUT/prof_bench/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step_breakdown.txt 2>&1
rm -f $OUT/prof_bench/*/*kernel_trace.csv $OUT/prof_bench/run_kernel_trace.csv 2>/dev/null
run rehearsal 1300 bash scripts/dist_rehearsal.sh
