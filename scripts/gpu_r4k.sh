#!/bin/bash
# round 4: dQ v2/v3/v4 A/B, re-run of the tests that failed on the codegen / decode fixes, bf16 step profile
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run dq_v4 300 python -u scripts/attn_dq_v3_check.py
run rope_bwd 300 python -u -m pytest tests/test_hip_kernels.py tests/test_gpu_7b_shape.py -q -m gpu -k "fused_rope or 7b_shape" --timeout 180 --timeout-method thread -p no:cacheprovider
run refail 500 python -u -m pytest tests/test_generate.py tests/test_networks.py tests/test_hipfuse.py -q -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider
run refail_ops 300 python -u -m pytest tests/test_ops.py -q -m gpu -k "interpolate or binary_cross or gaussian_nll or heaviside" --timeout 120 --timeout-method thread -p no:cacheprovider
rm -rf $OUT/prof_bench
run prof_bench 420 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- python bench.py --steps 3 --warmup 2
python scripts/step_breakdown.py $(ls $OUT/prof_bench/*/run_kernel_trace.csv $OUT/prof_bench/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step_breakdown.txt 2>&1
