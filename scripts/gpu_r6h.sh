#!/bin/bash
# round 3: cast_transpose pairwise-conversion A/B (new build, then the previous build) + fp8 kernel tests
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run fp8tests 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "fp8"
cp lightning_thunder_amd/ops/_lta_kernels.so lightning_thunder_amd/ops/_lta_kernels_new.so
run ct_new 200 python -u scripts/cast_transpose_bench.py
mv gpurun_out/cast_transpose_bench.json gpurun_out/cast_transpose_bench_new.json
cp lightning_thunder_amd/ops/_lta_kernels_prev.so lightning_thunder_amd/ops/_lta_kernels.so
run ct_old 200 python -u scripts/cast_transpose_bench.py
cp lightning_thunder_amd/ops/_lta_kernels_new.so lightning_thunder_amd/ops/_lta_kernels.so
run hipfuse_gpu 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_hipfuse.py -m gpu
rm -rf $OUT/prof_gpt2b
run prof_gpt2b 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_gpt2b -o run --output-format csv -- python scripts/gpt2_step_profile.py
