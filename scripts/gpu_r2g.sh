#!/bin/bash
# Attention BSHD output / strided dO, residual-fused backward GEMMs and RMSNorm backward:
# kernel numerics, model numerics, traces, headline step, kernel profile.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_kernels 400 python -u -m pytest tests/test_hip_kernels.py tests/test_extend_hip_kernel.py -m gpu -x -q --timeout 120 --timeout-method thread
run pytest_models 400 python -u -m pytest tests/test_gpu_models.py -m gpu -x -q --timeout 200 --timeout-method thread
run traces 300 python -u scripts/dump_traces.py gpurun_out/traces
run bench_bf16 300 python -u bench.py --steps 10 --warmup 3
rm -rf $OUT/prof_bench
run prof_bench 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- python bench.py --steps 3 --warmup 2
