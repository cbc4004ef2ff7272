#!/bin/bash
# host-path trims: GEMM launch plans, hipfuse output specs; GPU tests of the GEMM paths, then targets.py
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_gemm 600 python -u -m pytest tests/test_gpu_7b_shape.py tests/test_gpu_swiglu_gemm.py tests/test_hipfuse.py tests/test_gpu_models.py -x -q --timeout 200 --timeout-method thread
run targets 600 python -u -m lightning_thunder_amd.benchmarks.targets
run host_prof 300 python -u scripts/host_overhead_profile.py
