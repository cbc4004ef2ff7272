#!/bin/bash
# gemm4 with odd K-tile counts (K % 128 == 64) + launch plans: kernel tests, model tests, targets
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_gemm4 400 python -u -m pytest tests/test_hip_kernels.py -x -q -k "gemm4 or gemm_nt or linear" --timeout 120 --timeout-method thread
run t_models 600 python -u -m pytest tests/test_gpu_models.py tests/test_networks.py -x -q -m gpu --timeout 200 --timeout-method thread
run targets 600 python -u -m lightning_thunder_amd.benchmarks.targets -k nanogpt
