#!/bin/bash
# HF decode: grouped q/k/v projections + SDPA on grouped KV; numerics and generate latency.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_gemv 300 python -u -m pytest tests/test_hip_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemv or hf or generate"
run gen_hf 600 python -u -m lightning_thunder_amd.benchmarks.generate --modes hf_hipgraph,hipgraph --iters 3
rm -rf $OUT/prof_hf
run prof_hf 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_hf -o run --output-format csv -- python -m lightning_thunder_amd.benchmarks.generate --modes hf_hipgraph --iters 1 --warmup 0
