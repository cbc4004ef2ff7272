#!/bin/bash
# Round-2 session B: hipGraph storage tests, remaining GPU tests, generation benchmark.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_hg 300 python -u -m pytest tests/test_hipgraph.py tests/test_hip_kernels.py -m gpu -q --timeout 200 --timeout-method thread -k "hipgraph or generate or runner"
run pytest_gpu 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
run gen_bench 420 python -u -m lightning_thunder_amd.benchmarks.generate --iters 3 --modes eager,thunder,hipgraph,hf_eager,hf_thunder,hf_hipgraph
