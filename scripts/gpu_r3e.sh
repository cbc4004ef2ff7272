#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run gen 600 python -u -m lightning_thunder_amd.benchmarks.generate --modes hf_hipgraph,hipgraph --iters 3
