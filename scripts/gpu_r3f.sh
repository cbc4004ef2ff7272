#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run gen 600 python -u -m lightning_thunder_amd.benchmarks.generate --modes hf_hipgraph,hipgraph --iters 3
