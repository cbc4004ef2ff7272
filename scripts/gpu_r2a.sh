#!/bin/bash
# Round-2 session A: full GPU tests, 1-GPU headline bench, generation benchmark (all modes).
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run bench 300 python -u bench.py --steps 10 --warmup 3
run gen_bench 420 python -u -m lightning_thunder_amd.benchmarks.generate --iters 3 --modes eager,thunder,hipgraph,hf_eager,hf_thunder,hf_hipgraph
