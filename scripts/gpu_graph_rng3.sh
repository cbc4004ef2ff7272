#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_graph 500 python -u -m pytest tests/test_hipgraph.py tests/test_hipfuse.py tests/test_gpu_7b_shape.py -x -q -m gpu --timeout 200 --timeout-method thread
run targets 600 python -u -m lightning_thunder_amd.benchmarks.targets -k nanogpt --executors eager,thunder,thunder+hipgraph
