#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_dist_gpu 300 python -u -m pytest tests/test_distributed_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread
run pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run bench 600 python bench.py --steps 10 --warmup 3
