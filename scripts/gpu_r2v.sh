#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_dist_gpu 300 python -u -m pytest tests/test_distributed_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread
LTA_GEMM_SELECT_ROUNDS=1 run bench_r1 600 python bench.py --steps 10 --warmup 3
run bench_r3 600 python bench.py --steps 10 --warmup 3
LTA_GEMM_SELECT_ROUNDS=1 run bench_r1b 600 python bench.py --steps 10 --warmup 3
run bench_r3b 600 python bench.py --steps 10 --warmup 3
run pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
