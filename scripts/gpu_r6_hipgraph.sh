#!/bin/bash
# hipGraph step (donated gradients) test + bench + CU-contention step curve.
source "$(dirname "$0")/gpu_steps.sh"
export TMPDIR=/tmp
rm -f $OUT/status.log
run t_hipgraph 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_7b_shape.py -m gpu -k hipgraph
run bench_hipgraph2 420 python bench.py --hipgraph --steps 10 --warmup 3 --eager-baseline off
run bench_plain 420 python bench.py --steps 10 --warmup 3 --eager-baseline off
run cu_cont_rccl 400 python scripts/cu_contention.py --threads 256 --lds 37664 --n 0,8,32 --step
