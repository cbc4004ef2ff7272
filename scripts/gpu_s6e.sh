#!/bin/bash
# dQ-from-dS default-on: attention tests, 7B-shape test, interleaved step A/B vs the recompute path
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_attn 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py tests/test_gpu_7b_shape.py -k "attention or attn or rope or 7b"
for r in 1 2; do
  export LTA_ATTN_DQ_FROM_DS=0
  run bench_rc$r 400 python -u bench.py --steps 10 --warmup 3 --eager-baseline off
  grep -o '"ms_per_step": [0-9.]*' $OUT/bench_rc$r.log | head -1
  unset LTA_ATTN_DQ_FROM_DS
  run bench_ds$r 400 python -u bench.py --steps 10 --warmup 3 --eager-baseline off
  grep -o '"ms_per_step": [0-9.]*' $OUT/bench_ds$r.log | head -1
done
