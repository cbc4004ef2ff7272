#!/bin/bash
# dQ-from-dS attention backward: numerics, kernel A/B, Llama-2-7B step A/B
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_ds 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "dq_from_ds or fused_rope"
run ab 200 python -u scripts/attn_dq_ds_ab.py
run bench_a 400 python -u bench.py --steps 10 --warmup 3 --eager-baseline off
grep -o '"ms_per_step": [0-9.]*' $OUT/bench_a.log | head -1
export LTA_ATTN_DQ_FROM_DS=1
run bench_ds 400 python -u bench.py --steps 10 --warmup 3 --eager-baseline off
grep -o '"ms_per_step": [0-9.]*' $OUT/bench_ds.log | head -1
