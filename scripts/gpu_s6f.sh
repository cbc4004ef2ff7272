#!/bin/bash
# dK/dV v4 with the K stash in LDS (no scratch spills): attention tests + per-kernel times
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_attn 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "attention or attn or rope"
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_kst -o run -- python3 -u scripts/attn_dq_ds_ab.py
