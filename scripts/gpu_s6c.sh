#!/bin/bash
# dQ-from-dS numerics + per-kernel times of the two attention backward variants (rocprofv3 kernel trace)
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_ds 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "dq_from_ds"
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_ds -o run -- python3 -u scripts/attn_dq_ds_ab.py
