#!/bin/bash
# dQ-from-dS tiling sweep: numerics per config + per-kernel times
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
for c in 0 3 4; do
  export LTA_ATTN_DQDS_CFG=$c
  run t_ds$c 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "dq_from_ds"
  run prof$c 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_ds$c -o run -- python3 -u scripts/attn_dq_ds_ab.py
done
