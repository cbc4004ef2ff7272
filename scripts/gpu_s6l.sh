#!/bin/bash
# dQ-from-dS kernel after the template simplification: tests + kernel times
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_ds 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "dq_from_ds or fused_rope or flash_attention"
run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_l -o run -- python3 -u scripts/attn_dq_ds_ab.py
