#!/bin/bash
# dropout key / query term tables: dropout + attention tests, D=64 dropout A/B against the previous build
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_drop 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_ex.py tests/test_hip_kernels.py -k "dropout or flash_attention or mask"
for i in 1 2; do
  LTA_KERNELS_SO=scripts/exp/lta_prev.so run ab_prev$i 120 python -u scripts/attn_dropout_ab.py
  run ab_new$i 120 python -u scripts/attn_dropout_ab.py
done
grep -h "dropout attention" $OUT/ab_prev*.log $OUT/ab_new*.log
