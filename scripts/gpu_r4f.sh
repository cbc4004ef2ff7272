#!/bin/bash
# round 4: dK/dV v4 (VALU pipelined into the MFMA shadows) vs v3
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run bwd_v4 300 python -u scripts/attn_bwd_v4_check.py
