#!/bin/bash
# round 3: forward v3 (64 rows per wave) A/B against v1 and v2-att[2]
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run attn_ab3 300 python -u scripts/attn_fwd_ab.py 0,4,7,8 fwd
