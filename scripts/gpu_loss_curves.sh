#!/bin/bash
# 7B loss-curve diagnosis: thunder vs eager from the same init and data, then thunder with one
# component swapped at a time (torch AdamW; attention dQ recompute instead of dQ-from-dS).
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run lc_default 300 python bench.py --steps 20 --warmup 5
run lc_torch_adamw 240 env LTA_TORCH_ADAMW=1 python bench.py --steps 20 --warmup 5 --eager-baseline off
run lc_no_dqds 240 env LTA_ATTN_DQ_FROM_DS=0 python bench.py --steps 20 --warmup 5 --eager-baseline off
