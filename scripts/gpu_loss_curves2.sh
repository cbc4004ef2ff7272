#!/bin/bash
# 7B loss curves, thunder vs eager, under learning-rate settings that do not oscillate.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run lc_w10 300 python bench.py --steps 20 --warmup 5 --lr-warmup 10
run lc_lr1e4 300 python bench.py --steps 20 --warmup 5 --lr 1e-4
