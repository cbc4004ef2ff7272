#!/bin/bash
# TP program world-1 rehearsal after the vocab-parallel cross-entropy moved to the hand CE kernels,
# plus the same-box plain step; TP kernel trace breakdown
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
run tp_plain 400 python -u bench.py --model Llama-3-8B --n-layer 4 --seq 8192 --eager-baseline off
LTA_BENCH_FORCE_DIST=1 run tp_dist 500 python -u bench.py --model Llama-3-8B --n-layer 4 --seq 8192 --parallel tp --eager-baseline off
export LTA_BENCH_FORCE_DIST=1
rm -rf $OUT/prof_tp
run prof_tp 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_tp -o run --output-format csv -- python bench.py --model Llama-3-8B --n-layer 4 --seq 8192 --parallel tp --steps 2 --warmup 2 --eager-baseline off
python scripts/step_breakdown.py $(ls $OUT/prof_tp/*/run_kernel_trace.csv $OUT/prof_tp/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/tp_breakdown.txt 2>&1
rm -f $OUT/prof_tp/*/*kernel_trace.csv $OUT/prof_tp/run_kernel_trace.csv 2>/dev/null
exit 0
