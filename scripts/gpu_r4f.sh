#!/bin/bash
# Kernel stats of Llama-2-7B batch-1 decode at a 2k-token context (jit + hipGraph).
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
rm -rf $OUT/prof_dec
run prof_dec 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_dec -o run --output-format csv -- python -m lightning_thunder_amd.benchmarks.inference --model Llama-2-7b-hf --batch-size 1 --input-length 2048 --output-length 64 --num-iterations 2 --warmup-iterations 0 --modes hipgraph
run sum 60 python scripts/prof_summary.py $OUT/prof_dec/run_kernel_stats.csv 25
rm -f $OUT/prof_dec/run_kernel_trace.csv
