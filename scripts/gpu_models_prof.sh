#!/bin/bash
# Kernel breakdowns of the chart models that trail (Mistral-7B, Gemma-7b).
source "$(dirname "$0")/gpu_steps.sh"
export TMPDIR=/tmp
rm -f $OUT/status.log
for m in Mistral-7B-v0.1 Gemma-7b; do
  rm -rf $OUT/prof_$m
  run prof_$m 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_$m -o run --output-format csv -- python bench.py --model $m --steps 3 --warmup 2 --eager-baseline off
done
