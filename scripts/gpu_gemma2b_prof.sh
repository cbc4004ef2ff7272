#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
rm -rf $OUT/prof_g2b
run prof_g2b 420 rocprofv3 --kernel-trace --stats -d $OUT/prof_g2b -o run --output-format csv -- python bench.py --model Gemma-2b --steps 3 --warmup 2 --eager-baseline off
