#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
rm -rf $OUT/prof_l3 $OUT/prof_phi3
run prof_l3 420 rocprofv3 --kernel-trace --stats -d $OUT/prof_l3 -o run --output-format csv -- python bench.py --model Llama-3-8B --steps 3 --warmup 2 --eager-baseline off
run prof_phi3 420 rocprofv3 --kernel-trace --stats -d $OUT/prof_phi3 -o run --output-format csv -- python bench.py --model Phi-3-mini-4k-instruct --steps 3 --warmup 2 --eager-baseline off
