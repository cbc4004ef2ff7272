#!/bin/bash
# rocprofv3 kernel stats of the headline training step (Llama-2-7B, seq 4096, 1 GPU)
source "$(dirname "$0")/gpu_steps.sh"
export TMPDIR=/tmp
rm -rf $OUT/prof_bench
run prof_bench 900 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- python bench.py --steps 3 --warmup 2
