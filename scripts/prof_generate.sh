#!/bin/bash
# rocprofv3 kernel stats of the hipGraph decode path (Llama-3.2-1B, 100 new tokens)
source "$(dirname "$0")/gpu_steps.sh"
export TMPDIR=/tmp
run prof_gen 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_gen -o run --output-format csv -- python -m lightning_thunder_amd.benchmarks.generate --modes hipgraph --iters 1 --warmup 0
