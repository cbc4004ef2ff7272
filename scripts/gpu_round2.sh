#!/bin/bash
# Full GPU tests, then the generation benchmark and its kernel profile.
source "$(dirname "$0")/gpu_steps.sh"
export TMPDIR=/tmp
rm -f $OUT/status.log
run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
run gen_bench 600 python -u -m lightning_thunder_amd.benchmarks.generate --iters 3
run prof_gen 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_gen -o run --output-format csv -- python -m lightning_thunder_amd.benchmarks.generate --modes hipgraph --iters 1 --warmup 0
