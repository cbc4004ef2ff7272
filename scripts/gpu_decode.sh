#!/bin/bash
# Decode-path kernels: GEMV / decode-attention tests, generation benchmark and its kernel profile.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run dec_tests 300 python -u -m pytest tests/test_hip_kernels.py -x -q -k "gemv or decode" --timeout 120 --timeout-method thread
run gen_tests 300 python -u -m pytest tests/test_generate.py -x -q -m gpu --timeout 120 --timeout-method thread
run gen_bench 300 python -u -m lightning_thunder_amd.benchmarks.generate --iters 3
run prof_gen 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_gen -o run --output-format csv -- python -m lightning_thunder_amd.benchmarks.generate --modes hipgraph --iters 1 --warmup 0
