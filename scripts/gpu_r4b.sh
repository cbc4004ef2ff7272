#!/bin/bash
# MXFP4 training recipe + hook/MoE changes: targeted GPU tests, then fp8 benches.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_fp 300 python -u -m pytest tests/test_hip_kernels.py -k "mxfp4 or mxfp8 or fp8" -x -v --timeout 120 --timeout-method thread
run bench_mxfp4 480 python bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe mxfp4
run bench_mxfp8 480 python bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe mxfp8
