#!/bin/bash
# FP8 kernels: tests, then the three FP8 recipes on the headline step.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_fp8 240 python -u -m pytest tests/test_hip_kernels.py -m gpu -q --timeout 120 --timeout-method thread -k "fp8 or mx or mfma"
run bench_fp8_current 300 python -u bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe current
run bench_fp8_delayed 300 python -u bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe delayed
run bench_fp8_mxfp8 300 python -u bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe mxfp8
