#!/bin/bash
# MXFP4: operand-map probe, quantiser / GEMM / GEMV numerics, transform; fp8 cast regression; bench.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_mxfp4 300 python -u -m pytest tests/test_mxfp4.py -m gpu -x -v -s --timeout 120 --timeout-method thread
run pytest_fp8 300 python -u -m pytest tests/test_hip_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fp8 or mx or amax or cast"
run mxfp4_bench 300 python -u scripts/mxfp4_bench.py gpurun_out/mxfp4_bench.json
