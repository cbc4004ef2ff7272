#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_mxfp4 300 python -u -m pytest tests/test_mxfp4.py -m gpu -x -q --timeout 120 --timeout-method thread -k gemv
run mxfp4_bench 300 python -u scripts/mxfp4_bench.py gpurun_out/mxfp4_bench.json
