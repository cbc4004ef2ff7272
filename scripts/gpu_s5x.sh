#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run hipgraph 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hipgraph.py tests/test_hipfuse.py -m gpu
