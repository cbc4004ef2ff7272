#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_hg 300 python -u -m pytest tests/test_hipgraph.py -m gpu -x -q --timeout 280 --timeout-method thread
