#!/bin/bash
# GPU test suite + smoke on one MI355X (no bench).
source scripts/gpu_steps.sh
rm -f $OUT/status.log
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
