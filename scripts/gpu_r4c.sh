#!/bin/bash
# Full GPU suite + smoke after the hook-interpretation / MoE / MXFP4-recipe changes.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_moe 200 python -u -m pytest tests/test_llama4_moe.py -x -v --timeout 120 --timeout-method thread
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
