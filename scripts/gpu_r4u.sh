#!/bin/bash
# round 4: op-level GPU tests (hipfuse-heavy) after the hardware bf16 rounding change, smoke
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run suite_ops 300 python -u -m pytest tests/test_ops.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
