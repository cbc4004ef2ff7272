#!/bin/bash
# round 4: full GPU suite on the final tree, smoke, bench, attention backward clock experiment
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run suite 900 python -u -m pytest tests -q -m gpu --timeout 180 --timeout-method thread --ignore=tests/test_ops.py -p no:cacheprovider
run suite_ops 300 python -u -m pytest tests/test_ops.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run attn_cold 200 python -u scripts/attn_bwd_cold.py
