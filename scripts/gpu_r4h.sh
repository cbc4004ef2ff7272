#!/bin/bash
# round 4: full GPU suite on the current tree (ops consistency split out), smoke, GPT-2 profile + roofline
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run suite 1000 python -u -m pytest tests -q -m gpu --timeout 180 --timeout-method thread --ignore=tests/test_ops.py -p no:cacheprovider
run suite_ops 400 python -u -m pytest tests/test_ops.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run adamw_nt 180 python -u scripts/adamw_nt_ab.py
