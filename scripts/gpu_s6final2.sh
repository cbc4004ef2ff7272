#!/bin/bash
# round 5 last tree: full GPU suite, smoke, default bench (eager baseline on)
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run suite 900 python -u -m pytest tests -q -m gpu --timeout 180 --timeout-method thread --ignore=tests/test_ops.py -p no:cacheprovider
run suite_ops 400 python -u -m pytest tests/test_ops.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 500 python -u bench.py
grep '"metric"' $OUT/bench.log | head -1
