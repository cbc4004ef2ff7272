#!/bin/bash
# Final state check: smoke + default bench.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 480 python bench.py
