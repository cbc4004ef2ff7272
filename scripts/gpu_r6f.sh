#!/bin/bash
# round 3: smoke + full GPU test suite on the current defaults
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
run gputests 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
