#!/bin/bash
# end-of-round validation: the whole GPU suite (as the driver runs it), smoke(), the default bench
source "$(dirname "$0")/gpu_steps.sh"
export TMPDIR=/tmp
rm -f $OUT/status.log
run pytest_gpu 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python bench.py
