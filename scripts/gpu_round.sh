#!/bin/bash
# GPU session: gpu tests, smoke, 1-GPU bench. Every step time-limited; a crash ends the session.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_gpu 420 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 480 python bench.py --steps ${STEPS:-8} --warmup 3
