#!/bin/bash
# The whole GPU test suite (as the driver runs it at round end), then smoke() and the default bench,
# then the Gemma-7b profile.
source "$(dirname "$0")/gpu_steps.sh"
export TMPDIR=/tmp
rm -f $OUT/status.log
run pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python bench.py
rm -rf $OUT/prof_Gemma
run prof_Gemma 420 rocprofv3 --kernel-trace --stats -d $OUT/prof_Gemma -o run --output-format csv -- python bench.py --model Gemma-7b --steps 3 --warmup 2 --eager-baseline off
