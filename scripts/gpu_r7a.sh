#!/bin/bash
# Round-3 re-entry check: full GPU suite, smoke, bf16 + FP8 delayed bench of the current tree.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread
run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench_bf16 400 python -u bench.py --steps 10 --warmup 3
run bench_fp8d 400 python -u bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe delayed
