#!/bin/bash
# Full GPU suite + smoke + bf16 / FP8 bench of the current tree; generation benchmark (prefill paths).
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_gpu 700 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread
run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench_bf16 300 python -u bench.py --steps 10 --warmup 3
run gen_bench 300 python -u -m lightning_thunder_amd.benchmarks.generate --iters 3
