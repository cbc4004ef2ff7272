#!/bin/bash
# Full GPU suite after the interpreter / autodiff changes; bf16 + FP8 recipe benches.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run bench 600 python bench.py --steps 10 --warmup 3
run bench_fp8 600 python bench.py --steps 10 --warmup 3 --fp8
run bench_fp8_delayed 600 python bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe delayed
run bench_mxfp8 600 python bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe mxfp8
