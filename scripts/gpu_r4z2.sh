#!/bin/bash
# round 4: same-box A/B of the new defaults (GEMM tail split, non-temporal AdamW)
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run bench_default 300 python -u bench.py --steps 10 --warmup 3
LTA_GEMM_TAIL_SPLIT=0 run bench_nosplit 300 python -u bench.py --steps 10 --warmup 3
LTA_ADAMW_NT=0 run bench_nont 300 python -u bench.py --steps 10 --warmup 3
run bench_default2 300 python -u bench.py --steps 10 --warmup 3
