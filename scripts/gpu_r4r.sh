#!/bin/bash
# round 4: final checks on the current tree: optimizer overlap (plain AdamW default), attention backward
# timing variants, bench
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run ov 200 python -u -m pytest tests/test_optim_overlap.py tests/test_hip_kernels.py -q -m gpu -k "adamw or overlap" --timeout 120 --timeout-method thread -p no:cacheprovider
run attn_cold 240 python -u scripts/attn_bwd_cold.py
run bench_final 400 python -u bench.py
