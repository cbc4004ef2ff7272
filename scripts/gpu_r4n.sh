#!/bin/bash
# round 4: generated-kernel roofline after the column-reduction unroll; evidence refresh: speedup vs
# eager, FP8 delayed step; warm vs cold attention backward
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run roofline 300 python -u scripts/hipfuse_roofline.py
run attn_cold 200 python -u scripts/attn_bwd_cold.py
run bench_eager 700 python -u bench.py --steps 10 --warmup 3 --eager-baseline
run bench_fp8 500 python -u bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe delayed
