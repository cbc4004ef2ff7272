#!/bin/bash
# round 4: optimizer-in-backward (side-stream lean AdamW) A/B on the headline bench, Philox block
# draws, hipfuse GPU tests, generated-kernel roofline
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_ov 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_optim_overlap.py tests/test_hipfuse.py -m gpu
run bench_ov 600 python -u bench.py --steps 10 --warmup 3
run bench_noov 600 python -u bench.py --steps 10 --warmup 3 --optim-overlap off
run prof_ov 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_ov -o run --output-format csv -- python bench.py --steps 3 --warmup 2
run roofline 400 python -u scripts/hipfuse_roofline.py
