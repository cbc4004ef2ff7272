#!/bin/bash
# round 3: fixed attention fwd v2 A/B (+ bwd), attention GPU tests on the new bwd defaults, 1-GPU bench,
# world-1 RCCL FSDP rehearsal with a high-priority collective stream (queue assignment + overlap)
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
rm -rf $OUT/prof_fsdp2
run attn_ab2 300 python -u scripts/attn_fwd_ab.py 0,1,2,3,4,5,6
run attn_tests 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py tests/test_attention_ex.py -k "flash or attention or masked or dropout or sdpa"
run bench1 600 python -u bench.py --steps 10 --warmup 3
export LTA_BENCH_FORCE_DIST=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29562 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
run prof_fsdp2 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_fsdp2 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --parallel fsdp
