#!/bin/bash
# round 3: attention forward v2 A/B, then GPT-2-medium hipfuse profile and world-1 RCCL FSDP rehearsal
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
rm -rf $OUT/prof_gpt2 $OUT/prof_fsdp1
run attn_ab 300 python -u scripts/attn_fwd_ab.py
run gpt2 300 python -u scripts/gpt2_step_profile.py
run prof_gpt2 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_gpt2 -o run --output-format csv -- python scripts/gpt2_step_profile.py
export LTA_BENCH_FORCE_DIST=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
run fsdp1 600 python -u bench.py --steps 6 --warmup 2 --parallel fsdp
run prof_fsdp1 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_fsdp1 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --parallel fsdp
