#!/bin/bash
# world-1 RCCL rehearsal of the data-parallel bench programs on the final tree (the N > 1 code path)
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
run plain_mbs2 400 python -u bench.py --mbs 2 --eager-baseline off --steps 6 --warmup 2
LTA_BENCH_FORCE_DIST=1 run fsdp_mbs2 500 python -u bench.py --mbs 2 --parallel fsdp --eager-baseline off --steps 6 --warmup 2
LTA_BENCH_FORCE_DIST=1 run ddp_mbs2 500 python -u bench.py --mbs 2 --parallel ddp --eager-baseline off --steps 6 --warmup 2
grep -h '"metric"' $OUT/plain_mbs2.log $OUT/fsdp_mbs2.log $OUT/ddp_mbs2.log
