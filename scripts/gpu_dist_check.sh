#!/bin/bash
# distributed paths after the round-6 changes: 2 gloo ranks on one GPU (fsdp / ddp / tp), world-1 RCCL fsdp
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run rehearsal2 900 bash scripts/dist_rehearsal.sh
export LTA_BENCH_FORCE_DIST=1; run rccl_fsdp1 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 3 --warmup 2 --parallel fsdp --eager-baseline off
