#!/bin/bash
# One-GPU rehearsal of the multi-GPU bench programs over RCCL (world size 1): FSDP with block
# bucketing (coalesced all-gathers + bucketed reduce-scatter), ZeRO-3-free default, DDP.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
export LTA_BENCH_FORCE_DIST=1
run rehearse_fsdp 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --steps 3 --warmup 2 --parallel fsdp
run rehearse_ddp 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 1 --steps 3 --warmup 2 --parallel ddp
