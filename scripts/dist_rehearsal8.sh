#!/bin/bash
# World-8 rehearsal: 8 ranks sharing ONE GPU over gloo (never RCCL: one device), exercising the
# world-8 shard shapes of the bench programs end to end: FSDP padding and bucketed collectives at 8
# ranks (Llama-2-7B, 2 layers), DDP buckets, and TP=8 on Llama-3-8B (vocab 128256 / 8 = 16032-column
# LM-head shard on the hand GEMM's edge tiles).  Throughput numbers are NOT meaningful (8 processes
# on one card, gloo); the record is that every program runs and what it dispatches.
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PYTHONPATH LTA_BENCH_SAME_DEVICE=1 LTA_DIST_BACKEND=gloo
OUT=gpurun_out; mkdir -p $OUT
run8() {
  local name=$1; shift
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29519 bench.py --gpus 8 --steps 1 --warmup 1 --n-layer 2 --seq 1024 "$@" > $OUT/rehearsal8_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"; grep -E '^\{|\[gemm\]|first step' $OUT/rehearsal8_$name.log | tail -3
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run8 fsdp --parallel fsdp
run8 ddp --parallel ddp
run8 tp --parallel tp --model Llama-3-8B
