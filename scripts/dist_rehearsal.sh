#!/bin/bash
# 2 ranks sharing one GPU over gloo: exercises the DDP/FSDP compiled paths end-to-end (numbers not meaningful).
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PYTHONPATH LTA_BENCH_SAME_DEVICE=1 LTA_DIST_BACKEND=gloo
OUT=gpurun_out; mkdir -p $OUT
for P in fsdp ddp tp; do
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 2 --warmup 1 --n-layer 2 --seq 1024 --parallel $P > $OUT/rehearsal_$P.log 2>&1; echo "$P rc=$?"; tail -3 $OUT/rehearsal_$P.log
done
