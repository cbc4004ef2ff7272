#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run bench_ckpt 600 python bench.py --steps 5 --warmup 2 --checkpoint-activations
run bench_ckpt_seq16k 600 python bench.py --steps 3 --warmup 2 --checkpoint-activations --seq 16384
