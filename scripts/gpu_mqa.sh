#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_attn 500 python -u -m pytest tests/test_hip_kernels.py -x -q -k "attention or flash or attn" --timeout 200 --timeout-method thread
run mb_g2b 420 python bench.py --model Gemma-2b --steps 10 --warmup 3
run mb_mistral 420 python bench.py --model Mistral-7B-v0.2 --steps 10 --warmup 3 --eager-baseline off
