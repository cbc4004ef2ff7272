#!/bin/bash
# One-GPU bench.py records for more models of the reference's multi-model chart (BASELINE.md:26)
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
for m in Llama-3-8B Mistral-7B-v0.2 Nous-Hermes-13b Gemma-2b; do
  run "mb_$m" 420 python bench.py --model $m --steps 10 --warmup 3
done
