#!/bin/bash
# One-GPU bench.py records for the other models of the reference's multi-model chart (BASELINE.md:26),
# thunder vs eager on the same config (seq 4096, MBS 1, bf16, AdamW).
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
for m in ${MODELS:-Gemma-7b Mistral-7B-v0.1 Llama-2-13b-hf Phi-3-mini-4k-instruct Llama-3-8B Mistral-7B-v0.2 Nous-Hermes-13b}; do
  run "mb_$m" 420 python bench.py --model $m --steps 10 --warmup 3
done
