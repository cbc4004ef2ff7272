#!/bin/bash
# Decode-attention split retune: kernel tests, decode micro-timing, inference bench (7B / 1B batch 1).
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_dec 300 python -u -m pytest tests/test_hip_kernels.py tests/test_generate.py -k "decode or generate or inference" -x -v --timeout 150 --timeout-method thread
run inf_7b_b1 300 python -m lightning_thunder_amd.benchmarks.inference --model Llama-2-7b-hf --batch-size 1 --input-length 2048 --output-length 128 --num-iterations 3 --warmup-iterations 1 --modes hipgraph
run inf_1b 300 python -m lightning_thunder_amd.benchmarks.inference --model Llama-3.2-1B --batch-size 1 --input-length 2048 --output-length 128 --num-iterations 3 --warmup-iterations 1 --modes hipgraph
run inf_1b_b8 300 python -m lightning_thunder_amd.benchmarks.inference --model Llama-3.2-1B --batch-size 8 --input-length 2048 --output-length 128 --num-iterations 3 --warmup-iterations 1 --modes hipgraph
run gen 300 python -m lightning_thunder_amd.benchmarks.generate --modes hipgraph
