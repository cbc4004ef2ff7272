#!/bin/bash
# Inference benchmark: test + Llama-3.2-1B prefill/decode numbers (batch 1 and 8) + Llama-2-7B batch 1.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_inf 200 python -u -m pytest tests/test_generate.py -k inference -x -v --timeout 150 --timeout-method thread
run inf_1b_b1 300 python -m lightning_thunder_amd.benchmarks.inference --model Llama-3.2-1B --batch-size 1 --input-length 2048 --output-length 128 --num-iterations 3 --warmup-iterations 1
run inf_1b_b8 300 python -m lightning_thunder_amd.benchmarks.inference --model Llama-3.2-1B --batch-size 8 --input-length 2048 --output-length 128 --num-iterations 3 --warmup-iterations 1 --modes eager,hipgraph
run inf_7b_b1 300 python -m lightning_thunder_amd.benchmarks.inference --model Llama-2-7b-hf --batch-size 1 --input-length 2048 --output-length 128 --num-iterations 3 --warmup-iterations 1 --modes eager,hipgraph
run bench_lora 400 python bench.py --steps 8 --warmup 3 --lora 16
