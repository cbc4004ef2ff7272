#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run gen_mx7b 600 python -u -m lightning_thunder_amd.benchmarks.generate --model Llama-2-7b-hf --modes hipgraph,hipgraph_mxfp4 --iters 2
