#!/bin/bash
# round 3: gemm4 correctness + A/B on the Llama-2-7B training GEMMs
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run gemm4 600 python -u scripts/gemm4_bench.py --rounds 3 --iters 20
