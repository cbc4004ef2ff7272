#!/bin/bash
# round 4: gemm4 bias + GELU epilogue: pre-tail-split source vs current
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run g4_ab 200 python -u scripts/g4old/ab.py
