#!/bin/bash
# Round 5, session c: gemm4 epilogue anatomy (prologue / main loop / epilogue stamps); D = 192 / 256
# attention with masks and dropout.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run anatomy2 300 python -u scripts/exp/gemm_anatomy.py
run attn_ex 600 python -u -m pytest tests/test_attention_ex.py -x -q --timeout 120 --timeout-method thread
exit 0
