#!/bin/bash
# Round 5, session d: swapped-operand register epilogue (anatomy ABL 64) vs the LDS-image epilogue.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run anatomy3 300 python -u scripts/exp/gemm_anatomy.py 0,64,8
exit 0
