#!/bin/bash
# D = 256 forward ring kernel: fwd/bwd numerics vs fp32 (all head dims), A/B vs the generic kernel
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_fa 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "flash_attention_fwd_bwd"
run d256 300 python -u scripts/attn_d256_bench.py
