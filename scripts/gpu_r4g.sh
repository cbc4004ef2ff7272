#!/bin/bash
# round 4: dK/dV v4 (interleaved phases, early transposed reads) vs v3, dQ fragment prefetch; whole step
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run bwd_v4 300 python -u scripts/attn_bwd_v4_check.py
run t_attn 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py tests/test_attention_ex.py -k "attention or attn or sdpa" -m gpu
run bench 600 python -u bench.py --steps 10 --warmup 3
