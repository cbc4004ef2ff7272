#!/bin/bash
# D = 64 ring forward kernel: attention numerics (all head dims) + A/B vs generic; GPT-2 step
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_fa 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "flash_attention or attention_fwd or sdpa"
run ab 300 python -u scripts/attn_fwd_ring_ab.py
grep -v amdgpu.ids $OUT/ab.log
