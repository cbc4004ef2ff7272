#!/bin/bash
# round 4: attention backward defaults (dQ v4 + fused delta, dK/dV v4 reversed q sweep, fused RoPE backward):
# GPU numerics, then whole-step A/B of the dK/dV query order
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run attn_tests 400 python -u -m pytest tests/test_hip_kernels.py tests/test_attention_ex.py tests/test_generate.py tests/test_gpu_7b_shape.py -q -m gpu -k "flash or attention or rope or sdpa or generate or decode or 7b_shape" --timeout 180 --timeout-method thread -p no:cacheprovider
run bench_new 400 python -u bench.py --steps 10 --warmup 3
export LTA_DKDV_QREV=0
run bench_qfwd 400 python -u bench.py --steps 10 --warmup 3
