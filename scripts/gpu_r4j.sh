#!/bin/bash
# round 4: D=256 attention numerics + timing, then the full GPU suite
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run d256_tests 300 python -u -m pytest tests/test_hip_kernels.py tests/test_attention_ex.py -q -m gpu -k "256 or 192" --timeout 120 --timeout-method thread -p no:cacheprovider
run d256_bench 200 python -u scripts/attn_d256_bench.py
run dq_v3 300 python -u scripts/attn_dq_v3_check.py
run suite 1000 python -u -m pytest tests -q -m gpu --timeout 180 --timeout-method thread --ignore=tests/test_ops.py -p no:cacheprovider
run suite_ops 400 python -u -m pytest tests/test_ops.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run adamw_nt 180 python -u scripts/adamw_nt_ab.py
