#!/bin/bash
# dK/dV v2 kernel: numerics, A/B timing vs v1, headline step, PMC counters.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_attn 300 python -u -m pytest tests/test_hip_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "flash_attention or rmsnorm"
run attn_ab 300 python -u scripts/attn_bwd_ab.py
run bench_bf16 300 python -u bench.py --steps 10 --warmup 3
rm -rf $OUT/pmc_attn1
run pmc_attn1 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $OUT/pmc_attn1 -o run --output-format csv -- python scripts/attn_only.py 2
