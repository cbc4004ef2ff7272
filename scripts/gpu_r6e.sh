#!/bin/bash
# round 3: forward v3 (64 rows per wave) A/B against v1 / v2-att[2]; PMC counters of v1 and v3
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run attn_ab3 300 python -u scripts/attn_fwd_ab.py 0,4,7,8 fwd
for impl in 0 8; do
  rm -rf $OUT/pmc_fwd_a$impl $OUT/pmc_fwd_b$impl
  run pmc_fwd_a$impl 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $OUT/pmc_fwd_a$impl -o run --output-format csv -- python scripts/attn_fwd_only.py $impl 3
  run pmc_fwd_b$impl 120 timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/pmc_fwd_b$impl -o run --output-format csv -- python scripts/attn_fwd_only.py $impl 3
done
