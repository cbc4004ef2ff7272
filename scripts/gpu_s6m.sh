#!/bin/bash
# PMC passes (one counter group per run): attention backward (dK/dV v4 + dS, dQ from dS, dQ v4) and the
# D = 256 forward ring kernel
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
rm -rf $OUT/pmc_b1 $OUT/pmc_b2 $OUT/pmc_f1 $OUT/pmc_f2
run pmc_b1 120 timeout -s KILL 110 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU -d $OUT/pmc_b1 -o run --output-format csv -- python3 scripts/attn_dq_ds_ab.py
run pmc_b2 120 timeout -s KILL 110 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_b2 -o run --output-format csv -- python3 scripts/attn_dq_ds_ab.py
run pmc_f1 120 timeout -s KILL 110 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU -d $OUT/pmc_f1 -o run --output-format csv -- python3 scripts/attn_fwd_ring_ab.py
run pmc_f2 120 timeout -s KILL 110 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_f2 -o run --output-format csv -- python3 scripts/attn_fwd_ring_ab.py
python3 scripts/pmc_summary.py $OUT/attn_r5_pmc.json $OUT/pmc_b1 $OUT/pmc_b2 $OUT/pmc_f1 $OUT/pmc_f2 > $OUT/pmc_summary.log 2>&1
find $OUT/pmc_b1 $OUT/pmc_b2 $OUT/pmc_f1 $OUT/pmc_f2 -name "*.csv" -size +20M -delete
exit 0
