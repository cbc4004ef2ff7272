#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run ablate 300 python -u scripts/attn_v4_ablate.py
rm -rf $OUT/pmc4a $OUT/pmc4b
run pmc4a 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $OUT/pmc4a -o run --output-format csv -- python scripts/attn_fwd_only.py 10 3
run pmc4b 120 timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/pmc4b -o run --output-format csv -- python scripts/attn_fwd_only.py 10 3
run pmc4c 120 timeout -s KILL 100 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_IFETCH -d $OUT/pmc4c -o run --output-format csv -- python scripts/attn_fwd_only.py 10 3
