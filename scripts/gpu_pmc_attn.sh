#!/bin/bash
# PMC counters of the attention backward kernels (dK/dV and dQ) at the Llama-2-7B shape.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run counters_list 60 rocprofv3 -L
rm -rf $OUT/pmc_attn1 $OUT/pmc_attn2
run pmc_attn1 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $OUT/pmc_attn1 -o run --output-format csv -- python scripts/attn_only.py 2
run pmc_attn2 120 timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_UNALIGNED_STALL SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/pmc_attn2 -o run --output-format csv -- python scripts/attn_only.py 2
