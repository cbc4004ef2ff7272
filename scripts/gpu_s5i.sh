#!/bin/bash
# Round 5, session i: PMC study of the attention v4 kernels (fwd v4, dK/dV v4, dQ v4) at the Llama-2-7B
# shape, each counter pass its own short run; full GPU suite.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
rm -rf $OUT/pmc_a1 $OUT/pmc_a2 $OUT/pmc_a3
run pmc_a1 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d $OUT/pmc_a1 -o run --output-format csv -- python scripts/attn_only.py 2
run pmc_a2 120 timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/pmc_a2 -o run --output-format csv -- python scripts/attn_only.py 2
run pmc_a3 120 timeout -s KILL 100 rocprofv3 --pmc SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC -d $OUT/pmc_a3 -o run --output-format csv -- python scripts/attn_only.py 2
python scripts/pmc_summary.py $OUT/attn_v4_pmc.json $OUT/pmc_a1 $OUT/pmc_a2 $OUT/pmc_a3 > $OUT/attn_v4_pmc.txt 2>&1
rm -rf $OUT/pmc_a1 $OUT/pmc_a2 $OUT/pmc_a3
run gpu_suite 1100 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
exit 0
