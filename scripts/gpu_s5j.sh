#!/bin/bash
# Round 5, session j: per-kernel PMC of the attention v4 kernels; dK/dV v4 phase stamps (diagnostic build);
# vocab-parallel CE and TP shard-shape GEMM tests.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run tests_new 600 python -u -m pytest tests/test_distributed_gpu.py tests/test_gpu_7b_shape.py -x -q --timeout 300 --timeout-method thread -k "vocab or tensor_parallel"
LTA_KERNELS_SO=scripts/exp/lta_diag.so run bwd_stamps 300 python -u scripts/attn_bwd_stamps.py
rm -rf $OUT/pmc_a1 $OUT/pmc_a2 $OUT/pmc_a3
run pmc_a1 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d $OUT/pmc_a1 -o run --output-format csv -- python scripts/attn_only.py 2
run pmc_a2 120 timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/pmc_a2 -o run --output-format csv -- python scripts/attn_only.py 2
run pmc_a3 120 timeout -s KILL 100 rocprofv3 --pmc SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC -d $OUT/pmc_a3 -o run --output-format csv -- python scripts/attn_only.py 2
python scripts/pmc_summary.py $OUT/attn_v4_pmc.json $OUT/pmc_a1 $OUT/pmc_a2 $OUT/pmc_a3 > $OUT/attn_v4_pmc.txt 2>&1
rm -rf $OUT/pmc_a1 $OUT/pmc_a2 $OUT/pmc_a3
exit 0
