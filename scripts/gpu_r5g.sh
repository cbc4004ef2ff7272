#!/bin/bash
# round 3: gemm4 PMC (fwd many-tile vs dgrad few-tile), FP8 delayed bench + step profile
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
rm -rf $OUT/pmc_g1 $OUT/pmc_g2 $OUT/prof_fp8
run pmc_g1 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $OUT/pmc_g1 -o run --output-format csv -- python scripts/gemm4_pmc.py
run pmc_g2 120 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VALU -d $OUT/pmc_g2 -o run --output-format csv -- python scripts/gemm4_pmc.py
run bench_fp8 600 python -u bench.py --steps 10 --warmup 3 --fp8 --fp8-recipe delayed
run prof_fp8 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_fp8 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --fp8 --fp8-recipe delayed
