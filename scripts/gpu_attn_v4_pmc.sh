#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
timeout -k 5 60 rocprofv3 --list-avail > $OUT/counters_avail.txt 2>&1 || true
grep -iE "ICACHE|SQC_|INST_LEVEL|WAIT_BARRIER|BARRIER|LEVEL_WAVES|IFETCH" $OUT/counters_avail.txt | head -60 > $OUT/counters_grep.txt || true
for impl in 10 11 14; do
  rm -rf $OUT/pa$impl
  run pa$impl 90 timeout -s KILL 80 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU -d $OUT/pa$impl -o run --output-format csv -- python scripts/attn_fwd_only.py $impl 3 0
done
