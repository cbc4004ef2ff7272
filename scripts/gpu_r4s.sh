#!/bin/bash
# round 4: attention backward per-kernel time vs data magnitudes
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
for V in base dosmall qksmall both; do
  rm -rf $OUT/prof_mag_$V
  export LTA_VARIANT=$V
  run mag_$V 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_mag_$V -o run --output-format csv -- python scripts/attn_bwd_magnitude.py
  python scripts/prof_summary.py $(ls $OUT/prof_mag_$V/*/run_kernel_stats.csv $OUT/prof_mag_$V/run_kernel_stats.csv 2>/dev/null | head -1) 6 > $OUT/mag_$V.txt 2>&1
done
