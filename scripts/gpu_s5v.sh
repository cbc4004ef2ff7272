#!/bin/bash
# hipfuse column-mode grid size for regions that also write full-domain outputs (GPT-2 fused bias grads)
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
for w in 192 768 1536; do
  export LTA_HIPFUSE_COL_WGS=$w
  run roof_$w 300 python -u scripts/hipfuse_roofline.py --json $OUT/roof_$w.json
  grep "col(" $OUT/roof_$w.log
done
