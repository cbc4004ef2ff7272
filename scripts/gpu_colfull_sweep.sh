#!/bin/bash
# column-mode grid sweep on the GPT-2-medium step's generated kernels (device durations from the trace)
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
sweep() {
  local tag=$1
  shift
  rm -rf $OUT/prof_sw_$tag
  run sw_$tag 300 env "$@" rocprofv3 --kernel-trace -d $OUT/prof_sw_$tag -o run --output-format csv -- python scripts/hipfuse_roofline.py --json $OUT/roof_$tag.json
  run join_$tag 60 python scripts/roofline_from_trace.py $OUT/roof_$tag.json $OUT/prof_sw_$tag/run_kernel_trace.csv
}
sweep base LTA_HIPFUSE_COL_NW=8
sweep nw16 LTA_HIPFUSE_COL_NW=16
sweep ms128 LTA_HIPFUSE_COL_MAX_SPLITS=128
sweep ms256 LTA_HIPFUSE_COL_MAX_SPLITS=256
sweep nw16ms128 LTA_HIPFUSE_COL_NW=16 LTA_HIPFUSE_COL_MAX_SPLITS=128
sweep ms128u4 LTA_HIPFUSE_COL_MAX_SPLITS=128 LTA_HIPFUSE_COL_UNROLL=4
