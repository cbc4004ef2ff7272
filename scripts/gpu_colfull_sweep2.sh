#!/bin/bash
# column-mode kernels after the 4-word Philox draws: GPU tests, then the grid sweep on the GPT-2-medium step
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_hipfuse 400 python -u -m pytest tests/test_hipfuse.py -x -q -m gpu --timeout 120 --timeout-method thread
sweep() {
  local tag=$1
  shift
  rm -rf $OUT/prof_sw_$tag
  run sw_$tag 300 env "$@" rocprofv3 --kernel-trace -d $OUT/prof_sw_$tag -o run --output-format csv -- python scripts/hipfuse_roofline.py --json $OUT/roof_$tag.json
  run join_$tag 60 python scripts/roofline_from_trace.py $OUT/roof_$tag.json $OUT/prof_sw_$tag/run_kernel_trace.csv
}
sweep v4base LTA_HIPFUSE_COL_NW=8
sweep v4ms128u4 LTA_HIPFUSE_COL_MAX_SPLITS=128 LTA_HIPFUSE_COL_UNROLL=4
sweep v4ms128 LTA_HIPFUSE_COL_MAX_SPLITS=128
sweep v4u4 LTA_HIPFUSE_COL_UNROLL=4
