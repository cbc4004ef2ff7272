#!/bin/bash
# standalone column sums (x.float().sum(0) -> bf16) under the kernel trace, for several column-mode grids
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
sweep() {
  local tag=$1
  shift
  rm -rf $OUT/prof_cr_$tag
  run cr_$tag 300 env "$@" rocprofv3 --kernel-trace -d $OUT/prof_cr_$tag -o run --output-format csv -- python scripts/colred_bench.py --json $OUT/cr_$tag.json
  run crj_$tag 60 python scripts/colred_join.py $OUT/cr_$tag.json $OUT/prof_cr_$tag/run_kernel_trace.csv
}
sweep def LTA_HIPFUSE_COL_NW=8
sweep w384 LTA_HIPFUSE_COL_WGS=384
sweep w512nw4 LTA_HIPFUSE_COL_WGS=512 LTA_HIPFUSE_COL_NW=4
sweep w256u8 LTA_HIPFUSE_COL_WGS=256 LTA_HIPFUSE_COL_UNROLL=8
