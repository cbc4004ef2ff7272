#!/bin/bash
# column-reduction variants (unroll / waves / grid) under rocprof
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
rm -rf $OUT/prof_colred2
run prof_colred2 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_colred2 -o run --output-format csv -- python scripts/colred_bench.py --json $OUT/colred_bench2.json
grep -v amdgpu.ids $OUT/prof_colred2.log | grep shape
