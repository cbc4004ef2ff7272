#!/bin/bash
# column-reduction variants: direct-launch timings + rocprof kernel durations
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run colred 300 python -u scripts/colred_bench.py --json $OUT/colred_bench.json
grep -v amdgpu.ids $OUT/colred.log
rm -rf $OUT/prof_colred
run prof_colred 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_colred -o run --output-format csv -- python scripts/colred_bench.py --json $OUT/colred_bench_prof.json
cat $(ls $OUT/prof_colred/*/run_kernel_stats.csv $OUT/prof_colred/run_kernel_stats.csv 2>/dev/null | head -1) | cut -d, -f1-8 | head -60
