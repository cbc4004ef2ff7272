#!/bin/bash
# Round-6 perf records: hipGraph-captured 7B step, fresh FP8 (delayed) step + kernel breakdown,
# the bf16 step kernel breakdown on this tree.
source "$(dirname "$0")/gpu_steps.sh"
export TMPDIR=/tmp
rm -f $OUT/status.log
run bench_hipgraph 420 python bench.py --hipgraph --steps 10 --warmup 3 --eager-baseline off
run bench_fp8 420 python bench.py --fp8 --fp8-recipe delayed --steps 10 --warmup 3 --eager-baseline off
rm -rf $OUT/prof_fp8 $OUT/prof_bf16
run prof_fp8 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_fp8 -o run --output-format csv -- python bench.py --fp8 --fp8-recipe delayed --steps 3 --warmup 2 --eager-baseline off
run prof_bf16 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_bf16 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --eager-baseline off
