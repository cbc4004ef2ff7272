#!/bin/bash
# Llama-2-7B bench A/B: fused SwiGLU epilogues (register epilogue) vs separate passes; plus default bench
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run bench_default 500 python -u bench.py --steps 10 --warmup 3 --eager-baseline off
grep '"metric"' $OUT/bench_default.log
export LTA_FUSED_SWIGLU=1; run bench_fused 500 python -u bench.py --steps 10 --warmup 3 --eager-baseline off
grep "\"metric\"" $OUT/bench_fused.log; unset LTA_FUSED_SWIGLU
run bench_default2 500 python -u bench.py --steps 10 --warmup 3 --eager-baseline off
grep '"metric"' $OUT/bench_default2.log
