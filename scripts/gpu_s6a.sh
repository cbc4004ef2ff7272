#!/bin/bash
# forward GEMMs on hipBLASLt (LTA_GEMM_FWD_LIB=1) vs the hand kernel, Llama-2-7B step A/B
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run gateup 200 python -u scripts/gemm_shape_ab.py --model llama2-7b-gateup --json $OUT/gemm_gateup.json
grep '^{' $OUT/gateup.log
run bench_a 400 python -u bench.py --steps 10 --warmup 3 --eager-baseline off
grep -o '"ms_per_step": [0-9.]*' $OUT/bench_a.log | head -1
export LTA_GEMM_FWD_LIB=1
run bench_lib 400 python -u bench.py --steps 10 --warmup 3 --eager-baseline off
grep -o '"ms_per_step": [0-9.]*' $OUT/bench_lib.log | head -1
unset LTA_GEMM_FWD_LIB
run bench_b 400 python -u bench.py --steps 10 --warmup 3 --eager-baseline off
grep -o '"ms_per_step": [0-9.]*' $OUT/bench_b.log | head -1
