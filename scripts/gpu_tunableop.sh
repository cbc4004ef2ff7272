#!/bin/bash
# Tune ATen's hipBLASLt/rocBLAS GEMM choices for the headline step (PyTorch TunableOp), then re-bench with them.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1
export PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop_results%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=10
run tune 900 python -u bench.py --steps 2 --warmup 1
export PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_VERBOSE=0
run bench_tuned 300 python -u bench.py --steps 10 --warmup 3
unset PYTORCH_TUNABLEOP_ENABLED
run bench_plain 300 python -u bench.py --steps 10 --warmup 3
