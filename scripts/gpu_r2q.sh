#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run blas_sweep 300 python -u scripts/blas_n_sweep.py
