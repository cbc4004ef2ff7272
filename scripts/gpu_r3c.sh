#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_hf_gpu 600 python -u -m pytest tests/test_networks.py -m gpu -v --timeout 120 --timeout-method thread -k hf_architectures_gpu
