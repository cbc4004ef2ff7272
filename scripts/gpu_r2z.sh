#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run overlap 300 python -u scripts/overlap_probe.py
