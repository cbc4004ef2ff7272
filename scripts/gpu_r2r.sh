#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run tunable_probe 600 python -u scripts/tunable_probe.py
