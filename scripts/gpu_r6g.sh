#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run gpt2dump 300 python -u scripts/gpt2_trace_dump.py
