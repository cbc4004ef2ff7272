#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run hf_traces 300 python -u scripts/dump_hf_traces.py gpurun_out/hf_traces
