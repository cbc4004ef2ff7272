#!/bin/bash
# Full GPU suite after the round-2 kernel/fusion changes + HF decode trace dump.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run hf_traces 300 python -u scripts/dump_hf_traces.py gpurun_out/hf_traces
run pytest_gpu 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
