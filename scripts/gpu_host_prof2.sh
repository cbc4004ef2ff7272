#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run hp_xl 300 python -u scripts/host_overhead_profile.py --model gpt2-xl --fwd-only --iters 10 --top 60
