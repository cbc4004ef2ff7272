#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
rm -rf $OUT/pt_thunder $OUT/pt_eager
run pt_thunder 300 rocprofv3 --kernel-trace --stats -d $OUT/pt_thunder -o run --output-format csv -- python scripts/prof_target.py nanogpt_gpt2xl thunder
run pt_eager 300 rocprofv3 --kernel-trace --stats -d $OUT/pt_eager -o run --output-format csv -- python scripts/prof_target.py nanogpt_gpt2xl eager
