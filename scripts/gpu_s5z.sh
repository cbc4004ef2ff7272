#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run hostprof 300 python -u scripts/host_overhead_profile.py --top 30
head -40 $OUT/hostprof.log
run targets_gpt2 300 python -u -m lightning_thunder_amd.benchmarks.targets -k nanogpt_gpt2
grep '^{' $OUT/targets_gpt2.log
