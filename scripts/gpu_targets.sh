#!/bin/bash
# benchmarks/targets.py (the reference's component benchmarks) on this tree + the host-overhead profile
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run targets 600 python -u -m lightning_thunder_amd.benchmarks.targets
run host_prof 300 python -u scripts/host_overhead_profile.py
