#!/bin/bash
# component targets (benchmarks/targets.py: the reference's targets.py micro-benchmarks, fwd / bwd, eager vs jit)
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run targets 900 python -u -m lightning_thunder_amd.benchmarks.targets
grep '^{' $OUT/targets.log > $OUT/targets_r5.jsonl
wc -l $OUT/targets_r5.jsonl
