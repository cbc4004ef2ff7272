#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run bench 600 python bench.py --steps 10 --warmup 3
