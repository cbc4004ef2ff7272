#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run gen_mx 600 python -u -m lightning_thunder_amd.benchmarks.generate --modes eager,hipgraph,hipgraph_mxfp4 --iters 3
