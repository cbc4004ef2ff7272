#!/bin/bash
# RCCL workgroup shape (world-1 kernel trace) + the CU-contention curve (scripts/cu_contention.py).
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run rccl_shape 180 rocprofv3 --kernel-trace --stats -d $OUT/rccl_shape -o rccl -- python scripts/rccl_kernel_shape.py
run cu_cont_256 400 python scripts/cu_contention.py --threads 256 --lds 0 --step
run cu_cont_lds 300 python scripts/cu_contention.py --threads 256 --lds 65536
rm -rf $OUT/prof_hipgraph
run prof_hipgraph 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_hipgraph -o run --output-format csv -- python bench.py --hipgraph --steps 4 --warmup 3 --eager-baseline off
