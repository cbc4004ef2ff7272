#!/bin/bash
# round 4: attention v4 numerics/perf + GEMM edge-tile tests + gemm4 microbench
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run attn_check 300 python -u scripts/attn_v4_check.py 0,9,10
run gemm_edge 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "edge_tiles or gemm_bf16_layouts or gemm_nt_bf16" -m gpu
run gemm4_bench 300 python -u scripts/gemm4_bench.py
