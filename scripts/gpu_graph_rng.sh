#!/bin/bash
# graph-safe RNG: hipGraph tests (incl. the dropout model vs uncaptured), gemm4 odd-K / plan tests,
# targets.py NanoGPT rows with and without hipGraph, host profile of the GPT-2 XL forward
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_graph 400 python -u -m pytest tests/test_hipgraph.py tests/test_hipfuse.py -x -q -m gpu --timeout 200 --timeout-method thread
run t_gemm4 400 python -u -m pytest tests/test_hip_kernels.py -x -q -k "gemm4 or gemm_nt or linear or attn or dropout" --timeout 120 --timeout-method thread
run targets 600 python -u -m lightning_thunder_amd.benchmarks.targets -k nanogpt --executors eager,thunder,thunder+hipgraph
run hgdiag 300 python -u scripts/hipgraph_diag.py
