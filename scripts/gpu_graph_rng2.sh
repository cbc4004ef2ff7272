#!/bin/bash
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_graph 400 python -u -m pytest tests/test_hipgraph.py -x -q -m gpu --timeout 200 --timeout-method thread
run targets 600 python -u -m lightning_thunder_amd.benchmarks.targets -k nanogpt_gpt2xl --executors thunder,thunder+hipgraph
rm -rf $OUT/pt_hg
run pt_hg 300 rocprofv3 --kernel-trace --stats -d $OUT/pt_hg -o run --output-format csv -- python scripts/prof_target.py nanogpt_gpt2xl thunder+hipgraph backward
rm -rf $OUT/pt_th
run pt_th 300 rocprofv3 --kernel-trace --stats -d $OUT/pt_th -o run --output-format csv -- python scripts/prof_target.py nanogpt_gpt2xl thunder backward
