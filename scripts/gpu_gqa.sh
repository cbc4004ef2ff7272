#!/bin/bash
# GQA head split of the attention dK/dV pass: numerics (fp32-referenced kernel tests incl. the
# Mistral shape), model tests, then Mistral-7B bench with the split and without (A/B), and a profile.
source "$(dirname "$0")/gpu_steps.sh"
export TMPDIR=/tmp
rm -f $OUT/status.log
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
run t_attn 400 $PYT tests/test_hip_kernels.py -m gpu -k "dq_from_ds or attention_backward or attn_bwd or rope"
run t_models 300 $PYT tests/test_gpu_models.py -m gpu
run bench_mistral_split 420 python bench.py --model Mistral-7B-v0.1 --steps 10 --warmup 3 --eager-baseline off
run bench_mistral_nosplit 420 env LTA_ATTN_GQA_SPLIT=1 python bench.py --model Mistral-7B-v0.1 --steps 10 --warmup 3 --eager-baseline off
rm -rf $OUT/prof_Mistral
run prof_Mistral 500 rocprofv3 --kernel-trace --stats -d $OUT/prof_Mistral -o run --output-format csv -- python bench.py --model Mistral-7B-v0.1 --steps 3 --warmup 2 --eager-baseline off
