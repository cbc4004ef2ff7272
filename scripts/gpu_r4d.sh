#!/bin/bash
# round 4: hipfuse shape/index ops on the GPU (fp64-referenced), grouped GEMM fix, attention
# gradient layout, GPT-2 step profile + generated-kernel bandwidth roofline, v4 phase stamps
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run t_fuse 600 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_hipfuse.py -m gpu
run t_k 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "grouped or strided_qkv or flash_attention" -m gpu
run t_ops 900 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_ops.py -m gpu
run roofline 400 python -u scripts/hipfuse_roofline.py
run prof_gpt2 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_gpt2 -o run --output-format csv -- python scripts/gpt2_step_profile.py
run stamps 120 python -u scripts/attn_v4_stamps.py
