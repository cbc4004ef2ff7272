#!/bin/bash
# round 4: hipfuse 32-byte vectors: GPU numerics of the fusion tests + networks, GPT-2 roofline and step
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run hf_tests 400 python -u -m pytest tests/test_hipfuse.py tests/test_networks.py tests/test_gpu_models.py -q -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider
run roofline 300 python -u scripts/hipfuse_roofline.py
rm -rf $OUT/prof_gpt2
run prof_gpt2 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_gpt2 -o run --output-format csv -- python scripts/gpt2_step_profile.py
python scripts/step_breakdown.py gpurun_out/prof_gpt2/run_kernel_trace.csv > $OUT/gpt2_breakdown.txt 2>&1
