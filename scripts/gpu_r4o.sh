#!/bin/bash
# round 4: LayerNorm backward v2 + residual fusion: numerics, GPT-2 step profile
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run ln_tests 300 python -u -m pytest tests/test_hip_kernels.py tests/test_networks.py tests/test_gpu_models.py -q -m gpu -k "layer_norm or gpt or neox or hf_arch" --timeout 180 --timeout-method thread -p no:cacheprovider
rm -rf $OUT/prof_gpt2
run prof_gpt2 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_gpt2 -o run --output-format csv -- python scripts/gpt2_step_profile.py
python scripts/step_breakdown.py gpurun_out/prof_gpt2/run_kernel_trace.csv > $OUT/gpt2_breakdown.txt 2>&1
