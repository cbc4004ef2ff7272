#!/bin/bash
# hardware exp / rcp in 16-bit-output hipfuse regions: tests, roofline, GPT-2 step profile
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run hipfuse_test 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hipfuse.py -m gpu
grep -qE "[0-9]+ failed" $OUT/hipfuse_test.log && exit 1
run roofline 400 python -u scripts/hipfuse_roofline.py --json $OUT/hipfuse_roofline.json
grep -v amdgpu.ids $OUT/roofline.log
rm -rf $OUT/prof_gpt2
run prof_gpt2 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_gpt2 -o run --output-format csv -- python scripts/gpt2_step_profile.py
python scripts/step_breakdown.py $(ls $OUT/prof_gpt2/*/run_kernel_trace.csv $OUT/prof_gpt2/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/gpt2_breakdown.txt 2>&1
head -30 $OUT/gpt2_breakdown.txt
