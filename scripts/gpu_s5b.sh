#!/bin/bash
# Round 5, session b: gemm4 main-loop anatomy (scripts/exp) + step profile of the default bench.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
python -c "import torch; p=torch.cuda.get_device_properties(0); print('CUs', p.multi_processor_count, p.name)" > $OUT/cus.log 2>&1
run anatomy 300 python -u scripts/exp/gemm_anatomy.py
rm -rf $OUT/prof_bench
run prof_bench 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --eager-baseline off
python scripts/step_breakdown.py $(ls $OUT/prof_bench/*/run_kernel_trace.csv $OUT/prof_bench/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/step_breakdown.txt 2>&1
rm -f $OUT/prof_bench/*/*kernel_trace.csv $OUT/prof_bench/run_kernel_trace.csv 2>/dev/null
exit 0
