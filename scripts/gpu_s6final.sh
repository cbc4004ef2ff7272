#!/bin/bash
# round 5 closing run: GPT-2-medium step profile, full GPU suite, smoke, default bench (eager baseline on)
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
rm -rf $OUT/prof_gpt2
run prof_gpt2 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_gpt2 -o run --output-format csv -- python scripts/gpt2_step_profile.py
python scripts/step_breakdown.py $(ls $OUT/prof_gpt2/*/run_kernel_trace.csv $OUT/prof_gpt2/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/gpt2_breakdown.txt 2>&1
rm -f $OUT/prof_gpt2/*/*kernel_trace.csv $OUT/prof_gpt2/run_kernel_trace.csv 2>/dev/null
head -30 $OUT/gpt2_breakdown.txt
run suite 900 python -u -m pytest tests -q -m gpu --timeout 180 --timeout-method thread --ignore=tests/test_ops.py -p no:cacheprovider
run suite_ops 400 python -u -m pytest tests/test_ops.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
run bench 500 python -u bench.py
grep '"metric"' $OUT/bench.log | head -1
