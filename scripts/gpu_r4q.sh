#!/bin/bash
# round 4: optimizer-overlap bitwise test with / without the non-temporal post-backward AdamW
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
export LTA_ADAMW_NT=0
run ov_nt0 200 python -u -m pytest tests/test_optim_overlap.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
export LTA_ADAMW_NT=1
run ov_nt1 200 python -u -m pytest tests/test_optim_overlap.py -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
