#!/bin/bash
# round 4: v4 phase stamps, new GPU tests, world-8 gloo rehearsal
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run stamps 120 python -u scripts/attn_v4_stamps.py
run t_new 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py tests/test_dynamo_report.py -k "edge_tiles or flash_attention or fusion_repro or activation_checkpointing" -m gpu
bash scripts/dist_rehearsal8.sh
