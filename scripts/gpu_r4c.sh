#!/bin/bash
# round 4: v4 phase stamps, new GPU tests (edge tiles, padded head dims, fusion repro, fp8 x checkpoint,
# LDS-DMA OOB probe, grouped GEMMs + MoE backward), world-8 gloo rehearsal
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run stamps 120 python -u scripts/attn_v4_stamps.py
run t_probe 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread tests/test_hip_kernels.py -k "lds_dma_out_of_range" -m gpu
run t_new 600 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py tests/test_dynamo_report.py -k "edge_tiles or flash_attention or fusion_repro or activation_checkpointing or grouped or moe_training" -m gpu
run gpt2_trace 300 python -u scripts/gpt2_trace_dump.py
run prof_gpt2 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_gpt2 -o run --output-format csv -- python scripts/gpt2_step_profile.py
bash scripts/dist_rehearsal8.sh
