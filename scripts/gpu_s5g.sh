#!/bin/bash
# Round 5, session g: register epilogues for every gemm4 mode (incl. fused SwiGLU gate-up / backward);
# numerics; same-box A/B of the fused SwiGLU epilogues on the step.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run gemm_tests 600 python -u -m pytest tests/test_hip_kernels.py tests/test_gpu_swiglu_gemm.py tests/test_gpu_7b_shape.py -x -q --timeout 120 --timeout-method thread -k "gemm or qkv or grouped or moe or tail or swiglu or 7b or linear or fp8"
run epi_ab2 400 python -u scripts/exp/gemm_epi_ab.py
run bench_unfused 400 python -u bench.py --eager-baseline off
LTA_FUSED_SWIGLU=1 run bench_fused 400 python -u bench.py --eager-baseline off
run bench_unfused2 400 python -u bench.py --eager-baseline off
LTA_FUSED_SWIGLU=1 run bench_fused2 400 python -u bench.py --eager-baseline off
exit 0
