#!/bin/bash
# round 3: kernel tests after fixes (index, CE weights, hipfuse column mode, NF4, grouped fp8), decode
# logits, FP8xFSDP, gemm4 register-staged variant A/B
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run gemm4 600 python -u scripts/gemm4_bench.py --rounds 2 --iters 20 --variants 1,3
run kern 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_index_ops.py tests/test_hipfuse.py tests/test_hip_kernels.py -k "index or topk or sort or cumsum or embedding or cross_entropy or claimed or fused or nf4 or grouped or adamw"
run decode 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_generate.py -k teacher
run fp8_fsdp 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fp8_fsdp.py
run bench 600 python -u bench.py --steps 10 --warmup 3
