#!/bin/bash
# round 3: index kernels, weighted CE, hipfuse column mode, FP8xFSDP, 7B-shape numerics, decode logits,
# bench (gemm4 everywhere), step profile, gemm4 K-major pitch probe
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run kern 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_index_ops.py tests/test_hipfuse.py tests/test_hip_kernels.py -k "index or topk or sort or cumsum or embedding or cross_entropy or claimed or fused or nf4"
run decode 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_generate.py -k teacher
run fp8_fsdp 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_fp8_fsdp.py
run gpu7b 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_7b_shape.py
run bench 600 python -u bench.py --steps 10 --warmup 3
run probe 300 python -u scripts/gemm4_probe.py
rm -rf $OUT/prof_bench
run prof_bench 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o run --output-format csv -- python bench.py --steps 3 --warmup 2
