#!/bin/bash
# Layout-general backward GEMMs: numerics, microbenchmark, traces, headline step.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
run pytest_layouts 300 python -u -m pytest tests/test_hip_kernels.py tests/test_extend_hip_kernel.py -m gpu -x -q --timeout 120 --timeout-method thread -k "layouts or hip_kernel"
run gemm_bwd 300 python -u scripts/gemm_bwd_bench.py
run traces 300 python -u scripts/dump_traces.py gpurun_out/traces
run bench_bf16 300 python -u bench.py --steps 10 --warmup 3
