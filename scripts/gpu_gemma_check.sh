set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hipfuse.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/hf_gpu.log 2>&1 && tail -2 gpurun_out/hf_gpu.log &&
timeout -k 10 300 python -u scripts/fp8_cast_bench.py > gpurun_out/fp8_cast.log 2>&1 && cat gpurun_out/fp8_cast.log &&
timeout -k 10 300 python -u scripts/fusion_debug.py Gemma-7b 1 > gpurun_out/fd_gemma.log 2>&1 && grep -c hipFusion gpurun_out/fd_gemma.log &&
timeout -k 10 420 python -u bench.py --model Gemma-7b --steps 10 --warmup 3 > gpurun_out/mb_gemma.log 2>&1 && tail -1 gpurun_out/mb_gemma.log
