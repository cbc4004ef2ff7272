set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/gemm_shape_ab.py --model gpt2-medium --json gpurun_out/gemm_shape_ab_gpt2.json > gpurun_out/gemm_ab_gpt2.log 2>&1; echo "gpt2 rc=$?"
timeout -k 10 300 python -u scripts/gemm_shape_ab.py --model llama2-7b --json gpurun_out/gemm_shape_ab_llama.json > gpurun_out/gemm_ab_llama.log 2>&1; echo "llama rc=$?"
cat gpurun_out/gemm_ab_gpt2.log gpurun_out/gemm_ab_llama.log | grep -v amdgpu.ids
