set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_hip_kernels.py -k "splitk or tail_split" > gpurun_out/splitk_test.log 2>&1; rc=$?; echo "test rc=$rc"; tail -3 gpurun_out/splitk_test.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u scripts/gemm_shape_ab.py --model gpt2-medium --json gpurun_out/gemm_shape_ab_gpt2_splitk.json > gpurun_out/gemm_ab_gpt2_splitk.log 2>&1; echo "gpt2 rc=$?"
grep -v amdgpu.ids gpurun_out/gemm_ab_gpt2_splitk.log
