#!/bin/bash
# One GPU session: tests, smoke, bench (thunder + eager), kernel profile. Stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
export PYTHONPATH=$PWD:$PYTHONPATH
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
STEPS=${STEPS:-5}
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1; echo "pytest rc=$?" | tee -a $OUT/status.log
tail -5 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && echo "smoke ok" | tee -a $OUT/status.log || { echo "smoke FAILED"; tail -30 $OUT/smoke.log; exit 1; }
timeout -k 10 900 python bench.py --steps $STEPS --warmup 2 > $OUT/bench_thunder.log 2>&1; echo "bench thunder rc=$?" | tee -a $OUT/status.log
tail -4 $OUT/bench_thunder.log
if [ "${EAGER:-1}" = "1" ]; then
timeout -k 10 600 python bench.py --steps $STEPS --warmup 2 --mode eager > $OUT/bench_eager.log 2>&1; echo "bench eager rc=$?" | tee -a $OUT/status.log
tail -3 $OUT/bench_eager.log
fi
if [ "${PROF:-1}" = "1" ]; then
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 2 --warmup 1 > $OUT/prof.log 2>&1; echo "prof rc=$?" | tee -a $OUT/status.log
fi
