#!/bin/bash
# Helper for GPU sessions: `source scripts/gpu_steps.sh` then `run NAME TIMEOUT cmd...`.
# Every step has its own time limit; a crash/abort/timeout (rc not 0/1) ends the session.
set -o pipefail
cd "$(dirname "${BASH_SOURCE[0]}")/.."
export PYTHONPATH=$PWD:$PYTHONPATH
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
run() {
  local name=$1 t=$2
  shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $OUT/status.log
  tail -4 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)"
    exit $rc
  fi
  return 0
}
