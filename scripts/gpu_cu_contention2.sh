#!/bin/bash
# Whole-step sensitivity with RCCL-shaped occupiers (37.6 KB LDS, 256 VGPRs as ncclDevKernel_Generic on gfx950:
# more than the GEMM's 128 KB LDS ring leaves free, so no co-residency) and the hipGraph step profile.
source "$(dirname "$0")/gpu_steps.sh"
export TMPDIR=/tmp
rm -f $OUT/status.log
run cu_cont_rccl 400 python scripts/cu_contention.py --threads 256 --lds 37664 --n 0,8,32 --step
