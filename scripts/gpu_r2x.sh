#!/bin/bash
# Kernel profile of the world-1 RCCL rehearsals (DDP, FSDP) to find the data-parallel overheads.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
export LTA_BENCH_FORCE_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1
rm -rf $OUT/prof_ddp $OUT/prof_fsdp
MASTER_PORT=29621 run prof_ddp 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_ddp -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --parallel ddp
python scripts/step_breakdown.py $OUT/prof_ddp/run_kernel_trace.csv > $OUT/step_breakdown_ddp.txt
MASTER_PORT=29622 run prof_fsdp 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_fsdp -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --parallel fsdp
python scripts/step_breakdown.py $OUT/prof_fsdp/run_kernel_trace.csv > $OUT/step_breakdown_fsdp.txt
run pytest_dist_gpu 300 python -u -m pytest tests/test_distributed_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
