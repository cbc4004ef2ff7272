#!/bin/bash
# Round 5, session h: world-1 RCCL rehearsals of the data-/tensor-parallel programs with the round-5
# kernels (LTA_BENCH_FORCE_DIST=1: bucketed / coalesced collectives at full model size on one GPU),
# kernel traces for the FSDP and TP programs.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
run plain_mbs2 400 python -u bench.py --mbs 2 --eager-baseline off
LTA_BENCH_FORCE_DIST=1 run fsdp_mbs2 500 python -u bench.py --mbs 2 --parallel fsdp --eager-baseline off
LTA_BENCH_FORCE_DIST=1 run ddp_mbs2 500 python -u bench.py --mbs 2 --parallel ddp --eager-baseline off
run tp_plain 400 python -u bench.py --model Llama-3-8B --n-layer 4 --seq 8192 --eager-baseline off
LTA_BENCH_FORCE_DIST=1 run tp_dist 500 python -u bench.py --model Llama-3-8B --n-layer 4 --seq 8192 --parallel tp --eager-baseline off
export LTA_BENCH_FORCE_DIST=1
rm -rf $OUT/prof_fsdp $OUT/prof_tp
run prof_fsdp 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_fsdp -o run --output-format csv -- python bench.py --mbs 2 --parallel fsdp --steps 2 --warmup 2 --eager-baseline off
python scripts/step_breakdown.py $(ls $OUT/prof_fsdp/*/run_kernel_trace.csv $OUT/prof_fsdp/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/fsdp_breakdown.txt 2>&1
python scripts/collective_overlap.py $(ls $OUT/prof_fsdp/*/run_kernel_trace.csv $OUT/prof_fsdp/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/fsdp_overlap.txt 2>&1
run prof_tp 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_tp -o run --output-format csv -- python bench.py --model Llama-3-8B --n-layer 4 --seq 8192 --parallel tp --steps 2 --warmup 2 --eager-baseline off
python scripts/step_breakdown.py $(ls $OUT/prof_tp/*/run_kernel_trace.csv $OUT/prof_tp/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/tp_breakdown.txt 2>&1
python scripts/collective_overlap.py $(ls $OUT/prof_tp/*/run_kernel_trace.csv $OUT/prof_tp/run_kernel_trace.csv 2>/dev/null | head -1) > $OUT/tp_overlap.txt 2>&1
cp $(ls $OUT/prof_tp/*/run_kernel_trace.csv $OUT/prof_tp/run_kernel_trace.csv 2>/dev/null | head -1) $OUT/tp_kernel_trace.csv 2>/dev/null
rm -f $OUT/prof_fsdp/*/*kernel_trace.csv $OUT/prof_fsdp/run_kernel_trace.csv $OUT/prof_tp/*/*kernel_trace.csv $OUT/prof_tp/run_kernel_trace.csv 2>/dev/null
exit 0
