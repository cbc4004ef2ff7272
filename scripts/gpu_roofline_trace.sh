#!/bin/bash
# hipfuse roofline of the GPT-2-medium step with device-side kernel durations (rocprofv3 kernel trace)
# next to the event-timed launch batches; plus the column-reduction sweep under the same trace.
source "$(dirname "$0")/gpu_steps.sh"
rm -f $OUT/status.log
rm -rf $OUT/prof_roof $OUT/prof_colred
run roof 400 rocprofv3 --kernel-trace -d $OUT/prof_roof -o run --output-format csv -- python scripts/hipfuse_roofline.py --json $OUT/hipfuse_roofline.json
run roof_join 60 python scripts/roofline_from_trace.py $OUT/hipfuse_roofline.json $OUT/prof_roof/run_kernel_trace.csv
run colred 400 rocprofv3 --kernel-trace -d $OUT/prof_colred -o run --output-format csv -- python scripts/colred_bench.py --json $OUT/colred_bench.json
