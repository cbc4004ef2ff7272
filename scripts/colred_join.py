"""Device-side medians of scripts/colred_bench.py's kernels: joins its JSON with a rocprofv3 kernel trace.
    python scripts/colred_join.py gpurun_out/colred_bench.json gpurun_out/prof_colred/run_kernel_trace.csv"""
import csv
import json
import statistics
import sys
from collections import defaultdict

rows = json.load(open(sys.argv[1]))["rows"]
durs = defaultdict(list)
for r in csv.DictReader(open(sys.argv[2])):
    durs[r["Kernel_Name"].split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for row in rows:
    out = []
    for cfg, v in row.items():
        if isinstance(v, dict) and "kernel" in v:
            k = statistics.median(durs[v["kernel"]]) + (statistics.median(durs[v["kernel"] + "_fin"])
                                                         if v["kernel"] + "_fin" in durs else 0.0)
            out.append(f"{cfg} {v['mode']} {k:.2f}us {row['mbytes'] / k:.2f}TB/s")
    print(row["shape"], " | ".join(out), flush=True)
