"""Per-step kernel breakdown from a rocprofv3 kernel trace (steps delimited by the AdamW kernel)."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_bench/run_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
# complete steps between consecutive AdamW kernels; report the median-span one (a host stall -- GC,
# a page-in -- in a single step would otherwise set the printed span)
segs = [rows[a + 1: b + 1] for a, b in zip(idx[:-1], idx[1:])]
spans = [int(sg[-1]["End_Timestamp"]) - int(sg[0]["Start_Timestamp"]) for sg in segs]
order = sorted(range(len(segs)), key=lambda k: spans[k])
seg = segs[order[(len(order) - 1) // 2]]
if len(segs) > 1:
    print("step spans (ms): " + ", ".join(f"{x / 1e6:.2f}" for x in spans) + " -> median step below")


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    if "at::native" in n:
        for k in ["CUDAFunctor_add", "direct_copy", "bfloat16_copy", "FillFunctor", "MulFunctor", "sum", "reduce"]:
            if k in n:
                return "aten:" + k
        return "aten:" + n[:50]
    if n.startswith("Cijk") or n.startswith("Custom_Cijk"):
        return "hipBLASLt:" + n.split("_MT")[1][:12] if "_MT" in n else n[:40]
    return n.split("(")[0][:60]


t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
print(f"step span {(t1 - t0) / 1e6:.2f} ms, kernel busy {busy / 1e6:.2f} ms, {len(seg)} launches")
agg = defaultdict(lambda: [0, 0.0])
for r in seg:
    k = short(r["Kernel_Name"])
    agg[k][0] += 1
    agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{t:8.2f} ms {n:5d}x  {k}")
