"""Summarize a rocprofv3 kernel_stats.csv: top kernels by total time."""
import csv, sys
path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_stats.csv"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} launches")
for r in rows[:n]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f}ms {float(r['Percentage']):5.1f}% n={r['Calls']:>5} avg={float(r['AverageNs'])/1e3:8.1f}us  {r['Name'][:100]}")
