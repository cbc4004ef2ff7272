"""Device-side durations for the hipfuse roofline: joins ``scripts/hipfuse_roofline.py``'s JSON (bytes,
calls, event-timed batches of Python launches) with the median kernel duration of each generated kernel
in a rocprofv3 kernel trace of the same run.  The event-timed batches include the host cost of every
``hipfuse.launch`` call, so for kernels shorter than that (~10 us) they read the launch rate, not the
kernel; the trace reads the kernel.

    rocprofv3 --kernel-trace -d gpurun_out/prof_roof -o run --output-format csv -- \
        python scripts/hipfuse_roofline.py --json gpurun_out/hipfuse_roofline.json
    python scripts/roofline_from_trace.py gpurun_out/hipfuse_roofline.json gpurun_out/prof_roof/run_kernel_trace.csv
"""
import csv
import json
import statistics
import sys
from collections import defaultdict

HBM_TBS = 8.0


def main():
    roof = json.load(open(sys.argv[1]))
    durs = defaultdict(list)
    for r in csv.DictReader(open(sys.argv[2])):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if name.startswith("lta_fused_"):
            durs[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{'kernel':28s} {'mode':10s} {'calls':>5s} {'MB':>8s} {'batch us':>8s} {'kernel us':>9s} {'TB/s':>6s} "
          f"{'%HBM':>5s}  domain")
    total_b = total_k = 0.0
    for d in roof["kernels"]:
        ds = durs.get(d["kernel"])
        if not ds:
            continue
        k = statistics.median(ds)
        tbs = d["mbytes"] / k  # MB per us = TB/s
        total_b += d["us"] * d["calls_per_step"] / 1e3
        total_k += k * d["calls_per_step"] / 1e3
        print(f"{d['kernel']:28s} {d['mode']:10s} {d['calls_per_step']:5d} {d['mbytes']:8.2f} {d['us']:8.2f} {k:9.2f} "
              f"{tbs:6.2f} {100 * tbs / HBM_TBS:5.1f}  {d['domain']}  {','.join(d['ops'])[:60]}")
    print(f"per step: {total_b:.2f} ms event-timed batches, {total_k:.2f} ms kernel time (trace medians)")


if __name__ == "__main__":
    main()
