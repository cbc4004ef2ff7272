"""Per-kernel mean of rocprofv3 --pmc counters over dispatches (counter_collection.csv files).

    python scripts/pmc_summary.py OUT.json DIR [DIR ...]   (each DIR one --pmc pass)
Derived ratios (when the counters are present): clock (GRBM_GUI_ACTIVE / 8 XCDs / duration is not
available here, so quad-cycle ratios only), VALU / MFMA instructions, issue-stall and wait fractions."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(lambda: defaultdict(list))
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "").replace("(anonymous namespace)::", "").replace("void ", "")
            k = k.split("(")[0]
            name = r.get("Counter_Name")
            val = float(r.get("Counter_Value", 0) or 0)
            disp = r.get("Dispatch_Id", r.get("Correlation_Id", "0"))
            acc[k][(name, disp)].append(val)
    out = defaultdict(dict)
    for k, m in acc.items():
        per = defaultdict(list)
        for (name, disp), vals in m.items():
            per[name].append(sum(vals))  # sum over dimensions (XCD / SE instances) of one dispatch
        for name, vals in per.items():
            out[k][name] = sum(vals) / len(vals)
    return out


def main():
    dst = sys.argv[1]
    merged = defaultdict(dict)
    for d in sys.argv[2:]:
        for k, v in load(d).items():
            merged[k].update(v)
    for k, v in merged.items():
        if v.get("SQ_WAVE_CYCLES"):
            w = v["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in v:
                    v["frac_" + c] = round(v[c] / w, 3)
        if v.get("SQ_INSTS_MFMA"):
            v["valu_per_mfma"] = round(v.get("SQ_INSTS_VALU", 0) / v["SQ_INSTS_MFMA"], 2)
            v["lds_per_mfma"] = round(v.get("SQ_INSTS_LDS", 0) / v["SQ_INSTS_MFMA"], 2)
    json.dump(merged, open(dst, "w"), indent=1, sort_keys=True)
    for k, v in merged.items():
        print(k[:70], {kk: (round(vv, 3) if isinstance(vv, float) else vv) for kk, vv in v.items() if kk.startswith(("frac", "valu", "lds_per"))})


if __name__ == "__main__":
    main()
