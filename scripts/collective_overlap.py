"""Collective / compute overlap of one training step from a rocprofv3 kernel trace (CSV).

The step is the segment between the last two optimizer launches (``adamw`` kernels).  Collective
kernels are RCCL's (names with ``nccl`` / ``rccl`` / ``oneRank``) and the runtime copies it issues
(``copyBuffer``, RCCL's one-rank all-gather at world 1).  Prints span, kernel sum, busy union, the
collective kernel time, how much of it ran concurrently with compute kernels, and the copies per step."""
import csv
import sys


def is_coll(name: str) -> bool:
    n = name.lower()
    return any(k in n for k in ("nccl", "rccl", "onerank", "copybuffer", "allreduce", "allgather", "reducescatter"))


def union(iv):
    iv = sorted(iv)
    out, cur = 0, None
    for a, b in iv:
        if cur is None or a > cur[1]:
            if cur:
                out += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    if cur:
        out += cur[1] - cur[0]
    return out


def intersect(a_iv, b_iv):
    a_iv, b_iv = sorted(a_iv), sorted(b_iv)
    # merge b into disjoint intervals first
    merged = []
    for s, e in b_iv:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    tot, j = 0, 0
    for s, e in a_iv:
        while j < len(merged) and merged[j][1] <= s:
            j += 1
        k = j
        while k < len(merged) and merged[k][0] < e:
            tot += min(e, merged[k][1]) - max(s, merged[k][0])
            k += 1
    return tot


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"].lower()]
    seg = rows[idx[-2] + 1: idx[-1] + 1] if len(idx) >= 2 else rows
    iv = lambda rs: [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rs]  # noqa: E731
    coll = [r for r in seg if is_coll(r["Kernel_Name"])]
    comp = [r for r in seg if not is_coll(r["Kernel_Name"])]
    t0 = min(int(r["Start_Timestamp"]) for r in seg)
    t1 = max(int(r["End_Timestamp"]) for r in seg)
    ms = lambda ns: ns / 1e6  # noqa: E731
    csum = sum(b - a for a, b in iv(coll))
    cu = union(iv(coll))
    ov = intersect(iv(coll), iv(comp))
    print(f"step span {ms(t1 - t0):.2f} ms, kernel sum {ms(sum(b - a for a, b in iv(seg))):.2f} ms, busy union "
          f"{ms(union(iv(seg))):.2f} ms, compute union {ms(union(iv(comp))):.2f} ms")
    print(f"collective kernels: {len(coll)} launches, {ms(csum):.2f} ms summed, {ms(cu):.2f} ms union, "
          f"{ms(ov):.2f} ms of it concurrent with compute ({100 * ov / max(cu, 1):.0f} %)")
    names = {}
    for r in coll:
        k = r["Kernel_Name"].split("(")[0][:70]
        names[k] = names.get(k, 0) + 1
    for k, v in sorted(names.items(), key=lambda x: -x[1]):
        print(f"  {v:5d}x {k}")
    print(f"copyBuffer launches in the step: {sum(1 for r in seg if 'copybuffer' in r['Kernel_Name'].lower())}")


if __name__ == "__main__":
    main(sys.argv[1])
