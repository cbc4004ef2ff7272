"""Column reductions (``x.float().sum(0)``, the bias-grad shape) through hipfuse's single-launch
column mode: partial hand-off "coherent" (sc1 vector memory ops) vs "fence" (__threadfence), and
ATen's reduction, on the GPT-2-medium bias-grad shapes.  Per-launch time from batches of
back-to-back launches rotating over input copies totalling >= 1.5 GB (no Infinity Cache hits).

    python scripts/colred_bench.py [--json gpurun_out/colred_bench.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.executors import hipfuse
from lightning_thunder_amd.executors import hipfuse_codegen as cg

SHAPES = [(8192, 1024), (8192, 3072), (8192, 4096), (4096, 11008), (8192, 50304)]


# (name, hand-off, waves per workgroup, target workgroups, rows in flight per wave); "default" = the
# module's tuned configuration (hipfuse_codegen.COL_*)
CONFIGS = [("twopass", "twopass", 4, 512, 4), ("coh_nw8_128", "coherent", 8, 128, 4), ("coh_nw8_256_u8", "coherent", 8, 256, 8),
           ("default", "coherent", cg.COL_NW, cg.COL_WGS, cg.COL_UNROLL)]


def per_launch_us(fn, copies, reps=7):
    fn(copies[0])
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for c in copies:
            fn(c)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / len(copies))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default="gpurun_out/colred_bench.json")
    args = ap.parse_args()
    rows = []
    for R, C in SHAPES:
        x = torch.randn(R, C, device="cuda", dtype=torch.bfloat16)
        nbytes = x.numel() * 2 + C * 2
        k = max(2, min(64, -(-int(1.5e9) // nbytes)))
        copies = [x.clone() for _ in range(k)]
        ref = x.double().sum(0)
        row = dict(shape=[R, C], mbytes=round(nbytes / 1e6, 2))

        def f(t):
            return t.float().sum(0).to(torch.bfloat16)

        for name, mode, nw, wgs, un in CONFIGS:
            cg.COL_SYNC, cg.COL_NW, cg.COL_WGS, cg.COL_UNROLL = mode, nw, wgs, un
            jf = thunder.jit(f, executors=["hipfuse", "torch"])
            out = jf(x)
            fus = hipfuse.fusions(thunder.last_traces(jf)[-1])
            assert len(fus) == 1, fus
            hf = fus[0]._call_ctx[fus[0].sym.name]
            fns, ks = hf._variant([x])
            err = ((out.double() - ref).abs().max() / ref.abs().max()).item()
            again = jf(x)
            o = torch.empty(C, device="cuda", dtype=torch.bfloat16)
            us = per_launch_us(lambda t: hipfuse.launch(ks, fns, [t], [o], []), copies)
            row[name] = dict(kernel=ks.name, mode=ks.mode, us=round(us, 2), tb_s=round(nbytes / us / 1e6, 2), rel_err=err,
                             deterministic=bool(torch.equal(out, again)))
        cg.COL_SYNC, cg.COL_NW, cg.COL_WGS, cg.COL_UNROLL = CONFIGS[-1][1:]
        us = per_launch_us(f, copies)
        row["aten"] = dict(us=round(us, 2), tb_s=round(nbytes / us / 1e6, 2))
        rows.append(row)
        print(json.dumps(row), flush=True)
        del copies
    os.makedirs(os.path.dirname(args.json) or ".", exist_ok=True)
    with open(args.json, "w") as fh:
        json.dump(dict(note="per-launch us of the generated kernel(s), batched launches over rotating copies; "
                       "TB/s vs ~8 TB/s HBM", rows=rows), fh, indent=1)


if __name__ == "__main__":
    main()
