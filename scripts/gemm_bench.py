"""A/B of the NT GEMM variants against hipBLASLt on the Llama-2-7B training shapes (random data).

    python scripts/gemm_bench.py [--rounds 3] [--iters 20]
Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24); prints one JSON line.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops.gemm import gemm_nt

SHAPES = [(4096, 12288, 4096), (4096, 4096, 4096), (4096, 11008, 4096), (4096, 4096, 11008), (4096, 32000, 4096),
          (8192, 8192, 8192)]


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--iters", type=int, default=20)
    args = p.parse_args()
    out = {}
    for M, N, K in SHAPES:
        a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        ref = (a.float() @ b.float().t())
        errs = {}
        for v in (0, 1):
            y = gemm_nt(a, b, variant=v).float()
            errs[v] = ((y - ref).abs().max() / ref.abs().max()).item()
        fns = {"v0": lambda: gemm_nt(a, b, variant=0), "v1": lambda: gemm_nt(a, b, variant=1),
               "hipblaslt": lambda: torch.nn.functional.linear(a, b)}
        ts = {k: [] for k in fns}
        for _ in range(args.rounds):
            for k, f in fns.items():
                ts[k].append(timeit(f, args.iters))
        flops = 2 * M * N * K
        res = {k: round(flops / (min(v) * 1e-3) / 1e12) for k, v in ts.items()}
        res["rel_err_v0"], res["rel_err_v1"] = errs[0], errs[1]
        out[f"{M}x{N}x{K}"] = res
        print(f"{M}x{N}x{K}: {res}", file=sys.stderr, flush=True)
        del a, b, ref
    print(json.dumps({"gemm_nt_tflops_random": out}))


if __name__ == "__main__":
    main()
