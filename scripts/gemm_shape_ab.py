"""Per-shape A/B of the framework's GEMM dispatch (ops.gemm.linear / ops.gemm.matmul, i.e. what a
jitted step runs) against the library GEMM (torch -> hipBLASLt) for one model's training GEMMs:
forward ``x @ W^T``, dgrad ``dY @ W``, wgrad ``dY^T @ X``.  Random bf16 data, interleaved rounds,
best-of-3 means of 20 back-to-back calls.

    python scripts/gemm_shape_ab.py --model gpt2-medium [--json gpurun_out/gemm_shape_ab.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops import gemm as G

MODELS = {
    # tokens, [(N, K)] of the linears (qkv, attn proj, fc, mlp proj, lm head)
    "gpt2-medium": (8192, [(3072, 1024), (1024, 1024), (4096, 1024), (1024, 4096), (50304, 1024)]),
    "llama2-7b": (4096, [(12288, 4096), (4096, 4096), (11008, 4096), (4096, 11008), (32000, 4096)]),
    "llama2-7b-gateup": (4096, [(22016, 4096)]),
}


def timeit(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-medium", choices=sorted(MODELS))
    ap.add_argument("--json", default="gpurun_out/gemm_shape_ab.json")
    args = ap.parse_args()
    M, lins = MODELS[args.model]
    rows = []
    total = {"lta": 0.0, "blas": 0.0}
    for N, K in lins:
        x = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        w = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        dy = torch.empty(M, N, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        cases = {
            "fwd": (lambda: G.linear(x, w), lambda: torch.nn.functional.linear(x, w), (M, N, K)),
            "dgrad": (lambda: G.matmul(dy, w), lambda: dy @ w, (M, K, N)),
            "wgrad": (lambda: G.matmul(dy.t(), x), lambda: dy.t() @ x, (N, K, M)),
        }
        for name, (ours, blas, (m, n, k)) in cases.items():
            G.last_gemm_backend_counts(reset=True)
            ours()
            backend = ",".join(sorted(G.last_gemm_backend_counts(reset=True)))
            t = {"lta": [], "blas": []}
            for _ in range(3):
                t["lta"].append(timeit(ours))
                t["blas"].append(timeit(blas))
            us = {k: min(v) for k, v in t.items()}
            fl = 2 * m * n * k
            r = dict(gemm=name, M=m, N=n, K=k, backend=backend, lta_us=round(us["lta"], 1), blas_us=round(us["blas"], 1),
                     lta_tf=round(fl / us["lta"] / 1e6), blas_tf=round(fl / us["blas"] / 1e6),
                     tiles_256=-(-m // 256) * -(-n // 256))
            total["lta"] += us["lta"]
            total["blas"] += us["blas"]
            rows.append(r)
            print(json.dumps(r), flush=True)
    print(f"total per layer-set: lta {total['lta']:.1f} us, blas {total['blas']:.1f} us", flush=True)
    os.makedirs(os.path.dirname(args.json) or ".", exist_ok=True)
    with open(args.json, "w") as f:
        json.dump(dict(model=args.model, tokens=M, rows=rows, total_us=total), f, indent=1)


if __name__ == "__main__":
    main()
