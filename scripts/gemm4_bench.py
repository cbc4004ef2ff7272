"""Correctness + A/B of the 4-wave GEMM (csrc/gemm4.hip) on the Llama-2-7B training GEMMs.

    python scripts/gemm4_bench.py [--rounds 3] [--iters 20] [--variants 1] [--quick]

For every linear of the Llama-2-7B step (M = 4096 tokens) it times the forward (X . W^T), dgrad
(dY . W) and wgrad (dY^T . X) products on random data, interleaved in one process
(cdna_hip_programming.md §5.4 rule 24): gemm4 variants, the previous hand kernel (gemm.hip) and
torch.matmul (hipBLASLt).  Prints one JSON line; per-shape progress goes to stderr.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops import gemm as G

# (N, K) of each Llama-2-7B linear, as nn.Linear(K -> N); M = 4096 tokens
LINEARS = [(12288, 4096), (4096, 4096), (11008, 4096), (22016, 4096), (4096, 11008), (32000, 4096)]


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


def check_correctness():
    """Every layout and epilogue against an fp32 reference at a small tile-divisible shape."""
    torch.manual_seed(0)
    out = {}
    M, N, K = 512, 768, 512
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    dy = torch.randn(M, N, device="cuda").bfloat16()
    bias = torch.randn(N, device="cuda").bfloat16()
    res = torch.randn(M, N, device="cuda").bfloat16()

    def rel(y, ref):
        return ((y.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-6)).item()

    cases = {
        "fwd": (x, w.t(), x.float() @ w.float().t()),
        "dgrad": (dy, w, dy.float() @ w.float()),
        "wgrad": (dy.t(), x, dy.float().t() @ x.float()),
        "tn": (x.t().contiguous().t(), w.t(), x.float() @ w.float().t()),
    }
    for name, (a, b, ref) in cases.items():
        for v in (0, 1, 2):
            out[f"{name}_v{v}"] = rel(G.matmul4(a, b, variant=v), ref)
    ref = torch.nn.functional.silu(x.float() @ w.float().t() + bias.float())
    out["fwd_bias_silu"] = rel(G.matmul4(x, w.t(), bias=bias, act="silu", variant=1), ref)
    ref = (x.float() @ w.float().t()).bfloat16().float() + res.float()
    out["fwd_residual"] = rel(G.matmul4(x, w.t(), residual=res), ref)
    ref = dy.float() @ w.float() + res[:, :K].float()
    r2 = res[:, :K].contiguous()
    out["dgrad_residual"] = rel(G.matmul4(dy, w, residual=r2), ref)
    # asymmetric operands (catches a transposed C write): A = I
    eye = torch.eye(512, device="cuda").bfloat16()
    b = torch.arange(512 * 256, device="cuda").reshape(512, 256).float().remainder(97).bfloat16()
    out["identity_exact"] = bool(torch.equal(G.matmul4(eye, b), b))
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--variants", default="1")
    p.add_argument("--quick", action="store_true", help="only the 4096x4096x4096 products")
    args = p.parse_args()
    variants = [int(v) for v in args.variants.split(",")]
    res = {"correctness": check_correctness()}
    print(json.dumps(res["correctness"]), file=sys.stderr, flush=True)
    M = 4096
    linears = [(4096, 4096)] if args.quick else LINEARS
    perf = {}
    for N, K in linears:
        x = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        w = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        dy = torch.empty(M, N, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        prods = {"fwd": (x, w.t()), "dgrad": (dy, w), "wgrad": (dy.t(), x)}
        for kind, (a, b) in prods.items():
            fns = {f"g4v{v}": (lambda a=a, b=b, v=v: G.matmul4(a, b, variant=v)) for v in variants}
            if kind == "fwd":
                fns["old"] = lambda a=a, b=b: G.gemm_nt(a, w)
            elif G.matmul_layout(a, b) is not None:
                fns["old"] = lambda a=a, b=b: G.matmul_hip(a, b)
            fns["blas"] = lambda a=a, b=b: torch.matmul(a, b)
            ts = {k: [] for k in fns}
            for _ in range(args.rounds):
                for k, f in fns.items():
                    ts[k].append(timeit(f, args.iters))
            mm, nn_, kk = a.shape[0], b.shape[1], a.shape[1]
            flops = 2 * mm * nn_ * kk
            r = {k: round(flops / (min(v) * 1e-3) / 1e12) for k, v in ts.items()}
            r["us_best_g4"] = round(min(min(ts[f"g4v{v}"]) for v in variants) * 1e3, 1)
            r["us_blas"] = round(min(ts["blas"]) * 1e3, 1)
            key = f"{kind} M{mm} N{nn_} K{kk}"
            perf[key] = r
            print(key, r, file=sys.stderr, flush=True)
        del x, w, dy
    res["tflops"] = perf
    print(json.dumps(res))


if __name__ == "__main__":
    main()
