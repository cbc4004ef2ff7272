"""Backward GEMM shapes of the Llama-2-7B step (M = 4096 tokens): hipBLASLt dgrad / wgrad vs the
hand-written kernel reading the transposed operands in place (MN-major LDS images, transposing
LDS reads) (random data, interleaved rounds)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops.gemm import gemm_nt, matmul_hip

LINEARS = [(12288, 4096), (4096, 4096), (11008, 4096), (4096, 11008), (32000, 4096)]
M = 4096


def timeit(fn, iters=30):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


out = {}
for N, K in LINEARS:
    x = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    w = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    dy = torch.empty(M, N, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
    fns = {
        "fwd_blas": lambda: torch.nn.functional.linear(x, w),
        "fwd_hip": lambda: gemm_nt(x, w),
        "dgrad_blas": lambda: dy @ w,
        "dgrad_hip": lambda: matmul_hip(dy, w),
        "wgrad_blas": lambda: dy.t() @ x,
        "wgrad_hip": lambda: matmul_hip(dy.t(), x),
    }
    ref = (dy.t().float() @ x.float())
    err = ((matmul_hip(dy.t(), x).float() - ref).abs().max() / ref.abs().max()).item()
    err_d = ((matmul_hip(dy, w).float() - dy.float() @ w.float()).abs().max()).item()
    ts = {k: [] for k in fns}
    for _ in range(3):
        for k, f in fns.items():
            ts[k].append(timeit(f))
    flops = 2 * M * N * K
    r = {k: round(min(v) * 1000, 1) for k, v in ts.items()}  # us
    r.update({k.replace("blas", "blas_tf").replace("hip", "hip_tf"): round(flops / (min(ts[k]) * 1e-3) / 1e12)
              for k in ("fwd_blas", "fwd_hip", "dgrad_blas", "wgrad_blas", "dgrad_hip", "wgrad_hip")})
    r["wgrad_hip_rel_err"] = err
    r["dgrad_hip_abs_err"] = err_d
    out[f"N{N}_K{K}"] = r
    print(f"N={N} K={K}: {r}", file=sys.stderr, flush=True)
print(json.dumps({"llama2_7b_gemm_us_M4096": out}))
