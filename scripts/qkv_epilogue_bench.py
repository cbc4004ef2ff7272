"""Attention input projection of Llama-2-7B (x [4096, 4096] . W_qkv [12288, 4096]^T): the plain GEMM vs the
GEMM with the RoPE split in its epilogue, bf16 (gemm4 EPI 3) and fp8 (gemm4_fp8 QKV); interleaved rounds in
one process, random data.  python scripts/qkv_epilogue_bench.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops import fp8
from lightning_thunder_amd.ops import gemm as G

T, K, nh, ng, D = 4096, 4096, 32, 32, 128
N = (nh + 2 * ng) * D
x = torch.randn(1, T, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) / K ** 0.5
pos = torch.arange(T, device="cuda", dtype=torch.float32)
inv = 1.0 / (10000 ** (torch.arange(0, D // 2, device="cuda", dtype=torch.float32) * 2 / D))
ang = torch.outer(pos, inv).repeat(1, 2)
cos, sin = ang.cos(), ang.sin()
qx, sx = fp8.quantize_rows(x)
qw, sw = fp8.quantize_rows(w)
cases = {
    "bf16 plain": lambda: G.linear(x, w),
    "bf16 qkv-rope": lambda: G.linear_qkv_rope(x, w, cos, sin, nh, ng, D, D),
    "fp8 plain": lambda: fp8.gemm(qx, qw, sx, sw, 0, 0, None, (1, T, N)),
    "fp8 qkv-rope": lambda: fp8.gemm_qkv_rope(qx, qw, sx, sw, (1, T, N), cos, sin, nh, ng, D, D),
}
res = {k: [] for k in cases}
for rnd in range(6):
    for name, fn in cases.items():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        if rnd:
            res[name].append(e0.elapsed_time(e1) * 1e3 / 20)
for name, v in res.items():
    v.sort()
    print(f"{name:16s} median {v[len(v) // 2]:7.1f} us  min {v[0]:7.1f} us  {2 * T * N * K / v[0] / 1e6:6.0f} TF/s",
          flush=True)
