"""Attention backward at the Llama-2-7B shape with cache-resident vs cold inputs.

    python scripts/attn_bwd_cold.py
'warm' repeats the backward on one input set (q, k, v, o, dO stay in L2 / the 256 MB MALL);
'cold' cycles through 8 input sets (1.6 GB), so each backward starts from HBM as in a training
step, where the inputs were written long before.  Per-kernel times from rocprofv3 separate the
dK/dV and dQ kernels; this script reports the whole backward (median of rounds).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops.attention import attn_fwd, attn_bwd


def make():
    q = torch.randn(1, 32, 4096, 128, device="cuda", dtype=torch.bfloat16)
    k, v = torch.randn_like(q), torch.randn_like(q)
    do = torch.randn(1, 4096, 32, 128, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
    o, lse = attn_fwd(q, k, v, True)
    return do, q, k, v, o, lse


sets = [make() for _ in range(8)]
torch.cuda.synchronize()


def timed(seq):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for a in seq:
        attn_bwd(*a, True)
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / len(seq) * 1000


for _ in range(3):
    timed(sets)
warm, cold = [], []
for _ in range(5):
    warm.append(timed([sets[0]] * 8))
    cold.append(timed(sets))
print(f"causal backward per layer: warm {sorted(warm)[2]:.1f} us, cold {sorted(cold)[2]:.1f} us", flush=True)

# the same backward between large GEMMs (as in the training step, where the chip's clock is set by
# the GEMM-heavy load around the attention kernels)
a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
b = torch.randn(11008, 4096, device="cuda", dtype=torch.bfloat16)
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(8)]
mixed = []
for _ in range(5):
    for i, (s, e) in enumerate(ev):
        for _ in range(6):
            torch.nn.functional.linear(a, b)
        s.record()
        attn_bwd(*sets[i], True)
        e.record()
    torch.cuda.synchronize()
    mixed.append(sorted(s.elapsed_time(e) * 1000 for s, e in ev)[4])
print(f"causal backward per layer between GEMMs: {sorted(mixed)[2]:.1f} us", flush=True)

# training-step-like magnitudes: tiny upstream gradients (dO ~ 1e-6) and small scores
small = []
for do, q, k, v, o, lse in sets[:2]:
    qs, ks = q * 0.1, k * 0.1
    os_, ls = attn_fwd(qs, ks, v, True)
    small.append((do * 1e-6, qs, ks, v, os_, ls))
ts = []
for _ in range(5):
    ts.append(timed(small * 4))
print(f"causal backward per layer, small dO / scores: {sorted(ts)[2]:.1f} us", flush=True)
