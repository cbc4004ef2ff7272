"""dQ v3 / v4 (256 queries per workgroup, LDS-DMA K/V ring; v4 with the VALU in the MFMA shadows)
vs v2: numerics on odd shapes and timing at the Llama-2-7B shape.

    python scripts/attn_dq_v3_check.py
Prints per case the max |vN - v2| of dQ/dK/dV (v3: same arithmetic in the same key order, ~0;
v4 starts the dP chain at -delta, so it differs by rounding) and the fp32-reference error; then
the backward time (preprocess + dK/dV + dQ) per implementation, median of interleaved rounds.
"""
import ctypes
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops._lib import require
from lightning_thunder_amd.ops.attention import attn_fwd, attn_bwd

lib = require()
lib.lta_attn_bwd_set_dq_impl.argtypes = [ctypes.c_int]
lib.lta_attn_bwd_set_dq_impl.restype = ctypes.c_int


def run(impl, *a):
    lib.lta_attn_bwd_set_dq_impl(impl)
    return attn_bwd(*a)


def ref_bwd(do, q, k, v, causal):
    qf, kf, vf, dof = (t.float().requires_grad_(t is not do) for t in (q, k, v, do))
    g = q.shape[1] // k.shape[1]
    ke, ve = kf.repeat_interleave(g, 1), vf.repeat_interleave(g, 1)
    s = qf @ ke.transpose(-1, -2) / math.sqrt(q.shape[-1])
    if causal:
        T, S = s.shape[-2:]
        s = s.masked_fill(torch.ones(T, S, dtype=torch.bool, device=s.device).triu(S - T + 1), float("-inf"))
    o = torch.softmax(s, -1) @ ve
    return torch.autograd.grad(o, (qf, kf, vf), dof)


torch.manual_seed(0)
bad = False
for (B, Hq, Hkv, T, causal) in [(1, 4, 4, 1024, True), (2, 8, 2, 1000, True), (1, 2, 2, 300, False), (1, 4, 4, 77, True),
                               (1, 2, 1, 520, False), (1, 4, 4, 4096, True), (1, 2, 2, 600, False)]:
    q = torch.randn(B, Hq, T, 128, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, Hkv, T, 128, device="cuda", dtype=torch.bfloat16)
    v = torch.randn_like(k)
    do = torch.randn_like(q)
    o, lse = attn_fwd(q, k, v, causal)
    g2 = run(1, do, q, k, v, o, lse, causal)  # v2
    r = ref_bwd(do, q, k, v, causal)
    for impl in (2, 3):
        gn = run(impl, do, q, k, v, o, lse, causal)
        d = [(a.float() - b.float()).abs().max().item() for a, b in zip(g2, gn)]
        e = [((a.float() - b).abs().max() / b.abs().max()).item() for a, b in zip(gn, r)]
        ok = max(d) < 2e-2 and max(e) < 2e-2 and all(torch.isfinite(t).all() for t in gn)
        bad |= not ok
        print(f"B{B} H{Hq}/{Hkv} T{T} {'causal' if causal else 'full'}: |v{impl + 1}-v2| {['%.2e' % x for x in d]} "
              f"rel err vs fp32 {['%.2e' % x for x in e]} {'ok' if ok else 'BAD'}", flush=True)

q = torch.randn(1, 32, 4096, 128, device="cuda", dtype=torch.bfloat16)
k, v = torch.randn_like(q), torch.randn_like(q)
do = torch.randn(1, 4096, 32, 128, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
for causal in (True, False):
    o, lse = attn_fwd(q, k, v, causal)
    times = {1: [], 2: [], 3: []}
    for _ in range(3):
        for impl in (1, 2, 3):
            for _ in range(3):
                run(impl, do, q, k, v, o, lse, causal)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                run(impl, do, q, k, v, o, lse, causal)
            e.record()
            e.synchronize()
            times[impl].append(s.elapsed_time(e) / 10 * 1000)
    fl = 2.5 * 4 * 4096 * 4096 * 128 * 32 / (2 if causal else 1)
    for impl in (1, 2, 3):
        us = sorted(times[impl])[1]
        print(f"{'causal' if causal else 'full'} dq v{impl + 1}: bwd {us:.1f} us  {fl / us / 1e6:.0f} TF/s nominal", flush=True)
lib.lta_attn_bwd_set_dq_impl(1)
print("NUMERICS_FAIL" if bad else "NUMERICS_OK")
