"""Forward A/B of the LDS-DMA ring kernel (csrc/attention_fwd_d256.hip) against the generic kernel
(csrc/attention_fwd.hip) at the Gemma-7B shape (D 256), causal and full.

    python scripts/attn_fwd_ring_ab.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops._lib import require
from lightning_thunder_amd.ops.attention import attn_fwd


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n * 1000


lib = require()
for name, (B, H, T, D) in {"gemma-7b": (1, 16, 4096, 256)}.items():
    q, k, v = (torch.randn(B, H, T, D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    for causal in (True, False):
        fl = 4 * B * H * T * T * D / (2 if causal else 1)
        res = {}
        for ring in (0, 1):
            lib.lta_attn_fwd_set_ring(ring)
            res[ring] = (attn_fwd(q, k, v, causal), timeit(lambda: attn_fwd(q, k, v, causal)))
        (o0, l0), t0 = res[0]
        (o1, l1), t1 = res[1]
        print(f"{name} D={D} {'causal' if causal else 'full'}: generic {t0:.1f} us ({fl / t0 / 1e6:.0f} TF/s), "
              f"ring {t1:.1f} us ({fl / t1 / 1e6:.0f} TF/s); max|dO| {(o0.float() - o1.float()).abs().max().item():.2e} "
              f"max|dLSE| {(l0 - l1).abs().max().item():.2e}", flush=True)
lib.lta_attn_fwd_set_ring(1)
