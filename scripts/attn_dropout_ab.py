"""Attention with dropout at the GPT-2-medium training shape (B8 H16 T1024 D64, causal, p = 0.1):
fwd and bwd per-call time of the loaded library (LTA_KERNELS_SO selects another build for A/B).

    python scripts/attn_dropout_ab.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops.attention import attn_fwd, attn_bwd


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


torch.manual_seed(0)
B, H, T, D = 8, 16, 1024, 64
q, k, v = (torch.randn(B, H, T, D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
do = torch.randn(B, H, T, D, device="cuda", dtype=torch.bfloat16)
kw = dict(dropout_p=0.1, seed=1234, offset=0)
o, lse = attn_fwd(q, k, v, True, **kw)
tf = timeit(lambda: attn_fwd(q, k, v, True, **kw))
tb = timeit(lambda: attn_bwd(do, q, k, v, o, lse, True, **kw))
dq, dk, dv = attn_bwd(do, q, k, v, o, lse, True, **kw)
lib = os.environ.get("LTA_KERNELS_SO", "default")
print(f"[{os.path.basename(lib)}] dropout attention D=64: fwd {tf:.1f} us, bwd {tb:.1f} us; "
      f"checksums o {o.float().abs().sum().item():.6e} dq {dq.float().abs().sum().item():.6e} "
      f"dk {dk.float().abs().sum().item():.6e}", flush=True)
