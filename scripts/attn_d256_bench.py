"""D = 256 flash attention (Gemma-7B shape: 16 heads x 256, seq 4096, causal): hand kernels vs ATen SDPA.

    python scripts/attn_d256_bench.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops.attention import attn_fwd, attn_bwd


def timeit(fn, n=10):
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


B, H, T, D = 1, 16, 4096, 256
q, k, v = (torch.randn(B, H, T, D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
do = torch.randn_like(q)
from lightning_thunder_amd.ops._lib import require

lib = require()
for causal in (True, False):
    # generic kernel (the previous D = 256 path) for reference and A/B
    lib.lta_attn_fwd_set_ring(0)
    o0, lse0 = attn_fwd(q, k, v, causal)
    tf0 = timeit(lambda: attn_fwd(q, k, v, causal))
    lib.lta_attn_fwd_set_ring(1)
    o, lse = attn_fwd(q, k, v, causal)
    dmax = (o.float() - o0.float()).abs().max().item()
    dl = (lse - lse0).abs().max().item()
    fl = 4 * B * H * T * T * D / (2 if causal else 1)
    tf = timeit(lambda: attn_fwd(q, k, v, causal))
    tb = timeit(lambda: attn_bwd(do, q, k, v, o, lse, causal))
    qa, ka, va = (t.detach().requires_grad_(True) for t in (q, k, v))

    def aten_fb():
        y = torch.nn.functional.scaled_dot_product_attention(qa, ka, va, is_causal=causal)
        y.backward(do)

    ta_f = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=causal))
    ta_fb = timeit(aten_fb)
    print(f"{'causal' if causal else 'full'} D=256 generic fwd {tf0:.0f} us ({fl / tf0 / 1e6:.0f} TF/s); "
          f"ring kernel vs generic: max|dO| {dmax:.2e}, max|dLSE| {dl:.2e}", flush=True)
    print(f"{'causal' if causal else 'full'} D=256: fwd {tf:.0f} us ({fl / tf / 1e6:.0f} TF/s), bwd {tb:.0f} us "
          f"({2.5 * fl / tb / 1e6:.0f} TF/s); ATen SDPA fwd {ta_f:.0f} us, fwd+bwd {ta_fb:.0f} us vs ours {tf + tb:.0f} us",
          flush=True)
