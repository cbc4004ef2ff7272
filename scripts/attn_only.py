"""Runs the HIP attention fwd+bwd a few times at the Llama-2-7B shape (for PMC profiling)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops.attention import attn_fwd, attn_bwd

q = torch.randn(1, 32, 4096, 128, device="cuda", dtype=torch.bfloat16)
k, v, do = torch.randn_like(q), torch.randn_like(q), torch.randn_like(q)
o, lse = attn_fwd(q, k, v, True)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    attn_fwd(q, k, v, True)
    attn_bwd(do, q, k, v, o, lse, True)
torch.cuda.synchronize()
print("done")
