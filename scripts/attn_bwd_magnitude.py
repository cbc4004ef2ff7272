"""Attention backward kernel time vs data magnitudes (rocprofv3 --stats per variant).

    LTA_VARIANT=base|dosmall|qksmall|both python scripts/attn_bwd_magnitude.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops.attention import attn_fwd, attn_bwd

var = os.environ.get("LTA_VARIANT", "base")
torch.manual_seed(0)
q = torch.randn(1, 32, 4096, 128, device="cuda", dtype=torch.bfloat16)
k, v = torch.randn_like(q), torch.randn_like(q)
do = torch.randn(1, 4096, 32, 128, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
if var in ("qksmall", "both"):
    q, k = q * 0.1, k * 0.1
if var in ("dosmall", "both"):
    do = do * 1e-6
o, lse = attn_fwd(q, k, v, True)
for _ in range(20):
    attn_bwd(do, q, k, v, o, lse, True)
torch.cuda.synchronize()
print("done", var)
