"""Runs one forward attention kernel variant a few times at the Llama-2-7B shape (PMC profiling):
``python scripts/attn_fwd_only.py IMPL [N] [CAUSAL]`` (IMPL as lta_attn_fwd_set_impl)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops._lib import require
from lightning_thunder_amd.ops.attention import attn_fwd

require().lta_attn_fwd_set_impl(int(sys.argv[1]))
q = torch.randn(1, 32, 4096, 128, device="cuda", dtype=torch.bfloat16)
k, v = torch.randn_like(q), torch.randn_like(q)
causal = (sys.argv[3] != "0") if len(sys.argv) > 3 else True
for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 3):
    attn_fwd(q, k, v, causal)
torch.cuda.synchronize()
print("done")
