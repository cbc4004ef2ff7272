"""Fused AdamW: regular vs non-temporal streaming (A/B), Llama-2-7B-like parameter shapes
(8 transformer blocks' worth, ~1.6 B bf16 parameters, bf16 moments).  Median of interleaved rounds."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops._lib import require
from lightning_thunder_amd.optim import AdamW

lib = require()
lib.lta_adamw_set_nt.argtypes = [ctypes.c_int]
shapes = []
for _ in range(8):
    shapes += [(12288, 4096), (4096, 4096), (22016, 4096), (4096, 11008), (4096,), (4096,)]
ps = [torch.nn.Parameter(torch.randn(*s, device="cuda", dtype=torch.bfloat16) * 0.02) for s in shapes]
for p in ps:
    p.grad = torch.randn_like(p) * 1e-3
opt = AdamW(ps, lr=3e-4, betas=(0.9, 0.95), weight_decay=0.1)
n = sum(p.numel() for p in ps)
for _ in range(3):
    opt.step()
torch.cuda.synchronize()
res = {0: [], 1: []}
for rnd in range(5):
    for nt in (0, 1):
        lib.lta_adamw_set_nt(nt)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            opt.step()
        e1.record()
        e1.synchronize()
        res[nt].append(e0.elapsed_time(e1) / 5)
lib.lta_adamw_set_nt(0)
for nt in (0, 1):
    ms = sorted(res[nt])[2]
    print(f"nt={nt}: {ms:.3f} ms for {n / 1e9:.2f} B params, {14 * n / ms / 1e9:.2f} TB/s")
