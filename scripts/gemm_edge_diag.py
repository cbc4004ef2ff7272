"""Edge-tile GEMM epilogue diagnostic: max error per (bias, act) combination and the tile map of
the wrong outputs (rows / columns blocks of 256)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops.gemm import linear

torch.manual_seed(1)
K = 512
for (M, N) in [(1000, 16032), (300, 50304), (1024, 16128), (1000, 4096), (1024, 16032)]:
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) / K ** 0.5
    bias = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    for use_bias in (False, True):
        for act in (None, "gelu_tanh"):
            y = linear(x, w, bias if use_bias else None, act=act)
            ref = x.float() @ w.float().t() + (bias.float() if use_bias else 0)
            if act:
                ref = torch.nn.functional.gelu(ref, approximate="tanh")
            err = (y.float() - ref).abs()
            bad = (err > 5e-2).nonzero()
            tiles = sorted({(int(r) // 256, int(c) // 256) for r, c in bad[:2000].tolist()})
            print(f"M={M} N={N} bias={use_bias} act={act}: max err {err.max().item():.3g}, bad {bad.shape[0]}, "
                  f"tiles {tiles[:12]}", flush=True)
