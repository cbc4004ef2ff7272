"""Phase stamps of the dK/dV v4 kernel (diagnostic build: LTA_KERNELS_SO=scripts/exp/lta_diag.so, built by
``python -m lightning_thunder_amd.ops.build --diag scripts/exp/lta_diag.so``): workgroup (0, 0), its 4
waves, first 64 query tiles; median cycles per phase.  Phases: A (S = Q K^T), B (dP = dO V^T + exp),
mask+pack, C (dV^T += dO^T P, dS), D (dK^T += Q^T dS), tile-end wait, barrier."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
assert os.environ.get("LTA_KERNELS_SO"), "run with LTA_KERNELS_SO=<diagnostic build>"
from lightning_thunder_amd.ops._lib import require  # noqa: E402
from lightning_thunder_amd.ops.attention import attn_fwd, attn_bwd  # noqa: E402

lib = require()
lib.lta_attn_bwd_set_stamps.argtypes = [ctypes.c_void_p]
lib.lta_attn_bwd_set_stamps.restype = ctypes.c_int
q = torch.randn(1, 32, 4096, 128, device="cuda", dtype=torch.bfloat16)
k, v, do = torch.randn_like(q), torch.randn_like(q), torch.randn_like(q)
names = ["A:S=QK^T", "B:dP+exp", "mask+pack", "C:dV+dS", "D:dK", "wait", "barrier"]
for causal in (True, False):
    o, lse = attn_fwd(q, k, v, causal)
    buf = torch.zeros(4 * 64 * 8, dtype=torch.int64, device="cuda")
    lib.lta_attn_bwd_set_stamps(buf.data_ptr())
    for _ in range(3):
        attn_bwd(do, q, k, v, o, lse, causal)
    torch.cuda.synchronize()
    lib.lta_attn_bwd_set_stamps(None)
    st = buf.view(4, 64, 8).cpu()
    print("causal" if causal else "full")
    for w in range(4):
        d = (st[w, :, 1:] - st[w, :, :-1]).float()
        tot = (st[w, 1:, 0] - st[w, :-1, 0]).float()
        ok = (st[w, :, 7] > 0)
        med = d[ok].median(0).values.tolist()
        print(f"  wave {w}: tiles {int(ok.sum())} median cycles " + " ".join(f"{n} {m:.0f}" for n, m in zip(names, med))
              + f"  tile {tot[ok[1:]].median().item():.0f}  (MFMA floor 64 x 32 = 2048)", flush=True)
