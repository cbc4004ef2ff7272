"""Per-phase cycle stamps of the v4 forward (impl 15 = ABL 5 build): workgroup (0, 0), its 4 waves,
first 64 tiles; prints the median cycles of Ph1..Ph4 and the end-of-tile wait+barrier."""
import sys

import torch

sys.path.insert(0, ".")
from lightning_thunder_amd.ops._lib import require  # noqa: E402
from lightning_thunder_amd.ops.attention import attn_fwd  # noqa: E402

lib = require()
q = torch.randn(1, 32, 4096, 128, device="cuda", dtype=torch.bfloat16)
k, v = torch.randn_like(q), torch.randn_like(q)
for causal in (False, True):
    lib.lta_attn_fwd_set_impl(15)
    for _ in range(3):
        o, lse = attn_fwd(q, k, v, causal)
    torch.cuda.synchronize()
    st = lse.reshape(-1).view(torch.int64)[:4 * 64 * 6].view(4, 64, 6).cpu()
    names = ["Ph1 QK_A", "Ph2 PV_B", "Ph3 QK_B", "Ph4 PV_A", "wait+bar"]
    print("causal" if causal else "full")
    for w in range(4):
        d = (st[w, :, 1:] - st[w, :, :-1]).float()
        tot = (st[w, :, 5] - st[w, :, 0]).float()
        ok = tot > 0
        med = d[ok].median(0).values.tolist()
        print(f"  wave {w}: tiles {int(ok.sum())} median cycles " + " ".join(f"{n} {m:.0f}" for n, m in zip(names, med))
              + f"  tile {tot[ok].median().item():.0f}  (MFMA floor 2048)", flush=True)
lib.lta_attn_fwd_set_impl(10)
