"""Timing of the v4 forward ablation builds (impl 10 = full kernel; 11 no loop DMA, 12 no softmax
finish, 13 no per-tile barrier, 14 no softmax start) at the Llama-2-7B causal shape, interleaved."""
import sys

import torch

sys.path.insert(0, ".")
from lightning_thunder_amd.ops._lib import require  # noqa: E402
from lightning_thunder_amd.ops.attention import attn_fwd  # noqa: E402

lib = require()
IMPLS = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else "0,10,11,12,13,14".split(","))]
q = torch.randn(1, 32, 4096, 128, device="cuda", dtype=torch.bfloat16)
k, v = torch.randn_like(q), torch.randn_like(q)
for causal in (True, False):
    fl = 4 * 32 * 4096 * 4096 * 128 / (2 if causal else 1)
    times = {i: [] for i in IMPLS}
    for rnd in range(5):
        for impl in IMPLS:
            lib.lta_attn_fwd_set_impl(impl)
            attn_fwd(q, k, v, causal)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                attn_fwd(q, k, v, causal)
            e.record()
            torch.cuda.synchronize()
            times[impl].append(s.elapsed_time(e) / 10)
    for impl in IMPLS:
        ms = sorted(times[impl])[2]
        print(f"{'causal' if causal else 'full'} impl{impl}: {ms * 1000:.1f} us  {fl / ms / 1e9:.0f} TF/s", flush=True)
lib.lta_attn_fwd_set_impl(0)
