"""Dumps which ops of the GPT-2-medium training step still run as ATen (torch executor) vs HIP."""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.models.nanogpt import NanoGPT

B, T = 8, 1024
m = NanoGPT.from_name("gpt2-medium", seq_len=T).to(device="cuda", dtype=torch.bfloat16)
jm = thunder.jit(m)
x = torch.randint(0, m.config.vocab_size, (B, T), device="cuda")
y = torch.randint(0, m.config.vocab_size, (B, T), device="cuda")
_, loss = jm(x, y)
loss.backward()
for name, tr in (("forward", thunder.last_traces(jm)[-1]), ("backward", thunder.last_backward_traces(jm)[-1])):
    c = collections.Counter()
    for b in tr.bound_symbols:
        ex = getattr(b.sym, "executor", None)
        c[(getattr(ex, "name", str(ex)), b.sym.name)] += 1
    print(f"== {name}")
    for (ex, n), k in sorted(c.items(), key=lambda kv: -kv[1]):
        if n in ("python_del", "python_return", "unpack_trivial", "unpack_sequence"):
            continue
        print(f"{k:5d}  {ex:10s} {n}")
    open(f"gpurun_out/gpt2_{name}_trace.txt", "w").write(str(tr))
