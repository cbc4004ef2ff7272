"""Why a launch-bound training forward does or does not gain from HipGraphTransform: regions, replays,
per-call time (NanoGPT GPT-2 XL, batch 16 x 128).  python scripts/hipgraph_diag.py [gpt2-xl]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.models.nanogpt import NanoGPT
from lightning_thunder_amd.transforms.hipgraph import HipGraphTransform

name = sys.argv[1] if len(sys.argv) > 1 else "gpt2-xl"
torch.manual_seed(0)
m = NanoGPT.from_name(name).to(device="cuda", dtype=torch.bfloat16)
x = torch.randint(0, 255, (16, m.config.seq_len), device="cuda")
y = torch.randint(0, 255, (16, m.config.seq_len), device="cuda")
t = HipGraphTransform(donate_grads=True)
jm = thunder.jit(m, transforms=[t])
for _ in range(4):
    out = jm(x, y)
torch.cuda.synchronize()
tr = thunder.last_traces(jm)[-1]
names = [b.sym.name for b in tr.bound_symbols]
print("forward trace bsyms:", len(names), "graph regions:", sum(n.startswith("HipGraph") for n in names))
print("non-graph bsyms:", [n for n in names if not n.startswith("HipGraph")][:60])
out[1].backward()
for p in m.parameters():
    p.grad = None
bt = thunder.last_backward_traces(jm)[-1]
bn = [b.sym.name for b in bt.bound_symbols]
print("backward trace bsyms:", len(bn), "graph regions:", sum(n.startswith("HipGraph") for n in bn))
print("non-graph backward bsyms:", [n for n in bn if not n.startswith("HipGraph") and n != "python_del"][:60])
for r in t.runners:
    if r.captures:
        print(r.name, "captures", r.captures, "replays", r.replays, "inputs", len(next(iter(r.entries.values()))[0]))
for mode in ("no_grad", "grad"):
    ctx = torch.no_grad() if mode == "no_grad" else torch.enable_grad()
    with ctx:
        for _ in range(3):
            jm(x, y)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            out = jm(x, y)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    print(f"{mode}: host {1e3 * (t1 - t0) / 10:.2f} ms/call, wall {1e3 * (t2 - t0) / 10:.2f} ms/call")
for graphs in (True,):
    for _ in range(3):
        out = jm(x, y)
        out[1].backward()
        for p in m.parameters():
            p.grad = None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        out = jm(x, y)
        out[1].backward()
        for p in m.parameters():
            p.grad = None
    torch.cuda.synchronize()
    print(f"fwd+bwd with graphs: {1e3 * (time.perf_counter() - t0) / 5:.2f} ms/step")
import cProfile
import pstats

pr = cProfile.Profile()
pr.enable()
for _ in range(5):
    out = jm(x, y)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
