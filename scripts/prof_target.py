"""Run one benchmarks/targets.py benchmark's forward (or backward) N times for a kernel trace:
rocprofv3 --kernel-trace --stats -d gpurun_out/p -o run --output-format csv -- python scripts/prof_target.py nanogpt_gpt2xl thunder"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.benchmarks.targets import BENCHMARKS

name, executor = sys.argv[1], sys.argv[2]
phase = sys.argv[3] if len(sys.argv) > 3 else "forward"
fn, args, to_loss = BENCHMARKS[name].make("cuda")
if executor == "thunder":
    fn = thunder.jit(fn)
elif executor == "thunder+hipgraph":
    from lightning_thunder_amd.transforms.hipgraph import HipGraphTransform

    fn = thunder.jit(fn, transforms=[HipGraphTransform(donate_grads=True)])
params = list(fn.parameters()) if hasattr(fn, "parameters") else []
for _ in range(5):
    out = fn(*args)
    if phase == "backward":
        to_loss(out).backward()
        for p in params:
            p.grad = None
torch.cuda.synchronize()
for _ in range(10):
    out = fn(*args)
    if phase == "backward":
        to_loss(out).backward()
        for p in params:
            p.grad = None
torch.cuda.synchronize()
print("done", flush=True)
