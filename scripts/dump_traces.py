"""Dump the forward/backward execution traces of the bench model (debug aid, GPU)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.models.litgpt import GPT, Config

out_dir = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/traces"
executors = sys.argv[2].split(",") if len(sys.argv) > 2 else None
os.makedirs(out_dir, exist_ok=True)
cfg = Config.from_name("Llama-2-7b-hf", n_layer=2)
m = GPT(cfg).cuda().to(torch.bfloat16)
m.set_rope_cache(4096, device="cuda")
V = cfg.padded_vocab_size


class TrainStep(torch.nn.Module):
    def __init__(self, m):
        super().__init__()
        self.m = m

    def forward(self, x, y):
        return torch.nn.functional.cross_entropy(self.m(x).reshape(-1, V), y.reshape(-1))


kw = {"executors": executors} if executors else {}
jm = thunder.jit(TrainStep(m), **kw)
x = torch.randint(0, cfg.vocab_size, (1, 4096), device="cuda")
loss = jm(x, x)
loss.backward()
with open(os.path.join(out_dir, "forward.py"), "w") as f:
    f.write(str(thunder.last_traces(jm)[-1]))
with open(os.path.join(out_dir, "backward.py"), "w") as f:
    f.write(str(thunder.last_backward_traces(jm)[-1]))
print("ok", loss.item())
