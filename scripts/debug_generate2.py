"""Decode warm-up under HipGraphTransform: print the graphed decode trace and per-step logits diffs."""
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.models.litgpt import GPT, init_weights
from lightning_thunder_amd.transforms.hipgraph import HipGraphTransform


def steps(transforms):
    torch.manual_seed(0)
    m = GPT.from_name("llama3-like", n_layer=1).to(device="cuda", dtype=torch.bfloat16)
    init_weights(m, std=0.2)
    m.requires_grad_(False)
    m.set_kv_cache(1, 64)
    jm = thunder.jit(m, transforms=transforms)
    torch.manual_seed(1)
    p = torch.randint(0, 300, (1, 8), device="cuda")
    outs = []
    with torch.no_grad():
        lg = jm(p, torch.arange(8, device="cuda"))
        outs.append(lg.clone())
        pos = torch.tensor([8], device="cuda")
        nxt = lg[:, -1].argmax(-1, keepdim=True)
        for i in range(3):
            lg = jm(nxt, pos)
            outs.append(lg.clone())
            pos.add_(1)
            nxt = lg[:, -1].argmax(-1, keepdim=True)
    kc = m.transformer.h[0].attn.kv_cache.k.clone()
    return outs, kc, jm


a, ka, _ = steps([])
b, kb, jm = steps([HipGraphTransform()])
for i, (x, y) in enumerate(zip(a, b)):
    print("step", i, "max|diff| logits", (x.float() - y.float()).abs().max().item())
print("kv cache diff per position:", (ka.float() - kb.float()).abs().amax(dim=(0, 1, 3))[:12].tolist())
print(thunder.last_traces(jm)[-1])
