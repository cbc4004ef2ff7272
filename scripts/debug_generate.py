"""Per-step logits of generate(): thunder vs thunder+hipGraph (debugging aid)."""
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.models.litgpt import GPT, init_weights
from lightning_thunder_amd.transforms.hipgraph import HipGraphTransform


def run(transforms):
    torch.manual_seed(0)
    m = GPT.from_name("llama3-like", n_layer=2).to(device="cuda", dtype=torch.bfloat16)
    init_weights(m, std=0.2)
    m.requires_grad_(False)
    m.set_kv_cache(1, 64)
    jm = thunder.jit(m, transforms=transforms)
    torch.manual_seed(1)
    p = torch.randint(0, 300, (1, 8), device="cuda")
    outs = [jm(p, torch.arange(8, device="cuda")).clone()]
    nxt = outs[-1][:, -1].argmax(-1, keepdim=True)
    pos = torch.tensor([8], device="cuda")
    with torch.no_grad():
        for i in range(5):
            lg = jm(nxt, pos)
            outs.append(lg.clone())
            nxt = lg[:, -1].argmax(-1, keepdim=True)
            pos.add_(1)
    return outs, m


a, _ = run([])
b, m = run([HipGraphTransform()])
for i, (x, y) in enumerate(zip(a, b)):
    print(i, (x.float() - y.float()).abs().max().item(), x[:, -1].argmax().item(), y[:, -1].argmax().item())
