"""generate() under HipGraphTransform: which prior activity on the model changes the first decode step?"""
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.models.litgpt import GPT, init_weights, generate
from lightning_thunder_amd.transforms.hipgraph import HipGraphTransform


def fresh():
    torch.manual_seed(0)
    m = GPT.from_name("llama3-like", n_layer=2).to(device="cuda", dtype=torch.bfloat16)
    init_weights(m, std=0.2)
    m.requires_grad_(False)
    return m


torch.manual_seed(0)
p = torch.randint(0, 300, (1, 8), device="cuda")


def run(m, transforms):
    m.set_kv_cache(1, 64)
    jm = thunder.jit(m, transforms=transforms)
    return generate(m, p, 6, forward=jm)[0, 8:].tolist(), generate(m, p, 6, forward=jm)[0, 8:].tolist()


m = fresh()
print("B fresh graph        ", run(m, [HipGraphTransform()]))
m = fresh()
print("C fresh nograph      ", run(m, []))
print("C then graph         ", run(m, [HipGraphTransform()]))
m = fresh()
m.set_kv_cache(1, 64)
print("A eager              ", generate(m, p, 6)[0, 8:].tolist())
print("A then graph         ", run(m, [HipGraphTransform()]))
m = fresh()
t = HipGraphTransform(copy_outputs=True)
print("D fresh graph copyout", run(m, [t]))
