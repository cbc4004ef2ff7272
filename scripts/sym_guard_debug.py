"""Prints where a symbolic-shape compile of a small LitGPT records value specializations (debug aid)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import traceback

import torch

import lightning_thunder_amd as thunder
import lightning_thunder_amd.core.symbolic as S
from lightning_thunder_amd.models.litgpt import GPT, init_weights

orig = S.ShapeEnv.record
seen = set()


def rec(self, expr, outcome):
    if not self._suspended and outcome and " == " in expr and expr.rstrip()[-1].isdigit():
        st = tuple((fr.filename.split("repo/")[-1], fr.lineno, fr.name) for fr in traceback.extract_stack(limit=14)[:-2]
                   if "lightning_thunder_amd" in fr.filename and "symbolic.py" not in fr.filename)
        if st[-4:] not in seen:
            seen.add(st[-4:])
            print("GUARD", expr)
            for x in st[-6:]:
                print("   ", x)
    return orig(self, expr, outcome)


S.ShapeEnv.record = rec
dev = torch.device(sys.argv[2] if len(sys.argv) > 2 else "cuda")
m = GPT.from_name(sys.argv[1] if len(sys.argv) > 1 else "llama2-like").to(device=dev, dtype=torch.bfloat16)
init_weights(m)
m.set_rope_cache(256, device=dev)
jm = thunder.jit(m, cache="symbolic values")
for T in (64, 128):
    out = jm(torch.randint(0, 320, (2, T), device=dev))
    out.float().sum().backward()
print("misses", thunder.cache_misses(jm), "hits", thunder.cache_hits(jm))
