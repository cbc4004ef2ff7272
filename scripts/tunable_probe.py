"""Does a TunableOp-selected rocBLAS/hipBLASLt solution beat the default heuristic *as measured
back-to-back on random data* (the in-situ condition)?  Llama-2-7B GEMMs at M = 4096."""
import json
import sys

import torch
import torch.nn.functional as F


def t(fn, it=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


M = 4096
cases = {}
for N, K in ((11008, 4096), (4096, 11008), (12288, 4096), (4096, 4096), (32000, 4096)):
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    g = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    cases[f"fwd N{N} K{K}"] = (lambda x=x, w=w: F.linear(x, w), 2 * M * N * K)
    cases[f"dgrad N{N} K{K}"] = (lambda g=g, w=w: g @ w, 2 * M * N * K)
    cases[f"wgrad N{N} K{K}"] = (lambda g=g, x=x: g.t() @ x, 2 * M * N * K)

res = {}
for name, (fn, f) in cases.items():
    res[name] = {"default_tf": round(f / t(fn) / 1e6)}
torch.cuda.tunable.enable(True)
torch.cuda.tunable.tuning_enable(True)
torch.cuda.tunable.set_filename("gpurun_out/tunable_probe%d.csv")
torch.cuda.tunable.set_max_tuning_duration(200)
torch.cuda.tunable.set_rotating_buffer_size(256)
for name, (fn, f) in cases.items():
    fn()
torch.cuda.synchronize()
torch.cuda.tunable.tuning_enable(False)
for name, (fn, f) in cases.items():
    res[name]["tuned_tf"] = round(f / t(fn) / 1e6)
    print(name, res[name], flush=True)
torch.cuda.tunable.enable(False)
for name, (fn, f) in cases.items():
    res[name]["default_again_tf"] = round(f / t(fn) / 1e6)
    print(name, res[name], flush=True)
print(torch.cuda.tunable.get_results())
json.dump(res, open("gpurun_out/tunable_probe.json", "w"), indent=1)
