"""Times the FP8 cast+transpose kernel on the Llama-2-7B activation / gradient / weight shapes."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops.fp8 import cast_transpose, amax_into, E4M3_MAX, E5M2_MAX

res = {}
for (R, C) in [(4096, 4096), (4096, 11008), (4096, 12288), (4096, 22016), (11008, 4096), (32000, 4096)]:
    x = torch.randn(R, C, device="cuda", dtype=torch.bfloat16)
    amax = torch.zeros((), device="cuda", dtype=torch.float32)
    amax_into(x, amax)
    for e5 in (False, True):
        fmax = E5M2_MAX if e5 else E4M3_MAX
        for _ in range(3):
            q, qt = cast_transpose(x, amax, fmax, None, e5)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            q, qt = cast_transpose(x, amax, fmax, None, e5)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 20 * 1000
        res[f"{R}x{C}_{'e5m2' if e5 else 'e4m3'}"] = {"us": round(us, 1), "TB_s": round(R * C * 4 / us / 1e6, 2)}
        print(R, C, e5, res[f"{R}x{C}_{'e5m2' if e5 else 'e4m3'}"], flush=True)
json.dump(res, open("gpurun_out/cast_transpose_bench.json", "w"), indent=1)
