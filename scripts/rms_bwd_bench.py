"""RMSNorm backward (with the residual gradient) on the Llama-2-7B step shape, us per call."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops.rmsnorm import rms_norm_fwd, rms_norm_bwd

res = {}
x = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
w = torch.randn(4096, device="cuda", dtype=torch.bfloat16)
dy = torch.randn_like(x)
r = torch.randn_like(x)
_, rstd = rms_norm_fwd(x, w, 1e-5)
for nb in (256, 512, 768, 1024, 2048):
    os.environ["LTA_RMS_BWD_BLOCKS"] = str(nb)
    for _ in range(5):
        rms_norm_bwd(dy, x, w, rstd, r)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(50):
        rms_norm_bwd(dy, x, w, rstd, r)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 50 * 1000
    res[nb] = {"us": round(us, 1), "TB_s": round(4 * 4096 * 4096 * 2 / us / 1e6, 2)}
    print(nb, res[nb], flush=True)
json.dump(res, open("gpurun_out/rms_bwd_bench.json", "w"), indent=1)
