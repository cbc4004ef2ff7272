"""A/B of the dK/dV backward kernels (v1 register-staged vs v2 glds/dual-image/AGPR accumulators)
at the Llama-2-7B shape: runs each in a child process (the choice is read once per process)."""
import os
import subprocess
import sys

CHILD = r"""
import sys, torch
sys.path.insert(0, '.')
from lightning_thunder_amd.ops.attention import attn_fwd, attn_bwd
torch.manual_seed(0)
q = torch.randn(1, 32, 4096, 128, device='cuda', dtype=torch.bfloat16)
k, v = torch.randn_like(q), torch.randn_like(q)
do = torch.randn(1, 4096, 32, 128, device='cuda', dtype=torch.bfloat16).transpose(1, 2)
o, lse = attn_fwd(q, k, v, True)
for _ in range(3): attn_bwd(do, q, k, v, o, lse, True)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(20): dq, dk, dv = attn_bwd(do, q, k, v, o, lse, True)
e.record(); torch.cuda.synchronize()
ms = s.elapsed_time(e) / 20
fl = 2.5 * 4 * 4096 * 4096 * 128 * 32 / 2
print(f"{ms*1000:.1f} us/call  {fl/ms/1e9:.0f} TF/s  dk_sum={dk.float().abs().sum().item():.6e} dq_sum={dq.float().abs().sum().item():.6e}")
"""
for v1 in ("1", "0", "1", "0"):
    env = dict(os.environ, LTA_ATTN_BWD_V1=v1)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=240)
    print("v1" if v1 == "1" else "v2", r.stdout.strip(), r.stderr.strip()[-300:] if r.returncode else "", flush=True)
