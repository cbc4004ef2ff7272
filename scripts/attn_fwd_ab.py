"""A/B of the flash-attention forward kernels (impl 0 = v1 4-wave x 2 WG/CU; 1..4 = v2 8-wave
variants: one S tile / att[2] pipeline x exact / deferred rescale) at the Llama-2-7B shape, plus
numerics of every variant against an fp32 reference on small and ragged shapes."""
import json
import math
import sys

import torch

sys.path.insert(0, ".")
from lightning_thunder_amd.ops._lib import require  # noqa: E402
from lightning_thunder_amd.ops.attention import attn_fwd  # noqa: E402

lib = require()
IMPLS = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else "0,1,2,3,4".split(","))]


def ref(q, k, v, causal):
    qf, kf, vf = q.float(), k.float(), v.float()
    g = q.shape[1] // k.shape[1]
    kf, vf = kf.repeat_interleave(g, 1), vf.repeat_interleave(g, 1)
    s = qf @ kf.transpose(-1, -2) / math.sqrt(q.shape[-1])
    if causal:
        T, S = s.shape[-2:]
        s = s.masked_fill(torch.ones(T, S, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
    return torch.softmax(s, -1) @ vf, torch.logsumexp(s, -1)


out = {"numerics": {}, "perf": {}}
torch.manual_seed(0)
for (B, Hq, Hkv, T, S) in [(1, 4, 4, 1024, 1024), (2, 8, 2, 1000, 1000), (1, 2, 1, 77, 77), (1, 4, 4, 300, 700)]:
    q = torch.randn(B, Hq, T, 128, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, Hkv, S, 128, device="cuda", dtype=torch.bfloat16)
    v = torch.randn_like(k)
    for causal in ((False, True) if T == S else (False,)):
        ro, rl = ref(q, k, v, causal)
        for impl in IMPLS:
            lib.lta_attn_fwd_set_impl(impl)
            o, lse = attn_fwd(q, k, v, causal)
            torch.cuda.synchronize()
            key = f"B{B}_H{Hq}/{Hkv}_T{T}_S{S}_{'causal' if causal else 'full'}_impl{impl}"
            out["numerics"][key] = [float((o.float() - ro).abs().max()), float((lse - rl).abs().max())]
            print(key, out["numerics"][key], flush=True)

B, H, T, D = 1, 32, 4096, 128
q = torch.randn(B, H, T, D, device="cuda", dtype=torch.bfloat16)
k, v = torch.randn_like(q), torch.randn_like(q)
for causal in (True, False):
    fl = 4 * B * H * T * T * D / (2 if causal else 1)
    base = None
    for impl in IMPLS:
        lib.lta_attn_fwd_set_impl(impl)
        for _ in range(3):
            o, lse = attn_fwd(q, k, v, causal)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            o, lse = attn_fwd(q, k, v, causal)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 20
        if base is None:
            base = (o.float(), lse)
        d = float((o.float() - base[0]).abs().max())
        key = f"{'causal' if causal else 'full'}_impl{impl}"
        out["perf"][key] = {"us": round(ms * 1000, 1), "tflops": round(fl / ms / 1e9, 1), "max_diff_vs_first": d}
        print(key, out["perf"][key], flush=True)
lib.lta_attn_fwd_set_impl(0)
json.dump(out, open("gpurun_out/attn_fwd_ab.json", "w"), indent=1)

# ---- backward: dQ kernel v1 vs v2 ---------------------------------------------------------------
from lightning_thunder_amd.ops.attention import attn_bwd  # noqa: E402

if "fwd" in sys.argv[2:]:
    json.dump(out, open("gpurun_out/attn_fwd_ab.json", "w"), indent=1)
    sys.exit(0)

out["bwd_numerics"], out["bwd_perf"] = {}, {}
torch.manual_seed(1)
for (B, Hq, Hkv, T) in [(1, 4, 4, 1024), (2, 8, 2, 1000), (1, 2, 1, 77)]:
    for causal in (False, True):
        q = torch.randn(B, Hq, T, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        k = torch.randn(B, Hkv, T, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        v = torch.randn(B, Hkv, T, 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        do = torch.randn(B, Hq, T, 128, device="cuda", dtype=torch.bfloat16)
        ro, _ = ref(q, k, v, causal)
        rdq, rdk, rdv = torch.autograd.grad(ro, (q, k, v), do.float())
        lib.lta_attn_fwd_set_impl(0)
        o, lse = attn_fwd(q.detach(), k.detach(), v.detach(), causal)
        for impl in (0, 1, 2):
            lib.lta_attn_bwd_set_dq_impl(min(impl, 1))
            lib.lta_attn_bwd_set_dkdv_impl(1 if impl == 2 else 0)
            dq, dk, dv = attn_bwd(do, q.detach(), k.detach(), v.detach(), o, lse, causal)
            torch.cuda.synchronize()
            key = f"B{B}_H{Hq}/{Hkv}_T{T}_{'causal' if causal else 'full'}_dq{impl}"
            rel = lambda a, b: float((a.float() - b).norm() / b.norm())  # noqa: E731
            out["bwd_numerics"][key] = [rel(dq, rdq), rel(dk, rdk), rel(dv, rdv)]
            print(key, out["bwd_numerics"][key], flush=True)

B, H, T, D = 1, 32, 4096, 128
q = torch.randn(B, H, T, D, device="cuda", dtype=torch.bfloat16)
k, v = torch.randn_like(q), torch.randn_like(q)
do = torch.randn(B, T, H, D, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
lib.lta_attn_fwd_set_impl(0)
o, lse = attn_fwd(q, k, v, True)
for impl in (0, 1, 2, 0, 1, 2):
    lib.lta_attn_bwd_set_dq_impl(min(impl, 1))
    lib.lta_attn_bwd_set_dkdv_impl(1 if impl == 2 else 0)
    for _ in range(3):
        attn_bwd(do, q, k, v, o, lse, True)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        dq, dk, dv = attn_bwd(do, q, k, v, o, lse, True)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 20
    fl = 2.5 * 4 * B * H * T * T * D / 2
    out["bwd_perf"][f"causal_dq{impl}"] = {"us": round(ms * 1000, 1), "tflops_nominal": round(fl / ms / 1e9, 1),
                                           "dq_abs_sum": float(dq.float().abs().sum())}
    print("bwd", impl, out["bwd_perf"][f"causal_dq{impl}"], flush=True)
lib.lta_attn_bwd_set_dq_impl(0)
lib.lta_attn_bwd_set_dkdv_impl(0)
json.dump(out, open("gpurun_out/attn_fwd_ab.json", "w"), indent=1)
