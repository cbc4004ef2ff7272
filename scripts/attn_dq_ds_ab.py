"""A/B of the RoPE'd attention backward at the Llama-2-7B shape (B 1, 32 heads, T 4096, D 128,
causal): default (dK/dV kernel + dQ kernel recomputing S / P / dP) vs LTA_ATTN_DQ_FROM_DS=1 (dK/dV
kernel also stores dS^T, dQ = scale dS K streamed from it).  Interleaved rounds, best of 3 x 10 calls.

    python scripts/attn_dq_ds_ab.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.models.litgpt import build_rope_cache
from lightning_thunder_amd.ops.attention import attn_fwd, attn_bwd_rope


def main():
    torch.manual_seed(0)
    B, H, T, D = 1, 32, 4096, 128
    cos, sin = build_rope_cache(T, D, device="cuda")
    qkv = torch.randn(B, T, 3 * H * D, device="cuda", dtype=torch.bfloat16)
    q, k, v = (t.view(B, T, H, D).transpose(1, 2) for t in qkv.split(H * D, -1))
    do = torch.randn(B, T, H, D, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
    o, lse = attn_fwd(q, k, v, True)

    def run():
        return attn_bwd_rope(do, q, k, v, o, lse, True, None, cos, sin, H, H)

    res, outs = {"recompute": [], "from_ds": []}, {}
    for _ in range(3):
        for name, flag in (("recompute", "0"), ("from_ds", "1")):
            os.environ["LTA_ATTN_DQ_FROM_DS"] = flag
            outs[name] = run()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                run()
            e.record()
            torch.cuda.synchronize()
            res[name].append(s.elapsed_time(e) / 10 * 1e3)
    a, b = outs["recompute"].float(), outs["from_ds"].float()
    rel = ((a - b).norm() / a.norm()).item()
    for name, ts in res.items():
        print(f"{name}: {min(ts):.1f} us/call (all {[round(t, 1) for t in ts]})", flush=True)
    print(f"rel diff d(qkv) {rel:.3e}; dq cols {((a[..., :H*D] - b[..., :H*D]).norm() / a[..., :H*D].norm()).item():.3e}")


if __name__ == "__main__":
    main()
