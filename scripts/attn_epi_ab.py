"""A/B of the v4 attention forward epilogue on one box: the in-tree library (LDS-staged whole-row stores)
against a standalone build of an earlier attention_fwd4.hip (per-lane row-strided stores), same inputs,
alternating batches.  Also checks that both write bit-identical O and LSE.

    python scripts/attn_epi_ab.py scripts/exp/old_fwd4.so
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops._lib import require, stream_ptr, dcode

SIG = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
       ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int,
       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]


def main():
    new = require().lta_attn_fwd_v4
    old = ctypes.CDLL(os.path.abspath(sys.argv[1]), mode=os.RTLD_NOW).lta_attn_fwd_v4
    for f in (new, old):
        f.argtypes = SIG
        f.restype = ctypes.c_int
    B, H, T, D = 1, 32, 4096, 128
    torch.manual_seed(0)
    q = torch.randn(B, H, T, D, device="cuda", dtype=torch.bfloat16)
    k, v = torch.randn_like(q), torch.randn_like(q)
    for causal in (1, 0):
        outs = {}
        for name, f in (("new", new), ("old", old)):
            o = torch.empty(B, T, H, D, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
            lse = torch.empty(B, H, T, device="cuda", dtype=torch.float32)
            st = (ctypes.c_int64 * 3)(*o.stride()[:3])
            outs[name] = (f, o, lse, st)

        def call(name):
            f, o, lse, st = outs[name]
            rc = f(dcode(q), q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(), B, H, H, T, T, D,
                   D ** -0.5, causal, ctypes.cast(st, ctypes.c_void_p), None, 1, stream_ptr(q.device))
            assert rc == 0, (name, rc)

        for name in outs:
            call(name)
        torch.cuda.synchronize()
        same = torch.equal(outs["new"][1], outs["old"][1]) and torch.equal(outs["new"][2], outs["old"][2])
        ts = {"new": [], "old": []}
        for rnd in range(8):
            for name in (("new", "old") if rnd % 2 == 0 else ("old", "new")):  # alternate the order (clock bias)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    call(name)
                e1.record()
                e1.synchronize()
                ts[name].append(e0.elapsed_time(e1) * 1e3 / 20)
        med = {n: sorted(v)[len(v) // 2] for n, v in ts.items()}
        fl = 4 * B * H * T * T * D / (2 if causal else 1)
        print(f"causal={causal}: new {med['new']:.1f} us ({fl / med['new'] / 1e6:.0f} TF/s)  old {med['old']:.1f} us "
              f"({fl / med['old'] / 1e6:.0f} TF/s)  identical={same}", flush=True)


if __name__ == "__main__":
    main()
