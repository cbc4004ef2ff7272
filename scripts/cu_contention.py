"""What an overlapped collective's resident workgroups cost the compute stream.

At world size 8 every RCCL channel is one workgroup resident on a CU for the whole collective, and
the FSDP / DDP collectives run concurrently with the backward's GEMMs (high-priority stream, waits
sorted late).  The GEMMs are sized one 256x256 tile per CU, so a CU taken by a channel can turn a
one-wave GEMM into two.  One GPU cannot run a multi-rank collective, but it can run the same
*occupancy*: ``lta_cu_occupy`` (ops/csrc/probe.hip) keeps N workgroups of a given shape resident on a
high-priority stream for a fixed time while the compute stream runs the Llama-2-7B GEMM shapes and the
whole training step.  Output: one JSON line per (N, program) with the slowdown vs N = 0.

    python scripts/cu_contention.py [--threads 256] [--lds 0] [--n 0,8,16,32,64] [--step]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def occupier():
    from lightning_thunder_amd.ops._lib import require, register_signature, c_int, c_void_p

    register_signature("lta_cu_occupy", [c_int, c_int, c_int, ctypes.c_uint64, c_void_p])
    lib = require()
    hi = torch.cuda.Stream(priority=-1)

    def occupy(n: int, threads: int, lds: int, seconds: float):
        if n <= 0:
            return
        rc = lib.lta_cu_occupy(n, threads, lds, int(seconds * 1e8), ctypes.c_void_p(hi.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"lta_cu_occupy failed: {rc}")

    return occupy, hi


def time_gemms(reps: int = 20):
    from lightning_thunder_amd.ops.gemm import linear

    dev = torch.device("cuda")
    M = 4096
    shapes = {"qkv 4096x12288x4096": (4096, 12288), "o-proj 4096x4096x4096": (4096, 4096),
              "fc 4096x11008x4096": (4096, 11008), "mlp-proj 4096x4096x11008": (11008, 4096)}
    out = {}
    for name, (K, N) in shapes.items():
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            linear(x, w)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            linear(x, w)
        e.record()
        e.synchronize()
        out[name] = s.elapsed_time(e) / reps * 1000.0  # us
    return out


def build_step(n_layer=None):
    import lightning_thunder_amd as thunder
    from lightning_thunder_amd.models.litgpt import GPT, Config, init_weights
    from lightning_thunder_amd.optim import AdamW

    dev = torch.device("cuda")
    cfg = Config.from_name("Llama-2-7b-hf", **({} if n_layer is None else {"n_layer": n_layer}))
    with torch.device("meta"):
        m = GPT(cfg)
    m = m.to_empty(device=dev).to(torch.bfloat16)
    torch.manual_seed(0)
    init_weights(m)
    m.set_rope_cache(4096, device=dev)
    V = cfg.padded_vocab_size

    class TS(torch.nn.Module):
        def __init__(self, mm):
            super().__init__()
            self.m = mm

        def forward(self, x, y):
            return torch.nn.functional.cross_entropy(self.m(x).reshape(-1, V), y.reshape(-1))

    jm = thunder.jit(TS(m))
    opt = AdamW([p for p in m.parameters()], lr=1e-4, betas=(0.9, 0.95), weight_decay=0.1)
    x = torch.randint(0, cfg.vocab_size, (1, 4097), device=dev)
    a, b = x[:, :-1].contiguous(), x[:, 1:].contiguous()

    def step():
        jm(a, b).backward()
        opt.step()
        opt.zero_grad(set_to_none=True)

    return step


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--threads", type=int, default=256)
    p.add_argument("--lds", type=int, default=0, help="dynamic LDS bytes per occupying workgroup")
    p.add_argument("--n", default="0,8,16,32,64")
    p.add_argument("--step", action="store_true", help="also time the whole Llama-2-7B training step")
    p.add_argument("--steps", type=int, default=3)
    a = p.parse_args()
    occupy, hi = occupier()
    ns = [int(v) for v in a.n.split(",")]
    base = None
    for n in ns:
        torch.cuda.synchronize()
        occupy(n, a.threads, a.lds, 0.5)
        time.sleep(0.005)  # the occupying workgroups are resident before the GEMMs are issued
        g = time_gemms()
        torch.cuda.synchronize()
        if base is None:
            base = g
        print(json.dumps({"program": "gemms", "occupied_wg": n, "threads": a.threads, "lds": a.lds,
                          "us": {k: round(v, 1) for k, v in g.items()},
                          "slowdown": {k: round(v / base[k], 3) for k, v in g.items()}}), flush=True)
    if a.step:
        step = build_step()
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        sbase = None
        for n in ns:
            torch.cuda.synchronize()
            occupy(n, a.threads, a.lds, 0.3 * a.steps + 0.3)
            time.sleep(0.005)
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step()
            torch.cuda.current_stream().synchronize()  # not the occupier's stream: it outlives the steps
            ms = (time.perf_counter() - t0) / a.steps * 1000
            sbase = sbase or ms
            print(json.dumps({"program": "llama2-7b step", "occupied_wg": n, "threads": a.threads, "lds": a.lds,
                              "ms": round(ms, 2), "slowdown": round(ms / sbase, 3)}), flush=True)


if __name__ == "__main__":
    main()
