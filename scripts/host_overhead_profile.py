"""Host-side cost of a jitted call: cProfile over repeated forward (and backward) calls of a small,
launch-bound model (NanoGPT GPT-2 124M, batch 16 x seq 128: benchmarks/targets.py nanogpt_gpt2),
plus wall time per call with and without a device sync.

    python scripts/host_overhead_profile.py [--top 45]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.models.nanogpt import NanoGPT


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--top", type=int, default=45)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--fwd-only", action="store_true", help="profile forward calls only")
    args = ap.parse_args()
    torch.manual_seed(0)
    m = NanoGPT.from_name(args.model).to(device="cuda", dtype=torch.bfloat16)
    x = torch.randint(0, 255, (16, m.config.seq_len), device="cuda")
    y = torch.randint(0, 255, (16, m.config.seq_len), device="cuda")
    jm = thunder.jit(m)
    for _ in range(5):
        out = jm(x, y)
        out[1].backward()
    torch.cuda.synchronize()
    # host time of the forward call alone (no sync inside the loop): launch-queue bound if > GPU time
    t0 = time.perf_counter()
    for _ in range(args.iters):
        out = jm(x, y)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"forward: host {1e3 * (t1 - t0) / args.iters:.3f} ms/call, host+drain {1e3 * (t2 - t0) / args.iters:.3f} ms/call")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.iters):
        out = jm(x, y)
        if not args.fwd_only:
            out[1].backward()
    pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    ps = pstats.Stats(pr, stream=s).sort_stats("tottime")
    ps.print_stats(args.top)
    print(s.getvalue())
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(args.top)
    print(s.getvalue())


if __name__ == "__main__":
    main()
