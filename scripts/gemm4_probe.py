"""gemm4 forward (K-major) probe: is the K-major path limited by the power-of-two row pitch?

Times the same 4096^3 product with operands at pitch K (8 KiB rows) and at padded pitches, plus
the dgrad (MN-major B) layout for comparison.  Interleaved rounds; prints TF/s per arm.
"""
import argparse
import json

import torch

from lightning_thunder_amd.ops.gemm import matmul4


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    M = N = K = 4096
    flop = 2 * M * N * K
    g = torch.Generator(device="cuda").manual_seed(0)

    def padded(rows, cols, pad):
        t = torch.randn(rows, cols + pad, device="cuda", generator=g).to(torch.bfloat16)
        return t[:, :cols]

    arms = {}
    for pad in (0, 64, 128, 256):
        x, w = padded(M, K, pad), padded(N, K, pad)
        arms[f"fwd_pad{pad}"] = (lambda x=x, w=w: matmul4(x, w.t(), variant=1))
    dy = padded(M, N, 0)
    wt = padded(N, K, 0)
    arms["dgrad"] = lambda: matmul4(dy, wt, variant=1)
    res = {k: [] for k in arms}
    for _ in range(args.rounds):
        for k, fn in arms.items():
            res[k].append(flop / timed(fn, args.iters) / 1e9)
    out = {k: round(max(v)) for k, v in res.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
