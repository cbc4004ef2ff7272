"""MXFP4 kernel micro-benchmark: GEMM TF/s (random data) and decode GEMV weight bandwidth."""
import json
import sys

import torch

from lightning_thunder_amd.ops import mxfp4, fp8


def graph_time(fn, iters=50):
    """Kernel time without the Python launch overhead: `iters` calls captured in one graph."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


res = {"gemm": {}, "gemv": {}}
for M, N, K in [(4096, 4096, 4096), (4096, 11008, 4096), (8192, 8192, 8192)]:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    qa, sa = mxfp4.quantize(a)
    qb, sb = mxfp4.quantize(b)
    us = timeit(lambda: mxfp4.gemm_nt(qa, sa, qb, sb))
    q8a, s8a, _, _ = fp8.mx_quantize(a)
    q8b, s8b, _, _ = fp8.mx_quantize(b)
    us8 = timeit(lambda: fp8.gemm_nt_mx(q8a, s8a, q8b, s8b))
    usb = timeit(lambda: a @ b.T)
    f = 2 * M * N * K
    res["gemm"][f"{M}x{N}x{K}"] = {"mxfp4_us": round(us, 1), "mxfp4_tflops": round(f / us / 1e6),
                                   "mxfp8_tflops": round(f / us8 / 1e6), "bf16_hipblaslt_tflops": round(f / usb / 1e6)}
    print(M, N, K, res["gemm"][f"{M}x{N}x{K}"], flush=True)
for M, N, K in [(1, 2048, 2048), (1, 8192, 2048), (1, 2048, 8192), (1, 128256, 2048), (4, 8192, 2048)]:
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    q, s = mxfp4.quantize(w)
    us = graph_time(lambda: mxfp4.gemv(x, q, s))
    usb = graph_time(lambda: x @ w.T)
    nbytes = q.numel() + s.numel()
    res["gemv"][f"{M}x{N}x{K}"] = {"mxfp4_us": round(us, 1), "weight_GBps": round(nbytes / us / 1e3),
                                   "bf16_torch_us": round(usb, 1),
                                   "bf16_GBps": round(w.numel() * 2 / usb / 1e3)}
    print(M, N, K, res["gemv"][f"{M}x{N}x{K}"], flush=True)
json.dump(res, open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/mxfp4_bench.json", "w"), indent=1)
