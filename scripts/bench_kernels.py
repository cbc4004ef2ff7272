"""Micro-benchmarks of the hand-written HIP kernels vs PyTorch-ROCm at Llama-2-7B shapes.

Interleaved timing in one process (cdna_hip_programming.md §5.4 rule 24), random data.
"""
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def bench_attention(results, B=1, H=32, T=4096, D=128, causal=True):
    from lightning_thunder_amd.ops.attention import attn_fwd, attn_bwd

    q = torch.randn(B, H, T, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn_like(q)
    v = torch.randn_like(q)
    do = torch.randn_like(q)
    flops_fwd = 4 * B * H * T * T * D / (2 if causal else 1)
    o, lse = attn_fwd(q, k, v, causal)
    t_fwd = timeit(lambda: attn_fwd(q, k, v, causal))
    t_bwd = timeit(lambda: attn_bwd(do, q, k, v, o, lse, causal))
    r = torch.ops.aten._scaled_dot_product_flash_attention(q, k, v, 0.0, causal, False)
    t_tfwd = timeit(lambda: torch.ops.aten._scaled_dot_product_flash_attention(q, k, v, 0.0, causal, False))
    zero = torch.empty((), dtype=torch.int64)
    t_tbwd = timeit(lambda: torch.ops.aten._scaled_dot_product_flash_attention_backward(
        do, q, k, v, r[0], r[1], None, None, T, T, 0.0, causal, zero, zero))
    results["attention"] = {
        "shape": [B, H, T, D], "causal": causal,
        "hip_fwd_ms": t_fwd, "hip_fwd_tflops": flops_fwd / t_fwd / 1e9,
        "hip_bwd_ms": t_bwd, "hip_bwd_tflops": 2.5 * flops_fwd / t_bwd / 1e9,
        "torch_fwd_ms": t_tfwd, "torch_bwd_ms": t_tbwd,
    }


def bench_gemm(results):
    out = {}
    for (M, N, K) in [(4096, 12288, 4096), (4096, 4096, 4096), (4096, 11008, 4096), (4096, 4096, 11008), (4096, 32000, 4096)]:
        a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: torch.nn.functional.linear(a, w))
        out[f"{M}x{N}x{K}"] = {"torch_ms": t, "tflops": 2 * M * N * K / t / 1e9}
    results["gemm_hipblaslt"] = out
    # backward layouts: dgrad dY @ W, wgrad dY^T @ X; and the fused fc_1||fc_2 forward
    out = {}
    for (M, N, K) in [(4096, 4096, 11008), (4096, 4096, 12288), (4096, 4096, 4096), (4096, 11008, 4096)]:
        dy = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: torch.matmul(dy, w))
        out[f"dgrad {M}x{N}x{K}"] = {"torch_ms": t, "tflops": 2 * M * N * K / t / 1e9}
    for (N, K, M) in [(11008, 4096, 4096), (12288, 4096, 4096), (4096, 11008, 4096), (4096, 4096, 4096)]:
        dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: torch.matmul(dy.t(), x))
        out[f"wgrad {N}x{K}x{M}"] = {"torch_ms": t, "tflops": 2 * M * N * K / t / 1e9}
    a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(22016, 4096, device="cuda", dtype=torch.bfloat16)
    t = timeit(lambda: torch.nn.functional.linear(a, w))
    out["fwd fused fc 4096x22016x4096"] = {"torch_ms": t, "tflops": 2 * 4096 * 22016 * 4096 / t / 1e9}
    results["gemm_layouts"] = out
    from lightning_thunder_amd.ops.gemm import gemm_nt

    out = {}
    for (M, N, K) in [(4096, 12288, 4096), (4096, 4096, 4096), (4096, 11008, 4096), (4096, 4096, 11008),
                      (4096, 32000, 4096), (4096, 22016, 4096), (8192, 8192, 8192)]:
        a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        t_h = timeit(lambda: gemm_nt(a, w))
        t_t = timeit(lambda: torch.nn.functional.linear(a, w))
        out[f"{M}x{N}x{K}"] = {"hip_ms": t_h, "hip_tflops": 2 * M * N * K / t_h / 1e9, "hipblaslt_ms": t_t,
                               "hipblaslt_tflops": 2 * M * N * K / t_t / 1e9}
    results["gemm_hip_vs_hipblaslt"] = out


def bench_hipgemm(results):
    from lightning_thunder_amd.ops.gemm import gemm_nt

    out = {}
    for (M, N, K) in [(4096, 12288, 4096), (4096, 4096, 4096), (4096, 11008, 4096), (4096, 4096, 11008),
                      (4096, 32000, 4096), (4096, 22016, 4096), (8192, 8192, 8192)]:
        a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        t_h = timeit(lambda: gemm_nt(a, w))
        t_t = timeit(lambda: torch.nn.functional.linear(a, w))
        from lightning_thunder_amd.ops.fp8 import gemm_nt_fp8

        a8 = a.to(torch.float8_e4m3fn).view(torch.uint8)
        w8 = w.to(torch.float8_e4m3fn).view(torch.uint8)
        sc = torch.ones((), device="cuda")
        t_8 = timeit(lambda: gemm_nt_fp8(a8, w8, sc, sc)) if K % 128 == 0 else float("nan")
        out[f"{M}x{N}x{K}"] = {"hip_tflops": round(2 * M * N * K / t_h / 1e9), "hipblaslt_tflops": round(2 * M * N * K / t_t / 1e9),
                               "hip_fp8_tflops": round(2 * M * N * K / t_8 / 1e9)}
    results["gemm_hip_vs_hipblaslt"] = out


def main():
    torch.manual_seed(0)
    results = {}
    which = sys.argv[1:] or ["attention", "gemm"]
    if "attention" in which:
        bench_attention(results)
    if "gemm" in which:
        bench_gemm(results)
    if "hipgemm" in which:
        bench_hipgemm(results)
    print(json.dumps(results, indent=1))


if __name__ == "__main__":
    main()
