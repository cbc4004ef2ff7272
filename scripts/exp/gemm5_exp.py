"""Persistent swapped-epilogue GEMM experiment (scripts/exp/gemm5_exp.hip) vs the production gemm4
kernel, interleaved rounds in one process on random data; per-workgroup in-kernel clock."""
import ctypes
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from lightning_thunder_amd.ops import gemm as G  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "gemm5_exp.so"))
lib.g5_gemm.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int] * 7 + [ctypes.c_void_p] * 2
CUS = torch.cuda.get_device_properties(0).multi_processor_count


def operands(kind, M, N, K):
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: torch.empty(*s, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)  # noqa: E731
    if kind == "fwd":  # C = X W^T
        x, w = r(M, K), r(N, K)
        return (x, w.t()), (0, x, w, K, K)
    if kind == "dgrad":  # C = dY W, W stored [K][N]
        dy, w = r(M, K), r(K, N)
        return (dy, w), (1, dy, w, K, N)
    a, b = r(K, M), r(K, N)  # wgrad: C = A^T B, A stored [K][M], B stored [K][N]
    return (a.t(), b), (2, a, b, M, N)


def main():
    shapes = [("fwd", 4096, 12288, 4096), ("fwd", 4096, 4096, 4096), ("fwd", 4096, 22016, 4096),
              ("fwd", 4096, 4096, 11008), ("fwd", 4096, 32000, 4096), ("dgrad", 4096, 11008, 4096),
              ("dgrad", 4096, 4096, 12288), ("wgrad", 22016, 4096, 4096), ("wgrad", 4096, 11008, 4096),
              ("wgrad", 12288, 4096, 4096)]
    if len(sys.argv) > 1:
        shapes = shapes[: int(sys.argv[1])]
    rounds = int(os.environ.get("ROUNDS", "5"))
    out = []
    for kind, M, N, K in shapes:
        (a4, b4), (lay, A, B, lda, ldb) = operands(kind, M, N, K)
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        nwg = -(-M // 256) * -(-N // 256)
        st = torch.zeros(nwg * 4, dtype=torch.int64, device="cuda")
        s = torch.cuda.current_stream().cuda_stream

        def g5(p):
            rc = lib.g5_gemm(lay, p, A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, lda, ldb, N, CUS, st.data_ptr(), s)
            assert rc == 0, rc

        fns = {"gemm4": lambda: G.matmul4(a4, b4, out=C), "g5": lambda: g5(0), "g5_persist": lambda: g5(1)}
        ref = (a4.float() @ b4.float())
        for name, fn in fns.items():
            C.zero_()
            fn()
            torch.cuda.synchronize()
            err = ((C.float() - ref).abs().max() / ref.abs().max()).item()
            assert err < 1e-2, (kind, M, N, K, name, err)
        del ref
        t_end = time.time() + 1.5
        while time.time() < t_end:
            for _ in range(10):
                fns["gemm4"]()
            torch.cuda.synchronize()
        ts = {k: [] for k in fns}
        for r in range(rounds):
            for name, fn in fns.items():
                for _ in range(2):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                ts[name].append(e0.elapsed_time(e1) * 100)
        fl = 2 * M * N * K
        row = {"kind": kind, "M": M, "N": N, "K": K}
        for name in fns:
            us = statistics.median(ts[name])
            row[name + "_us"] = round(us, 1)
            row[name + "_tflops"] = round(fl / us / 1e6)
        print(json.dumps(row), flush=True)
        out.append(row)
    print("JSON", json.dumps(out))


if __name__ == "__main__":
    main()
