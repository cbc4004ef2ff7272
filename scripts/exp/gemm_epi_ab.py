"""A/B of the gemm4 epilogue: the reference build (scripts/exp/gemm4_ref.hip: LDS-image epilogue)
vs the production library (swapped-operand register epilogue), same box, interleaved rounds, random
data, every Llama-2-7B training GEMM shape and layout."""
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
ref = ctypes.CDLL(os.path.join(HERE, "gemm4_ref.so"))
ref.lta_gemm4_bf16.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int] * 7 + [ctypes.c_float] + [ctypes.c_int] * 4 + [ctypes.c_void_p]

SHAPES = [("fwd", 4096, 12288, 4096), ("fwd", 4096, 4096, 4096), ("fwd", 4096, 22016, 4096), ("fwd", 4096, 4096, 11008),
          ("fwd", 4096, 32000, 4096), ("dgrad", 4096, 4096, 12288), ("dgrad", 4096, 4096, 4096),
          ("dgrad", 4096, 11008, 4096), ("dgrad", 4096, 4096, 22016), ("wgrad", 12288, 4096, 4096),
          ("wgrad", 4096, 4096, 4096), ("wgrad", 22016, 4096, 4096), ("wgrad", 4096, 11008, 4096)]


def operands(kind, M, N, K):
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: torch.empty(*s, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1, generator=g)  # noqa: E731
    if kind == "fwd":
        return r(M, K), r(N, K).t()
    if kind == "dgrad":
        return r(M, K), r(K, N)
    return r(K, M).t(), r(K, N)


def main():
    rounds = int(os.environ.get("ROUNDS", "5"))
    out = []
    s = torch.cuda.current_stream().cuda_stream
    for kind, M, N, K in SHAPES:
        a, b = operands(kind, M, N, K)
        at, bt, lda, ldb = G.gemm4_layout(a, b)
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)

        def old():
            rc = ref.lta_gemm4_bf16(a.data_ptr(), b.data_ptr(), C.data_ptr(), None, None, M, N, K, lda, ldb, N, 0, 1.0,
                                    0, at, bt, 1, s)
            assert rc == 0, rc

        fns = {"ref_lds_epilogue": old, "new_register_epilogue": lambda: G.matmul4(a, b, out=C)}
        want = a.float() @ b.float()
        for name, fn in fns.items():
            C.zero_()
            fn()
            torch.cuda.synchronize()
            err = ((C.float() - want).abs().max() / want.abs().max()).item()
            assert err < 1e-2, (kind, M, N, K, name, err)
        del want
        t_end = time.time() + 1.0
        while time.time() < t_end:
            old()
            torch.cuda.synchronize()
        ts = {k: [] for k in fns}
        for _ in range(rounds):
            for name, fn in fns.items():
                fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                ts[name].append(e0.elapsed_time(e1) * 100)
        row = {"kind": kind, "M": M, "N": N, "K": K}
        for name in fns:
            row[name + "_us"] = round(statistics.median(ts[name]), 1)
            row[name + "_tflops"] = round(2 * M * N * K / statistics.median(ts[name]) / 1e6)
        row["speedup"] = round(row["ref_lds_epilogue_us"] / row["new_register_epilogue_us"], 4)
        print(json.dumps(row), flush=True)
        out.append(row)
    print("JSON", json.dumps(out))


if __name__ == "__main__":
    main()
