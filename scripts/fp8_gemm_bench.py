"""FP8 NT GEMM A/B on the Llama-2-7B training shapes (fwd, dgrad, wgrad as the FP8 recipe runs them:
all NT on transposed fp8 copies): the 4-wave pipelined kernel (lta_gemm4_fp8) vs the 8-wave one
(lta_gemm_nt_fp8).  Interleaved rounds, TF/s; correctness of gemm4_fp8 vs the old kernel first."""
import json

import torch

from lightning_thunder_amd.ops._lib import require, stream_ptr
from lightning_thunder_amd.ops import fp8 as F  # noqa: F401  (registers the signatures)

lib = require()


def run(fn, a, b, out, sa, sb, fa, fb):
    M, K = a.shape
    N = b.shape[0]
    return fn(a.data_ptr(), b.data_ptr(), out.data_ptr(), None, M, N, K, a.stride(0), b.stride(0), out.stride(0),
              fa, fb, sa.data_ptr(), sb.data_ptr(), stream_ptr(a.device))


def timed(f, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    f()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    sa = torch.tensor(1.0, device="cuda")
    sb = torch.tensor(1.0, device="cuda")
    shapes = []
    for n, k in [(12288, 4096), (4096, 4096), (11008, 4096), (22016, 4096), (4096, 11008), (32000, 4096)]:
        shapes += [("fwd", 4096, n, k, 0), ("dgrad", 4096, k, n, 1), ("wgrad", n, k, 4096, 1)]
    res = {}
    for kind, M, N, K, fa in shapes:
        a = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(torch.float8_e5m2 if fa else torch.float8_e4m3fn).view(torch.uint8)
        b = (torch.randn(N, K, device="cuda", generator=g) * 0.5).to(torch.float8_e4m3fn).view(torch.uint8)
        o1 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        o2 = torch.empty_like(o1)
        assert run(lib.lta_gemm4_fp8, a, b, o1, sa, sb, fa, 0) == 0
        assert run(lib.lta_gemm_nt_fp8, a, b, o2, sa, sb, fa, 0) == 0
        torch.cuda.synchronize()
        err = ((o1.float() - o2.float()).norm() / o2.float().norm()).item()
        t4, t8 = [], []
        for _ in range(3):
            t4.append(timed(lambda: run(lib.lta_gemm4_fp8, a, b, o1, sa, sb, fa, 0)))
            t8.append(timed(lambda: run(lib.lta_gemm_nt_fp8, a, b, o2, sa, sb, fa, 0)))
        fl = 2 * M * N * K
        key = f"{kind} M{M} N{N} K{K}"
        res[key] = {"gemm4_fp8": round(fl / min(t4) / 1e9), "old": round(fl / min(t8) / 1e9), "rel_err_vs_old": err}
        print(key, res[key], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
