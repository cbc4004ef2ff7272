"""Prices the parts of the gemm4 NT main loop (scripts/exp/gemm_anatomy.hip) on random data:
wall time per launch, in-kernel clock (median s_memtime / s_memrealtime ratio over workgroups) and
cycles per K-tile, interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24)."""
import ctypes
import json
import os
import statistics
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "gemm_anatomy.so"))
lib.anat_gemm.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 + [ctypes.c_void_p, ctypes.c_void_p]
NAMES = {0: "full", 1: "no_glds", 2: "no_dsread", 3: "no_glds_no_dsread", 4: "no_barrier", 7: "mfma_only",
         8: "no_epilogue", 15: "mfma_only_no_epi", 16: "epi_no_global_store", 32: "epi_regs_store_only",
         17: "no_glds_epi_no_store", 64: "swapped_regs_epilogue"}


def run(abl, a, b, c, st, M, N, K):
    rc = lib.anat_gemm(abl, a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, st.data_ptr(),
                       torch.cuda.current_stream().cuda_stream)
    assert rc == 0, rc


def main():
    shapes = [(4096, 12288, 4096), (4096, 4096, 4096)]
    abls = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else "0,64,8,16".split(","))]
    rounds = int(os.environ.get("ROUNDS", "6"))
    out = {}
    for (M, N, K) in shapes:
        a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        nwg = (M // 256) * (N // 256)
        st = torch.zeros(nwg * 6, dtype=torch.int64, device="cuda")
        ref = (a.float() @ b.float().t())
        for x in (0, 64):
            if x not in abls:
                continue
            c.zero_()
            run(x, a, b, c, st, M, N, K)
            torch.cuda.synchronize()
            err = ((c.float() - ref).abs().max() / ref.abs().max()).item()
            print(f"{M}x{N}x{K} {NAMES[x]} rel err {err:.2e}", flush=True)
            assert err < 1e-2, (x, err)
        t_end = time.time() + 2.0
        while time.time() < t_end:
            for _ in range(20):
                run(0, a, b, c, st, M, N, K)
            torch.cuda.synchronize()
        res = {x: {"us": [], "ghz": [], "cyc_per_ktile": [], "pro": [], "loop": [], "epi": []} for x in abls}
        for r in range(rounds):
            for x in abls:
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                for _ in range(3):
                    run(x, a, b, c, st, M, N, K)
                ev0.record()
                n = 20
                for _ in range(n):
                    run(x, a, b, c, st, M, N, K)
                ev1.record()
                torch.cuda.synchronize()
                res[x]["us"].append(ev0.elapsed_time(ev1) * 1000 / n)
                s = st.view(nwg, 6).cpu().double()
                dt, dr = s[:, 1] - s[:, 0], s[:, 3] - s[:, 2]
                res[x]["pro"].append((s[:, 4] - s[:, 0]).median().item())
                res[x]["loop"].append(((s[:, 5] - s[:, 4]) / (K // 64)).median().item())
                res[x]["epi"].append((s[:, 1] - s[:, 5]).median().item())
                ghz = (dt / dr * 0.1).median().item()
                res[x]["ghz"].append(ghz)
                res[x]["cyc_per_ktile"].append((dt.median() / (K // 64)).item())
        fl = 2 * M * N * K
        out[f"{M}x{N}x{K}"] = {}
        for x in abls:
            us = statistics.median(res[x]["us"])
            row = {"us_median": round(us, 1), "us_min": round(min(res[x]["us"]), 1),
                   "tflops": round(fl / us / 1e6), "clock_ghz": round(statistics.median(res[x]["ghz"]), 3),
                   "cycles_per_ktile_per_wg": round(statistics.median(res[x]["cyc_per_ktile"])),
                   "prologue_cyc": round(statistics.median(res[x]["pro"])),
                   "loop_cyc_per_ktile": round(statistics.median(res[x]["loop"])),
                   "epilogue_cyc": round(statistics.median(res[x]["epi"]))}
            out[f"{M}x{N}x{K}"][NAMES[x]] = row
            print(f"{M}x{N}x{K} {NAMES[x]:>18}: {row}", flush=True)
    print("JSON", json.dumps(out))


if __name__ == "__main__":
    main()
