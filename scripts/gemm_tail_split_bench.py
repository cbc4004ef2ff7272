"""Event-timed A/B of the gemm4 tail split on the Llama-2-7B gate/up shapes (forward NT and wgrad TN),
back-to-back calls (as in the step) with 4 operand sets rotating so reads are not all L2 hits."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops import gemm

torch.manual_seed(0)
res = {}
for name, M, N, K in [("gate_up_fwd", 4096, 22016, 4096), ("gate_up_wgrad", 22016, 4096, 4096)]:
    if name == "gate_up_fwd":
        ops = [(torch.randn(M, K, device="cuda", dtype=torch.bfloat16),
                torch.randn(N, K, device="cuda", dtype=torch.bfloat16).t()) for _ in range(4)]
    else:  # dW = dY^T @ X: dY [T, N_out] stored token-major, read transposed
        ops = [(torch.randn(K, M, device="cuda", dtype=torch.bfloat16).t(),
                torch.randn(K, N, device="cuda", dtype=torch.bfloat16)) for _ in range(4)]
    outs = {}
    for split in (True, False, True, False):
        gemm._TAIL_SPLIT = split
        for i in range(8):
            y = gemm.matmul4(*ops[i % 4])
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for i in range(40):
            y = gemm.matmul4(*ops[i % 4])
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 40 * 1000
        outs[split] = gemm.matmul4(*ops[0]).float()
        key = f"{name}_split{int(split)}"
        res.setdefault(key, []).append(round(us, 1))
        print(key, round(us, 1), "us", round(2 * M * N * K / us / 1e6, 1), "TF/s", flush=True)
    print(name, "split vs plain max |diff|", (outs[True] - outs[False]).abs().max().item(), flush=True)
gemm._TAIL_SPLIT = True
print(res)
