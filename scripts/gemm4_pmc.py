"""Workload for PMC passes over gemm4: the fwd shape with many short tiles (X[4096,4096] @ W^T,
N 12288: 768 tiles x 64 K-steps) and the dgrad shape with few long tiles (dY @ W, K 12288:
256 tiles x 192 K-steps).  Same FLOPs; kernels are told apart by their template arguments."""
import torch

from lightning_thunder_amd.ops.gemm import matmul4

g = torch.Generator(device="cuda").manual_seed(0)
x = torch.randn(4096, 4096, device="cuda", generator=g).bfloat16()
w = torch.randn(12288, 4096, device="cuda", generator=g).bfloat16()
dy = torch.randn(4096, 12288, device="cuda", generator=g).bfloat16()
for _ in range(10):
    matmul4(x, w.t())   # fwd: at 0, bt 0
    matmul4(dy, w)      # dgrad: at 0, bt 1
torch.cuda.synchronize()
