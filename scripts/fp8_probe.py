"""Determines the operand layout of v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3) on the GPU."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from lightning_thunder_amd.ops._lib import require, stream_ptr

lib = require()
lib.lta_fp8_mfma_probe.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
torch.manual_seed(0)
av = torch.randint(-3, 4, (64, 32)).float()
bv = torch.randint(-3, 4, (64, 32)).float()
a = av.to(torch.float8_e4m3fn).view(torch.uint8).cuda().contiguous()
b = bv.to(torch.float8_e4m3fn).view(torch.uint8).cuda().contiguous()
c = torch.zeros(64, 4, device="cuda")
lib.lta_fp8_mfma_probe(a.data_ptr(), b.data_ptr(), c.data_ptr(), 0, 0, stream_ptr())
torch.cuda.synchronize()
C = torch.zeros(16, 16)
for l in range(64):
    for j in range(4):
        C[4 * (l // 16) + j, l % 16] = c[l, j].cpu()
cands = {
    "a": lambda l, i: (l % 16, 32 * (l // 16) + i),
    "b": lambda l, i: (l % 16, 16 * (l // 16) + (i % 16) + 64 * (i // 16)),
    "c": lambda l, i: (l % 16, 8 * (l // 16) + (i % 8) + 32 * (i // 8)),
    "d": lambda l, i: (l % 16, 4 * (l // 16) + (i % 4) + 16 * (i // 4)),
}
found = []
for na, fa in cands.items():
    At = torch.zeros(16, 128)
    for l in range(64):
        for i in range(32):
            r, k = fa(l, i)
            At[r, k] = av[l, i]
    for nb, fb in cands.items():
        Bt = torch.zeros(16, 128)
        for l in range(64):
            for i in range(32):
                r, k = fb(l, i)
                Bt[r, k] = bv[l, i]
        if torch.equal(At @ Bt.t(), C):
            found.append((na, nb))
print("matching (A layout, B layout):", found)
print("C[0,:4] =", C[0, :4].tolist())
