"""Lane mapping of ds_read_b64_tr_b8 (scripts/exp/tr8_probe.hip): hypothesis, by analogy with the
documented tr_b16 form, = per 16-lane group a block of 8 rows x 16 byte columns; lane 2q + p supplies
the address of row q, columns 8p .. 8p + 7; lane i receives column i of the 8 rows, row q in byte q."""
import ctypes
import os
import sys

import torch

here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "tr8_probe.so"))
lib.tr8_probe.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
addr = torch.zeros(64, dtype=torch.int32)
for lane in range(64):
    g, i = lane // 16, lane % 16
    q, p = i // 2, i % 2
    addr[lane] = (8 * g + q) * 256 + 16 * g + 8 * p  # group g: rows 8g .. 8g+7, columns 16g .. 16g+15
a = addr.cuda()
out = torch.zeros(128, dtype=torch.int32, device="cuda")
rc = lib.tr8_probe(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(out.data_ptr()), None)
torch.cuda.synchronize()
o = out.cpu().numpy().view("uint8").reshape(64, 8)
ok = True
for lane in range(64):
    g, i = lane // 16, lane % 16
    exp = [(((8 * g + q) & 15) << 4) | ((16 * g + i) & 15) for q in range(8)]
    if list(o[lane]) != exp:
        ok = False
    if lane < 18 or list(o[lane]) != exp:
        print(lane, [hex(x) for x in o[lane]], "expected", [hex(x) for x in exp])
print("rc", rc, "HYPOTHESIS", "CONFIRMED" if ok else "REJECTED")
sys.exit(0 if ok else 3)
