"""Host cost of output allocation variants on the GPU (caching allocator): python scripts/alloc_bench.py"""
import time

import torch

dev = torch.device("cuda", 0)
x = torch.empty(16, device=dev, dtype=torch.bfloat16)
shape = (2048, 1600)
n = 20000
cases = {
    "torch.empty(shape, dtype, device=torch.device)": lambda: torch.empty(shape, dtype=torch.bfloat16, device=dev),
    "torch.empty(shape, dtype, device=0)": lambda: torch.empty(shape, dtype=torch.bfloat16, device=0),
    "torch.empty(shape, dtype, device='cuda')": lambda: torch.empty(shape, dtype=torch.bfloat16, device="cuda"),
    "x.new_empty(shape)": lambda: x.new_empty(shape),
    "torch.empty_like(y)": None,
    "data_ptr": lambda: x.data_ptr(),
    "torch.cuda.current_stream().cuda_stream": lambda: torch.cuda.current_stream().cuda_stream,
    "torch._C._cuda_getCurrentRawStream(0)": lambda: torch._C._cuda_getCurrentRawStream(0),
}
y = torch.empty(shape, dtype=torch.bfloat16, device=dev)
cases["torch.empty_like(y)"] = lambda: torch.empty_like(y)
for name, fn in cases.items():
    for _ in range(1000):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    print(f"{name:48s} {1e6 * (t1 - t0) / n:6.2f} us", flush=True)
