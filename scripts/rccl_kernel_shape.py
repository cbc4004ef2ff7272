"""World-1 RCCL collectives of the FSDP / DDP message sizes, for a kernel trace that shows the RCCL
kernel's workgroup shape (threads, LDS, VGPRs) — the shape scripts/cu_contention.py occupies CUs with.

    rocprofv3 --kernel-trace --stats -d gpurun_out/rccl_shape -- python scripts/rccl_kernel_shape.py
"""
import os

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
n = 64 << 20 >> 1  # 64 MiB of bf16
x = torch.randn(n, device=dev, dtype=torch.bfloat16)
out = torch.empty_like(x)
for _ in range(5):
    dist.all_reduce(x)
    dist.reduce_scatter_tensor(out, x)
    dist.all_gather_into_tensor(out, x)
torch.cuda.synchronize()
dist.destroy_process_group()
print("ok")
