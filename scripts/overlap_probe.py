"""Does a memory-bound optimizer kernel on a side stream overlap with compute-bound GEMMs?
(Sequential vs two-stream time; the answer decides whether AdamW can hide under the backward.)"""
import torch

from lightning_thunder_amd.optim import AdamW

torch.manual_seed(0)
dev = torch.device("cuda")
a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
w = torch.randn(11008, 4096, device=dev, dtype=torch.bfloat16)
params = [torch.nn.Parameter(torch.randn(11008, 4096, device=dev, dtype=torch.bfloat16)) for _ in range(24)]
for p in params:
    p.grad = torch.randn_like(p)
opt = AdamW(params, lr=1e-4)
opt.step()
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def gemms(n=24):
    for _ in range(n):
        torch.nn.functional.linear(a, w)


def timed(fn):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def seq():
    gemms()
    opt.step()


def conc():
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        gemms()
    with torch.cuda.stream(s2):
        opt.step()
    cur.wait_stream(s1)
    cur.wait_stream(s2)


for name, fn in (("gemms", gemms), ("adamw", opt.step), ("sequential", seq), ("two streams", conc)):
    fn()
    ts = sorted(timed(fn) for _ in range(5))
    print(f"{name:12s} {ts[len(ts) // 2]:8.2f} ms", flush=True)
