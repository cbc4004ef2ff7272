"""hipBLASLt (torch.mm) TF/s across N near 11008 for the Llama-2-7B MLP shapes (random data)."""
import torch

def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3

M = K = 4096
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
for N in (10752, 11008, 11264, 11520, 12288):
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    g = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    f = 2 * M * N * K
    fwd = t(lambda: x @ w.T)            # Y = X W^T
    fwdT = t(lambda: w @ x.T)           # Y^T = W X^T
    wgrad = t(lambda: g.T @ x)          # dW = dY^T X
    dgrad = t(lambda: g @ w)            # dX = dY W
    print(f"N={N}: fwd {f/fwd/1e6:.0f} TF ({fwd:.0f} us)  fwd^T {f/fwdT/1e6:.0f}  wgrad {f/wgrad/1e6:.0f}  dgrad {f/dgrad/1e6:.0f}", flush=True)
