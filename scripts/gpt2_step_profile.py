"""GPT-2-medium (nanoGPT, LayerNorm + bias linears + GELU + dropout) training step on the HIP
executors, for a rocprofv3 step breakdown: shows which kernels run the LayerNorm / bias-grad /
dropout / GELU work (hipfuse ``lta_fused_*`` regions, LayerNorm kernel, hand GEMMs) instead of
ATen.  Synthetic tokens, random init.

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt2 -o run --output-format csv -- \\
        python scripts/gpt2_step_profile.py
"""
import time

import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.models.nanogpt import NanoGPT
from lightning_thunder_amd.optim import AdamW


def main(steps=6, B=8, T=1024):
    torch.manual_seed(0)
    m = NanoGPT.from_name("gpt2-medium", seq_len=T).to(device="cuda", dtype=torch.bfloat16)
    m.train()
    jm = thunder.jit(m)
    opt = AdamW(list(m.parameters()), lr=3e-4, betas=(0.9, 0.95), weight_decay=0.1)
    V = m.config.vocab_size
    x = torch.randint(0, V, (B, T), device="cuda")
    y = torch.randint(0, V, (B, T), device="cuda")
    for i in range(steps):
        t0 = time.perf_counter()
        _, loss = jm(x, y)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        print(f"step {i}: {1e3 * (time.perf_counter() - t0):.1f} ms loss {loss.item():.4f}", flush=True)


if __name__ == "__main__":
    main()
