"""MXFP4 recipe diagnostics: GEMM vs dequantised product on the Llama-2-7B linear shapes, and a
few optimizer steps of a small LitGPT model (loss must fall)."""
import torch

from lightning_thunder_amd.ops import mxfp4

torch.manual_seed(0)
for (M, N, K) in ((4096, 12288, 4096), (4096, 4096, 4096), (4096, 22016, 4096), (4096, 4096, 11008), (4096, 32000, 4096)):
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    qx, sx = mxfp4.quantize(x)
    qw, sw = mxfp4.quantize(w)
    got = mxfp4.gemm_nt(qx, sx, qw, sw).float()
    exact = mxfp4.dequantize(qx, sx) @ mxfp4.dequantize(qw, sw).T
    ref = x.float() @ w.float().T
    print(f"{M}x{N}x{K}: kernel-vs-dequant {((got - exact).norm() / exact.norm()).item():.3e}  "
          f"vs-bf16 {((got - ref).norm() / ref.norm()).item():.3e}", flush=True)

import lightning_thunder_amd as thunder
from lightning_thunder_amd.models.litgpt import GPT, Config, init_weights
from lightning_thunder_amd.transforms.fp8 import FP8LinearTransform

for recipe in ("mxfp8", "mxfp4"):
    torch.manual_seed(0)
    cfg = Config.from_name("Llama-2-7b-hf", n_layer=2, n_embd=1024, n_head=8, n_query_groups=8, intermediate_size=2816,
                           padded_vocab_size=32000, block_size=1024)
    m = GPT(cfg).cuda().bfloat16()
    init_weights(m)
    m.set_rope_cache(1024, device="cuda")
    t = FP8LinearTransform(recipe=recipe)
    jm = thunder.jit(m, transforms=[t])
    opt = torch.optim.AdamW(m.parameters(), lr=3e-4)
    idx = torch.randint(0, 32000, (1, 1024), device="cuda")
    losses = []
    for step in range(8):
        logits = jm(idx)
        loss = torch.nn.functional.cross_entropy(logits.float().reshape(-1, logits.shape[-1]), idx.reshape(-1))
        loss.backward()
        gn = sum(p.grad.float().norm() ** 2 for p in m.parameters() if p.grad is not None) ** 0.5
        opt.step()
        opt.zero_grad()
        losses.append((round(loss.item(), 4), round(gn.item(), 4)))
    print(recipe, t.n_converted, losses, flush=True)
