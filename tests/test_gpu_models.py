"""End-to-end compiled LitGPT-style models on the GPU vs eager (reference analogue: test_networks.py)."""
import pytest
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.models.litgpt import GPT, init_weights

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["llama2-like", "llama3-like", "gpt-neox-like"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_litgpt_fwd_bwd_gpu(name, dtype):
    torch.manual_seed(0)
    dev = torch.device("cuda")
    m = GPT.from_name(name).to(device=dev, dtype=dtype)
    init_weights(m)
    m.set_rope_cache(64, device=dev)
    idx = torch.randint(0, 320, (2, 64), device=dev)
    tm = thunder.jit(m)
    out = tm(idx)
    ref = m(idx)
    tol = 1e-4 if dtype == torch.float32 else 5e-2
    torch.testing.assert_close(out.float(), ref.float(), atol=tol, rtol=tol)
    g = torch.randn_like(out)
    out.backward(g)
    got = {n: p.grad.float().clone() for n, p in m.named_parameters()}
    for p in m.parameters():
        p.grad = None
    ref.backward(g)
    for n, p in m.named_parameters():
        torch.testing.assert_close(got[n], p.grad.float(), atol=tol * 10, rtol=tol * 10, msg=n)
    src = str(thunder.last_traces(tm)[-1])
    if name != "gpt-neox-like":
        assert "hip_rms_norm_fwd" in src
