"""Llama-4-style MoE block (``models/llama4_moe.py``; reference ``thunder/tests/llama4_moe.py``):
top-1 sigmoid router, tokens sorted by expert, grouped-GEMM SwiGLU experts over int32 offsets,
shared expert.  Outputs and every gradient match eager PyTorch."""
import pytest
import torch

import lightning_thunder_amd as thunder
from lightning_thunder_amd.models.llama4_moe import Llama4MoE, MoEConfig


def _check(m, x, out_tol, grad_tol):
    jm = thunder.jit(m)
    out, ref = jm(x), m(x)
    torch.testing.assert_close(out.float(), ref.float(), atol=out_tol, rtol=out_tol)
    g = torch.randn_like(out)
    ins = [x] + list(m.parameters())
    ga = torch.autograd.grad(out, ins, g)
    gr = torch.autograd.grad(ref, ins, g)
    for a, b in zip(ga, gr):
        rel = ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-6)).item()
        assert rel < grad_tol, (tuple(a.shape), rel)
    return jm


def test_llama4_moe_cpu():
    torch.manual_seed(0)
    m = Llama4MoE(MoEConfig(hidden_size=64, intermediate_size=128, num_routed_experts=4)).bfloat16()
    x = torch.randn(2, 32, 64, dtype=torch.bfloat16, requires_grad=True)
    _check(m, x, 1e-2, 2e-2)


@pytest.mark.gpu
def test_llama4_moe_gpu():
    """The reference's test configuration (hidden 256, intermediate 512, 8 routed experts, one
    shared expert, 2048 tokens) on the HIP executors: the routed projections run on the grouped
    MFMA GEMM."""
    torch.manual_seed(0)
    m = Llama4MoE(MoEConfig()).cuda().bfloat16()
    x = torch.randn(1, 2048, 256, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    jm = _check(m, x, 3e-2, 3e-2)
    assert "hip_grouped_mm" in str(thunder.last_traces(jm)[-1])
