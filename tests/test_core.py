"""Core compile pipeline tests (CPU, torch executor) — reference analogue: thunder/tests/test_core.py."""
import pytest
import torch

import lightning_thunder_amd as thunder


def test_mlp_forward_backward_matches_eager():
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(4, 8), torch.nn.ReLU(), torch.nn.Linear(8, 2))
    tm = thunder.jit(m)
    x = torch.randn(5, 4)
    out = tm(x)
    ref = m(x)
    torch.testing.assert_close(out, ref)
    out.sum().backward()
    g1 = [p.grad.clone() for p in m.parameters()]
    for p in m.parameters():
        p.grad = None
    ref.sum().backward()
    for a, p in zip(g1, m.parameters()):
        torch.testing.assert_close(a, p.grad)


def test_function_trace_printable_and_cached():
    def f(x, y):
        return torch.nn.functional.gelu(x @ y + 1.0).sum()

    jf = thunder.jit(f)
    x, y = torch.randn(3, 4), torch.randn(4, 5)
    torch.testing.assert_close(jf(x, y), f(x, y))
    src = str(thunder.last_traces(jf)[-1])
    assert "def computation" in src
    jf(x, y)
    assert thunder.cache_hits(jf) == 1 and thunder.cache_misses(jf) == 1
    # new shape -> prologue guard fails -> recompile
    jf(torch.randn(2, 4), y)
    assert thunder.cache_misses(jf) == 2


def test_python_number_specialization():
    def f(x, k):
        return x * k

    jf = thunder.jit(f)
    x = torch.randn(3)
    torch.testing.assert_close(jf(x, 2.0), x * 2.0)
    torch.testing.assert_close(jf(x, 3.0), x * 3.0)
    assert thunder.cache_misses(jf) == 2


@pytest.mark.parametrize("op", [
    lambda x: torch.tanh(x).sum(),
    lambda x: torch.sigmoid(x * 2).mean(),
    lambda x: torch.softmax(x, -1).pow(2).sum(),
    lambda x: torch.log_softmax(x, -1)[:, 1].sum(),
    lambda x: x.reshape(-1).cumsum(0).sum(),
    lambda x: torch.nn.functional.silu(x).sum(),
    lambda x: torch.nn.functional.layer_norm(x, (x.shape[-1],)).square().sum(),
    lambda x: x.transpose(0, 1).contiguous().view(-1)[::2].sum(),
    lambda x: torch.cat([x, x * 2], 0).amax(0).sum(),
    lambda x: (x / (x.abs() + 1)).var(),
    lambda x: torch.where(x > 0, x, x * 0.1).exp().sum(),
])
def test_grads_match_eager(op):
    torch.manual_seed(1)
    x = torch.randn(4, 6, dtype=torch.float64, requires_grad=True)
    jf = thunder.jit(op)
    out = jf(x)
    (g,) = torch.autograd.grad(out, x)
    x2 = x.detach().clone().requires_grad_(True)
    ref = op(x2)
    (g2,) = torch.autograd.grad(ref, x2)
    torch.testing.assert_close(out, ref)
    torch.testing.assert_close(g, g2)
