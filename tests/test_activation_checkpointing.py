"""Activation checkpointing: ``torch.utils.checkpoint`` regions are traced as ``ltorch.checkpoint``
and their intermediates recomputed in the backward instead of saved (reference
``thunder/torch/__init__.py:6348``, ``transforms/autodiff.py:190-209``)."""
import pytest
import torch
from torch.utils.checkpoint import checkpoint

import lightning_thunder_amd as thunder


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.l1 = torch.nn.Linear(16, 64)
        self.l2 = torch.nn.Linear(64, 16)

    def block(self, x):
        return self.l2(torch.nn.functional.gelu(self.l1(x))).tanh()

    def forward(self, x, ck: bool):
        for _ in range(3):
            x = checkpoint(self.block, x, use_reentrant=False) if ck else self.block(x)
        return x.sum()


def _saved(jm):
    ret = thunder.last_traces(jm)[-1].bound_symbols[-1]
    return ret.args[0][1]


def test_checkpoint_recomputes_instead_of_saving():
    torch.manual_seed(0)
    m = _Net()
    x0 = torch.randn(8, 16)
    grads, saved = {}, {}
    for ck in (False, True):
        jm = thunder.jit(lambda x, ck=ck: m(x, ck))
        x = x0.clone().requires_grad_(True)
        jm(x).backward()
        grads[ck] = x.grad
        saved[ck] = len(_saved(jm))
    torch.testing.assert_close(grads[True], grads[False])
    assert saved[True] < saved[False], saved
    # eager reference
    x = x0.clone().requires_grad_(True)
    m(x, True).backward()
    torch.testing.assert_close(grads[True], x.grad)


def test_litgpt_activation_checkpointing():
    from lightning_thunder_amd.models.litgpt import GPT

    torch.manual_seed(0)
    m = GPT.from_name("llama2-like")
    m.set_rope_cache(32, device="cpu")
    idx = torch.randint(0, m.config.vocab_size, (2, 32))
    outs = {}
    for ck in (False, True):
        m.activation_checkpointing = ck
        m.zero_grad()
        jm = thunder.jit(m)
        jm(idx).float().pow(2).mean().backward()
        outs[ck] = ({n: p.grad.clone() for n, p in m.named_parameters()}, len(_saved(jm)))
    for n, g in outs[False][0].items():
        torch.testing.assert_close(outs[True][0][n], g, rtol=1e-4, atol=1e-5)
    assert outs[True][1] < outs[False][1]


def test_auto_recompute_intermediates():
    """``auto_recompute_intermediates=True`` (reference ``core/trace_interpreter.py:204-222``):
    intermediates of differentiated decompositions are recomputed in the backward, so fewer
    tensors are saved; gradients are unchanged."""
    def f(x, w):
        return torch.logsumexp(x * w, -1).sum()

    x0 = torch.arange(128.0).reshape(8, 16).sin()
    w0 = torch.linspace(-1, 1, 16)
    res = {}
    for opt in (False, True):
        x, w = x0.clone().requires_grad_(True), w0.clone().requires_grad_(True)
        jf = thunder.jit(f, auto_recompute_intermediates=opt)
        jf(x, w).backward()
        res[opt] = (len(_saved(jf)), x.grad, w.grad)
    assert res[True][0] < res[False][0], (res[True][0], res[False][0])
    x, w = x0.clone().requires_grad_(True), w0.clone().requires_grad_(True)
    f(x, w).backward()
    for opt in (False, True):
        torch.testing.assert_close(res[opt][1], x.grad)
        torch.testing.assert_close(res[opt][2], w.grad)
