"""Finite-difference gradient checks of the analytic VJPs (``transforms/autodiff.py``) through
``thunder.jit``, in fp64 on CPU.

Parity: the reference's ``thunder/tests/test_grad.py`` (``check_vjp`` / numerical Jacobian checks of
the VJP rules across op families).  Each case is ``torch.autograd.gradcheck`` of the jitted function,
so first derivatives are compared against central differences, not against PyTorch's own backward.
"""
import pytest
import torch
import torch.nn.functional as F

import lightning_thunder_amd as thunder


def _x(*shape, seed=0, positive=False):
    t = torch.randn(*shape, generator=torch.Generator().manual_seed(seed), dtype=torch.float64)
    if positive:
        t = t.abs() + 0.5
    return t.requires_grad_(True)


CASES = {
    "softmax_matmul": (lambda a, b: torch.softmax(a @ b, -1), lambda: (_x(3, 4), _x(4, 5, seed=1))),
    "layer_norm": (lambda a, w, b: F.layer_norm(a, (6,), w, b), lambda: (_x(4, 6), _x(6, seed=1), _x(6, seed=2))),
    "rms_norm": (lambda a, w: a * torch.rsqrt(a.pow(2).mean(-1, keepdim=True) + 1e-6) * w,
                 lambda: (_x(3, 8), _x(8, seed=1))),
    "gelu_tanh": (lambda a: F.gelu(a, approximate="tanh"), lambda: (_x(5, 5),)),
    "silu_mul": (lambda a, b: F.silu(a) * b, lambda: (_x(4, 4), _x(4, 4, seed=1))),
    "cross_entropy": (lambda a: F.cross_entropy(a, torch.tensor([1, 0, 3])), lambda: (_x(3, 5),)),
    "logsumexp": (lambda a: torch.logsumexp(a, 1), lambda: (_x(4, 7),)),
    "var_std": (lambda a: torch.var(a, 0) + torch.std(a, 1).sum(), lambda: (_x(5, 4),)),
    "pow_div": (lambda a, b: a.pow(b) / (b + 1.0), lambda: (_x(3, 3, positive=True), _x(3, 3, seed=1, positive=True))),
    "atan2_hypot": (lambda a, b: torch.atan2(a, b) + torch.hypot(a, b), lambda: (_x(4), _x(4, seed=1))),
    "cumsum_flip": (lambda a: torch.cumsum(a.flip(1), 1) * a, lambda: (_x(3, 5),)),
    "gather_scatter_add": (lambda a: torch.gather(a, 1, torch.tensor([[0, 2], [1, 1]])).sum(1)
                           + torch.zeros(2, 3, dtype=torch.float64).scatter_add(1, torch.tensor([[0, 2], [1, 1]]), a[:, :2]).sum(1),
                           lambda: (_x(2, 3),)),
    "cat_split_stack": (lambda a, b: torch.stack(torch.split(torch.cat([a, b], 0), 2, 0), 0).sum(1),
                        lambda: (_x(2, 3), _x(2, 3, seed=1))),
    "where_clamp_abs": (lambda a: torch.where(a > 0, a.clamp(max=0.7), a.abs() * 2), lambda: (_x(6),)),
    "sdpa": (lambda q, k, v: F.scaled_dot_product_attention(q, k, v, is_causal=True),
             lambda: (_x(1, 2, 4, 8), _x(1, 2, 4, 8, seed=1), _x(1, 2, 4, 8, seed=2))),
    "linear_bias": (lambda x, w, b: F.linear(x, w, b).tanh(), lambda: (_x(3, 4), _x(5, 4, seed=1), _x(5, seed=2))),
    "embedding": (lambda w: F.embedding(torch.tensor([[0, 2, 2], [1, 0, 3]]), w).sum(-1), lambda: (_x(4, 3),)),
    "amax_prod": (lambda a: a.amax(1).sum() + a.prod(0).sum(), lambda: (_x(3, 4),)),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_gradcheck_jitted(name):
    fn, make = CASES[name]
    jf = thunder.jit(fn)
    assert torch.autograd.gradcheck(jf, make(), eps=1e-6, atol=1e-6, rtol=1e-4)
