"""In-place updates through views and aliases (functionalization, ``core/functionalization.py``).

Parity: the reference's ``thunder/tests/test_update_aliases.py`` (setitem on a view, in-place on
``chunk`` outputs at default and non-default dims, chained in-place ops, aliased inputs, writes to
intermediates, viewed inputs of different shapes).  Every case checks the returned values AND the
state of every input after the call against eager PyTorch, on fresh copies of the same data.
"""
import pytest
import torch

import lightning_thunder_amd as thunder


def _run_both(fn, make_args, cache=None):
    ea = make_args()
    ga = make_args()
    exp = fn(*ea)
    jf = thunder.jit(fn) if cache is None else thunder.jit(fn, cache=cache)
    got = jf(*ga)
    exp_l = exp if isinstance(exp, (tuple, list)) else (exp,)
    got_l = got if isinstance(got, (tuple, list)) else (got,)
    for e, g in zip(exp_l, got_l):
        if isinstance(e, torch.Tensor):
            torch.testing.assert_close(g, e)
    for e, g in zip(ea, ga):
        if isinstance(e, torch.Tensor):
            torch.testing.assert_close(g, e)  # the input mutations match eager
    return jf, ga


def _x(*shape, seed=0):
    return torch.randn(*shape, generator=torch.Generator().manual_seed(seed))


def test_setitem_on_view():
    def f(a):
        v = a[1:3]
        v[0] = 5.0
        return a * 2

    _run_both(f, lambda: (_x(4, 3),))


def test_inplace_on_view_of_input():
    def f(a, b):
        v = a.view(-1)
        v.mul_(2).add_(b.reshape(-1))
        return v.sum()

    _run_both(f, lambda: (_x(2, 3), _x(2, 3, seed=1)))


@pytest.mark.parametrize("dim", [0, 1])
def test_inplace_on_chunk(dim):
    def f(a):
        c0, c1 = a.chunk(2, dim)
        c0.add_(1.0)
        c1.mul_(3.0)
        return a.exp()

    _run_both(f, lambda: (_x(4, 6),))


def test_chained_inplace():
    def f(a):
        a.add_(1).mul_(2).sub_(0.5).div_(4)
        return a + 0

    _run_both(f, lambda: (_x(5),))


def test_inplace_on_intermediate_then_read():
    def f(a):
        t = a.sin()
        t.mul_(2)
        u = t.view(-1)
        u[0] = -1.0
        return t, u.sum()

    _run_both(f, lambda: (_x(3, 2),))


def test_aliased_inputs_same_tensor():
    def f(a, b):
        a.add_(1.0)
        return b * 2  # b IS a: sees the update

    x = _x(4)
    xe = x.clone()
    e_out = f(xe, xe)
    xg = x.clone()
    g_out = thunder.jit(f)(xg, xg)
    torch.testing.assert_close(g_out, e_out)
    torch.testing.assert_close(xg, xe)


def test_partially_overlapping_inputs_raise_clearly():
    """Two inputs whose storages overlap only in part (a[:4], a[2:6]) with one of them updated in
    place: not functionalised; the call fails with an explicit NotImplementedError rather than
    returning stale values."""
    def f(a, b):
        a.mul_(3.0)
        return a + b

    base = _x(8)
    with pytest.raises(NotImplementedError, match="partially overlaps"):
        thunder.jit(f)(base[:4], base[2:6])


@pytest.mark.parametrize("cache", [None, "no caching"])
def test_write_to_intermediate_result(cache):
    def f(a):
        y = a.view(-1)
        y.add_(1)
        return y

    _run_both(f, lambda: (_x(2, 3),), cache=cache)


@pytest.mark.parametrize("cache", [None, "no caching"])
def test_viewed_inputs_of_different_shapes(cache):
    """The base and two disjoint row views of it as three inputs; one view is updated in place
    (reference test_update_aliases.py:534-551)."""
    def f(x, y, z):
        return x + 2, y.add_(z)

    a = _x(2, 3)
    a_ = a.clone()
    jf = thunder.jit(f) if cache is None else thunder.jit(f, cache=cache)
    got = jf(a, a[0, :], a[1, :])
    exp = f(a_, a_[0, :], a_[1, :])
    torch.testing.assert_close(got, exp)
    torch.testing.assert_close(a, a_)


def test_nn_module_inplace_activation():
    m = torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.ReLU(inplace=True), torch.nn.Linear(4, 2))
    x = _x(3, 4)
    jm = thunder.jit(m)
    torch.testing.assert_close(jm(x), m(x))


def test_inplace_grad_through_view():
    def f(a):
        t = a * 1.0
        t[:, 0].mul_(2.0)
        return (t * t).sum()

    x = _x(3, 3)
    xe = x.clone().requires_grad_(True)
    xg = x.clone().requires_grad_(True)
    f(xe).backward()
    thunder.jit(f)(xg).backward()
    torch.testing.assert_close(xg.grad, xe.grad)
