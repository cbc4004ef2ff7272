"""Reduction / shape-op / elementwise batteries through ``thunder.jit`` vs eager PyTorch on CPU.

Parity: the reference's ``thunder/tests/test_reductions.py`` (var / std corrections, keepdim, tuple
dims, arg-reductions), ``test_shape_ops.py`` (views, splits, pads, movedim, unfold) and
``test_elementwise.py`` (type promotion, scalar operands, integer division semantics).  Every case
runs the traced program and compares values, dtypes and shapes to eager; where a gradient is defined
the backward is compared too (fp64, tight tolerances).
"""
import pytest
import torch

import lightning_thunder_amd as thunder


def _check(fn, *args, grad=True, atol=1e-10, rtol=1e-8):
    jf = thunder.jit(fn)
    exp = fn(*args)
    got = jf(*args)
    exp_l = exp if isinstance(exp, (tuple, list)) else (exp,)
    got_l = got if isinstance(got, (tuple, list)) else (got,)
    assert len(exp_l) == len(got_l)
    for e, g in zip(exp_l, got_l):
        assert g.shape == e.shape, (g.shape, e.shape)
        assert g.dtype == e.dtype, (g.dtype, e.dtype)
        torch.testing.assert_close(g, e, atol=atol, rtol=rtol, equal_nan=True)
    if not grad:
        return
    fl = [a for a in args if isinstance(a, torch.Tensor) and a.is_floating_point()]
    if not fl:
        return
    ins_e = [a.detach().clone().requires_grad_(True) if isinstance(a, torch.Tensor) and a.is_floating_point() else a
             for a in args]
    ins_g = [a.detach().clone().requires_grad_(True) if isinstance(a, torch.Tensor) and a.is_floating_point() else a
             for a in args]
    oe = fn(*ins_e)
    og = jf(*ins_g)
    oe = oe if isinstance(oe, (tuple, list)) else (oe,)
    og = og if isinstance(og, (tuple, list)) else (og,)
    le = sum((o.float() * (i + 1)).sum() for i, o in enumerate(oe) if o.is_floating_point())
    lg = sum((o.float() * (i + 1)).sum() for i, o in enumerate(og) if o.is_floating_point())
    if not isinstance(le, torch.Tensor) or not le.requires_grad:
        return
    le.backward()
    lg.backward()
    for a, b in zip(ins_e, ins_g):
        if isinstance(a, torch.Tensor) and a.requires_grad:
            ga = torch.zeros_like(a) if a.grad is None else a.grad
            gb = torch.zeros_like(b) if b.grad is None else b.grad
            torch.testing.assert_close(gb, ga, atol=1e-9, rtol=1e-7)


def _x(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g, dtype=torch.float64)


# ---------------------------------------------------------------- reductions (test_reductions.py)

@pytest.mark.parametrize("correction", [0, 1, 2])
@pytest.mark.parametrize("dim,keepdim", [(None, False), (1, False), (1, True), ((0, 2), False), ((0, 2), True), (-1, True)])
def test_var_std_corrections(correction, dim, keepdim):
    x = _x(4, 5, 6)
    _check(lambda a: torch.var(a, dim=dim, correction=correction, keepdim=keepdim), x)
    _check(lambda a: torch.std(a, dim=dim, correction=correction, keepdim=keepdim), x)


@pytest.mark.parametrize("dim", [0, 1, -1])
def test_var_mean_pair(dim):
    _check(lambda a: torch.var_mean(a, dim=dim, correction=1), _x(6, 7))


@pytest.mark.parametrize("op", ["sum", "mean", "amax", "amin", "prod"])
@pytest.mark.parametrize("dim,keepdim", [(0, False), (-1, True), ((0, 1), False), ((1, 2), True)])
def test_reductions_dims(op, dim, keepdim):
    x = _x(3, 4, 5) * 0.5 + 1.0
    f = getattr(torch, op)
    if op == "prod":
        if isinstance(dim, tuple):
            pytest.skip("torch.prod takes a single dim")
        _check(lambda a: f(a, dim, keepdim=keepdim), x)
    else:
        _check(lambda a: f(a, dim, keepdim=keepdim), x)


@pytest.mark.parametrize("op", ["argmax", "argmin"])
@pytest.mark.parametrize("dim,keepdim", [(None, False), (0, False), (1, True), (-1, False)])
def test_arg_reductions(op, dim, keepdim):
    x = _x(5, 7)
    f = getattr(torch, op)
    _check(lambda a: f(a, dim=dim, keepdim=keepdim), x, grad=False)


def test_sum_dtype_and_integer_promotion():
    xi = torch.arange(24, dtype=torch.int32).reshape(4, 6)
    _check(lambda a: torch.sum(a, 1), xi, grad=False)  # int32 sums promote to int64
    _check(lambda a: torch.sum(a, 0, dtype=torch.float64), xi, grad=False)
    xb = torch.tensor([[True, False, True], [True, True, True]])
    _check(lambda a: a.sum(-1), xb, grad=False)
    _check(lambda a: (a.all(-1), a.any(0)), xb, grad=False)


def test_cumulative_and_norms():
    x = _x(4, 6)
    _check(lambda a: torch.cumsum(a, 1), x)
    _check(lambda a: torch.linalg.vector_norm(a, 2, dim=-1), x)
    _check(lambda a: torch.logsumexp(a, 0), x)
    _check(lambda a: torch.softmax(a, -1), x)
    _check(lambda a: torch.log_softmax(a, 0), x)


# ---------------------------------------------------------------- shape ops (test_shape_ops.py)

def test_reshape_view_flatten():
    x = _x(2, 3, 4)
    _check(lambda a: a.reshape(-1, 4), x)
    _check(lambda a: a.view(6, 4).t(), x)
    _check(lambda a: torch.flatten(a, 1), x)
    _check(lambda a: a.unflatten(-1, (2, 2)), x)
    _check(lambda a: a.reshape(4, -1).contiguous(), x.transpose(0, 2))


def test_permutes_and_moves():
    x = _x(2, 3, 4, 5)
    _check(lambda a: a.permute(3, 1, 0, 2), x)
    _check(lambda a: torch.movedim(a, 1, -1), x)
    _check(lambda a: torch.movedim(a, (0, 1), (2, 3)), x)
    _check(lambda a: a.transpose(-1, -3), x)
    _check(lambda a: a.mT, x)


def test_squeeze_unsqueeze_expand():
    x = _x(1, 3, 1, 4)
    _check(lambda a: a.squeeze(), x)
    _check(lambda a: a.squeeze(0), x)
    _check(lambda a: a.squeeze((0, 2)), x)
    _check(lambda a: a.unsqueeze(-1).unsqueeze(0), x)
    _check(lambda a: a.expand(2, 3, 5, 4) * 1.0, x)
    _check(lambda a: a.expand_as(torch.empty(6, 3, 2, 4)) + 0.0, x)


@pytest.mark.parametrize("how", ["split_int", "split_list", "chunk", "tensor_split", "unbind"])
def test_splits(how):
    x = _x(7, 6)
    fns = {
        "split_int": lambda a: torch.split(a, 3, dim=0),
        "split_list": lambda a: torch.split(a, [1, 2, 3], dim=1),
        "chunk": lambda a: torch.chunk(a, 3, dim=0),
        "tensor_split": lambda a: torch.tensor_split(a, [2, 5], dim=0),
        "unbind": lambda a: torch.unbind(a, 1),
    }
    _check(fns[how], x)


def test_cat_stack_and_friends():
    a, b = _x(2, 3), _x(2, 3, seed=1)
    _check(lambda p, q: torch.cat([p, q], 0), a, b)
    _check(lambda p, q: torch.cat([p, q], -1), a, b)
    _check(lambda p, q: torch.stack([p, q], 1), a, b)
    _check(lambda p, q: torch.hstack([p, q]), a, b)
    _check(lambda p, q: torch.vstack([p, q]), a, b)


def test_slicing_and_indexing_views():
    x = _x(6, 8)
    _check(lambda a: a[1:5:2, ::3], x)
    _check(lambda a: a[..., -3:], x)
    _check(lambda a: a[None, 2, :, None], x)
    _check(lambda a: torch.narrow(a, 1, 2, 4), x)
    _check(lambda a: a.flip(0, 1), x)
    _check(lambda a: torch.roll(a, 3, 1), x)
    _check(lambda a: torch.roll(a, (1, -2), (0, 1)), x)


def test_pad_and_unfold():
    x = _x(2, 3, 5)
    _check(lambda a: torch.nn.functional.pad(a, (1, 2)), x)
    _check(lambda a: torch.nn.functional.pad(a, (0, 1, 2, 0), value=0.5), x)
    _check(lambda a: a.unfold(-1, 2, 1), x)


def test_gather_take_along_dim_index_select():
    x = _x(4, 5)
    idx = torch.tensor([[0, 4], [1, 3], [2, 2], [4, 0]])
    _check(lambda a: torch.gather(a, 1, idx), x)
    _check(lambda a: torch.take_along_dim(a, idx, 1), x)
    _check(lambda a: torch.index_select(a, 0, torch.tensor([3, 0, 3])), x)


# ---------------------------------------------------------------- elementwise (test_elementwise.py)

@pytest.mark.parametrize("op", ["add", "sub", "mul", "true_divide", "maximum", "minimum", "atan2", "pow"])
def test_binary_float(op):
    a, b = _x(3, 4), _x(3, 4, seed=1)
    if op == "pow":
        a = a.abs() + 0.5
    _check(lambda p, q: getattr(torch, op)(p, q), a, b)


@pytest.mark.parametrize("rounding_mode", [None, "trunc", "floor"])
def test_integer_division_semantics(rounding_mode):
    a = torch.tensor([7, -7, 9, -9, 0], dtype=torch.int64)
    b = torch.tensor([2, 2, -4, -4, 3], dtype=torch.int64)
    _check(lambda p, q: torch.div(p, q, rounding_mode=rounding_mode), a, b, grad=False)
    _check(lambda p, q: (p % q, torch.remainder(p, q), torch.fmod(p, q)), a, b, grad=False)


def test_scalar_operands_and_promotion():
    xi = torch.arange(6, dtype=torch.int32)
    xh = torch.arange(6, dtype=torch.float16)
    _check(lambda a: a * 2.5, xi, grad=False)        # int tensor * float scalar -> default float
    _check(lambda a: a + 3, xh, grad=False)          # half tensor + int scalar stays half
    _check(lambda a, b: a + b, xi, xh, grad=False)   # int32 + half -> half
    _check(lambda a: (a > 2) & (a < 5), xi, grad=False)
    _check(lambda a: torch.where(a > 2, a, 0), xi, grad=False)


@pytest.mark.parametrize("op", ["exp", "log1p", "tanh", "sigmoid", "erf", "rsqrt", "sin", "cos", "abs", "reciprocal"])
def test_unary_float(op):
    x = _x(5, 3)
    if op in ("log1p", "rsqrt", "reciprocal"):
        x = x.abs() + 0.25
    _check(lambda a: getattr(torch, op)(a), x)


def test_clamp_and_lerp():
    x, y = _x(4, 4), _x(4, 4, seed=2)
    _check(lambda a: torch.clamp(a, -0.5, 0.5), x)
    _check(lambda a: a.clamp(min=0.0), x)
    _check(lambda a, b: torch.lerp(a, b, 0.3), x, y)
