"""OpInfo table: sample inputs + torch reference for the ltorch operator library.

Parity: reference ``thunder/tests/opinfos.py`` (``OpInfo`` :138, sample generators, dtypes,
``DecorateInfo`` skips).  Each :class:`OpInfo` gives a callable to compile (``op``), a sample
generator ``samples(device, dtype, requires_grad)`` yielding ``SampleInput``s, the dtypes it
supports and whether it is differentiable.  The torch reference is the op itself run eagerly
(float64 for gradient checks).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable

import torch
import torch.nn.functional as F


@dataclass
class SampleInput:
    args: tuple
    kwargs: dict = field(default_factory=dict)

    def __repr__(self):
        def r(x):
            if isinstance(x, torch.Tensor):
                return f"T{tuple(x.shape)}:{str(x.dtype).split('.')[-1]}"
            return repr(x)

        return "(" + ", ".join([r(a) for a in self.args] + [f"{k}={r(v)}" for k, v in self.kwargs.items()]) + ")"


FLOATS = (torch.float32, torch.bfloat16, torch.float16)
FLOAT32 = (torch.float32,)
INTS = (torch.int64, torch.int32)


@dataclass
class OpInfo:
    name: str
    op: Callable
    samples: Callable
    dtypes: tuple = FLOATS
    differentiable: bool = True
    atol: float | None = None
    rtol: float | None = None
    skip_gpu: bool = False
    grad_atol: float = 1e-6

    def __repr__(self):
        return self.name


def _t(shape, device, dtype, requires_grad=False, low=-2.0, high=2.0):
    if dtype.is_floating_point:
        x = torch.empty(shape, device=device, dtype=torch.float32).uniform_(low, high).to(dtype)
    elif dtype == torch.bool:
        x = torch.rand(shape, device=device) > 0.5
    else:
        x = torch.randint(int(low) if low > -100 else -5, int(high) + 1 if high < 100 else 6, shape, device=device, dtype=dtype)
    if requires_grad and dtype.is_floating_point:
        x.requires_grad_(True)
    return x


SHAPES = [(5,), (3, 4), (2, 3, 5)]


def unary_samples(low=-2.0, high=2.0, shapes=SHAPES):
    def gen(device, dtype, requires_grad):
        for s in shapes:
            yield SampleInput((_t(s, device, dtype, requires_grad, low, high),))

    return gen


def binary_samples(low=-2.0, high=2.0, rhs_low=None, rhs_high=None, scalar=True):
    rl = low if rhs_low is None else rhs_low
    rh = high if rhs_high is None else rhs_high

    def gen(device, dtype, requires_grad):
        yield SampleInput((_t((3, 4), device, dtype, requires_grad, low, high), _t((3, 4), device, dtype, requires_grad, rl, rh)))
        yield SampleInput((_t((2, 3, 4), device, dtype, requires_grad, low, high), _t((3, 1), device, dtype, requires_grad, rl, rh)))
        if scalar:
            yield SampleInput((_t((4,), device, dtype, requires_grad, low, high), (rl + rh) / 2 + 0.75))

    return gen


def reduction_samples(dims=(None, 0, -1, (0, 1)), keepdim=(False, True), extra=None):
    def gen(device, dtype, requires_grad):
        x = _t((3, 4, 5), device, dtype, requires_grad)
        for d in dims:
            for k in keepdim:
                kw = {} if d is None else {"dim": d, "keepdim": k}
                if d is None and k:
                    continue
                kw.update(extra or {})
                yield SampleInput((x,), kw)

    return gen


def _pos(shapes=SHAPES):
    return unary_samples(0.1, 3.0, shapes)


def elementwise_unary(name, fn, low=-2.0, high=2.0, dtypes=FLOATS, differentiable=True, **kw):
    return OpInfo(name, fn, unary_samples(low, high), dtypes=dtypes, differentiable=differentiable, **kw)


def elementwise_binary(name, fn, dtypes=FLOATS, differentiable=True, **kw):
    s = kw.pop("samples", None) or binary_samples(**kw.pop("sample_kw", {}))
    return OpInfo(name, fn, s, dtypes=dtypes, differentiable=differentiable, **kw)


def _shape_samples(fn_args):
    def gen(device, dtype, requires_grad):
        for shape, args, kwargs in fn_args:
            yield SampleInput((_t(shape, device, dtype, requires_grad),) + tuple(args), dict(kwargs))

    return gen


def _matmul_samples(device, dtype, requires_grad):
    yield SampleInput((_t((3, 4), device, dtype, requires_grad), _t((4, 5), device, dtype, requires_grad)))
    yield SampleInput((_t((2, 3, 4), device, dtype, requires_grad), _t((4, 5), device, dtype, requires_grad)))
    yield SampleInput((_t((2, 3, 4), device, dtype, requires_grad), _t((2, 4, 5), device, dtype, requires_grad)))
    yield SampleInput((_t((4,), device, dtype, requires_grad), _t((4, 3), device, dtype, requires_grad)))


def _linear_samples(device, dtype, requires_grad):
    yield SampleInput((_t((3, 4), device, dtype, requires_grad), _t((5, 4), device, dtype, requires_grad)))
    yield SampleInput((_t((2, 3, 4), device, dtype, requires_grad), _t((5, 4), device, dtype, requires_grad),
                       _t((5,), device, dtype, requires_grad)))


def _norm_samples(kind):
    def gen(device, dtype, requires_grad):
        x = _t((2, 3, 8), device, dtype, requires_grad)
        w = _t((8,), device, dtype, requires_grad, 0.5, 1.5)
        b = _t((8,), device, dtype, requires_grad)
        if kind == "layer_norm":
            yield SampleInput((x, (8,)), {})
            yield SampleInput((x, (8,), w, b), {"eps": 1e-5})
        else:
            yield SampleInput((x, (8,)), {"eps": 1e-6})
            yield SampleInput((x, (8,), w), {"eps": 1e-6})

    return gen


def _softmax_samples(device, dtype, requires_grad):
    x = _t((3, 4, 5), device, dtype, requires_grad)
    for d in (0, -1, 1):
        yield SampleInput((x,), {"dim": d})


def _ce_samples(device, dtype, requires_grad):
    logits = _t((6, 10), device, dtype, requires_grad)
    tgt = torch.randint(0, 10, (6,), device=device)
    yield SampleInput((logits, tgt))
    tgt2 = tgt.clone()
    tgt2[1] = -100
    yield SampleInput((logits, tgt2), {"ignore_index": -100})
    yield SampleInput((logits, tgt), {"label_smoothing": 0.1})
    yield SampleInput((logits, tgt), {"reduction": "sum"})


def _sdpa_samples(device, dtype, requires_grad):
    q = _t((1, 2, 8, 16), device, dtype, requires_grad)
    k = _t((1, 2, 8, 16), device, dtype, requires_grad)
    v = _t((1, 2, 8, 16), device, dtype, requires_grad)
    yield SampleInput((q, k, v), {"is_causal": True})
    yield SampleInput((q, k, v), {})


def _embedding_samples(device, dtype, requires_grad):
    idx = torch.randint(0, 10, (3, 4), device=device)
    w = _t((10, 6), device, dtype, requires_grad)
    yield SampleInput((idx, w))


def _where_samples(device, dtype, requires_grad):
    c = torch.rand(3, 4, device=device) > 0.5
    yield SampleInput((c, _t((3, 4), device, dtype, requires_grad), _t((3, 4), device, dtype, requires_grad)))
    yield SampleInput((c, _t((3, 4), device, dtype, requires_grad), 0.5))


def _cat_samples(device, dtype, requires_grad):
    a, b = _t((2, 3), device, dtype, requires_grad), _t((4, 3), device, dtype, requires_grad)
    yield SampleInput(([a, b],), {"dim": 0})
    c = _t((2, 5), device, dtype, requires_grad)
    yield SampleInput(([a, c],), {"dim": 1})


def _stack_samples(device, dtype, requires_grad):
    a, b = _t((2, 3), device, dtype, requires_grad), _t((2, 3), device, dtype, requires_grad)
    yield SampleInput(([a, b],), {"dim": 0})
    yield SampleInput(([a, b],), {"dim": -1})


def _getitem_samples(device, dtype, requires_grad):
    x = _t((4, 5, 6), device, dtype, requires_grad)
    for key in (1, (slice(1, 3), 2), (Ellipsis, 0), (slice(None), None, slice(0, 4, 2)), -1):
        yield SampleInput((x, key))


def _gather_samples(device, dtype, requires_grad):
    x = _t((3, 5), device, dtype, requires_grad)
    idx = torch.randint(0, 5, (3, 2), device=device)
    yield SampleInput((x, 1, idx))


def _index_select_samples(device, dtype, requires_grad):
    x = _t((4, 5), device, dtype, requires_grad)
    yield SampleInput((x, 0, torch.tensor([0, 2, 3], device=device)))
    yield SampleInput((x, 1, torch.tensor([4, 1], device=device)))


def _masked_fill_samples(device, dtype, requires_grad):
    x = _t((3, 4), device, dtype, requires_grad)
    m = torch.rand(3, 4, device=device) > 0.5
    yield SampleInput((x, m, -1.5))


def _clamp_samples(device, dtype, requires_grad):
    x = _t((3, 4), device, dtype, requires_grad)
    yield SampleInput((x,), {"min": -0.5, "max": 0.5})
    yield SampleInput((x,), {"min": -0.3})


def _pad_samples(device, dtype, requires_grad):
    x = _t((2, 3, 4), device, dtype, requires_grad)
    yield SampleInput((x, (1, 2)))
    yield SampleInput((x, (1, 0, 0, 2)), {"value": 0.5})


def _topk_samples(device, dtype, requires_grad):
    x = _t((3, 6), device, dtype, requires_grad)
    yield SampleInput((x, 2))
    yield SampleInput((x, 3), {"dim": 0})


def _cumsum_samples(device, dtype, requires_grad):
    x = _t((3, 4), device, dtype, requires_grad)
    yield SampleInput((x, 0))
    yield SampleInput((x, -1))


def _einsum_samples(device, dtype, requires_grad):
    a, b = _t((2, 3), device, dtype, requires_grad), _t((3, 4), device, dtype, requires_grad)
    yield SampleInput(("ij,jk->ik", a, b))
    c = _t((2, 3, 4), device, dtype, requires_grad)
    yield SampleInput(("bij->bji", c))


def _mse_samples(device, dtype, requires_grad):
    yield SampleInput((_t((3, 4), device, dtype, requires_grad), _t((3, 4), device, dtype, requires_grad)))


def _group_norm_samples(device, dtype, requires_grad):
    x = _t((2, 4, 3, 3), device, dtype, requires_grad)
    yield SampleInput((x, 2), {"weight": _t((4,), device, dtype, requires_grad), "bias": _t((4,), device, dtype, requires_grad)})


def _split_samples(device, dtype, requires_grad):
    x = _t((6, 4), device, dtype, requires_grad)
    yield SampleInput((x, 2))
    yield SampleInput((x, [1, 5]))
    yield SampleInput((x, 2), {"dim": 1})


def _bce_samples(device, dtype, requires_grad):
    yield SampleInput((_t((3, 4), device, dtype, requires_grad), torch.rand(3, 4, device=device, dtype=dtype)))


def _scatter_add_samples(device, dtype, requires_grad):
    x = _t((3, 5), device, dtype, requires_grad)
    idx = torch.randint(0, 5, (3, 2), device=device)
    src = _t((3, 2), device, dtype, requires_grad)
    yield SampleInput((x, 1, idx, src))


def _index_add_samples(device, dtype, requires_grad):
    x = _t((5, 3), device, dtype, requires_grad)
    idx = torch.tensor([0, 2, 2], device=device)
    src = _t((3, 3), device, dtype, requires_grad)
    yield SampleInput((x, 0, idx, src))


OPS: list[OpInfo] = [
    # ---- unary elementwise ----
    elementwise_unary("abs", torch.abs),
    elementwise_unary("neg", torch.neg),
    elementwise_unary("exp", torch.exp),
    elementwise_unary("exp2", torch.exp2),
    elementwise_unary("expm1", torch.expm1),
    elementwise_unary("log", torch.log, 0.1, 3.0),
    elementwise_unary("log2", torch.log2, 0.1, 3.0),
    elementwise_unary("log10", torch.log10, 0.1, 3.0),
    elementwise_unary("log1p", torch.log1p, -0.5, 3.0),
    elementwise_unary("sqrt", torch.sqrt, 0.1, 3.0),
    elementwise_unary("rsqrt", torch.rsqrt, 0.1, 3.0),
    elementwise_unary("reciprocal", torch.reciprocal, 0.5, 3.0),
    elementwise_unary("sin", torch.sin),
    elementwise_unary("cos", torch.cos),
    elementwise_unary("tan", torch.tan, -1.0, 1.0),
    elementwise_unary("asin", torch.asin, -0.9, 0.9),
    elementwise_unary("acos", torch.acos, -0.9, 0.9),
    elementwise_unary("atan", torch.atan),
    elementwise_unary("sinh", torch.sinh),
    elementwise_unary("cosh", torch.cosh),
    elementwise_unary("tanh", torch.tanh),
    elementwise_unary("asinh", torch.asinh),
    elementwise_unary("acosh", torch.acosh, 1.1, 3.0),
    elementwise_unary("atanh", torch.atanh, -0.9, 0.9),
    elementwise_unary("sigmoid", torch.sigmoid),
    elementwise_unary("erf", torch.erf),
    elementwise_unary("erfc", torch.erfc),
    elementwise_unary("erfinv", torch.erfinv, -0.9, 0.9),
    elementwise_unary("lgamma", torch.lgamma, 0.5, 3.0),
    elementwise_unary("digamma", torch.digamma, 0.5, 3.0),
    elementwise_unary("square", torch.square),
    elementwise_unary("sign", torch.sign, differentiable=False),
    elementwise_unary("floor", torch.floor, differentiable=False),
    elementwise_unary("ceil", torch.ceil, differentiable=False),
    elementwise_unary("round", torch.round, differentiable=False),
    elementwise_unary("trunc", torch.trunc, differentiable=False),
    elementwise_unary("isnan", torch.isnan, differentiable=False),
    elementwise_unary("isfinite", torch.isfinite, differentiable=False),
    elementwise_unary("relu", F.relu),
    elementwise_unary("relu6", F.relu6, -7.0, 7.0),
    elementwise_unary("gelu", F.gelu),
    elementwise_unary("gelu_tanh", lambda x: F.gelu(x, approximate="tanh")),
    elementwise_unary("silu", F.silu),
    elementwise_unary("mish", F.mish),
    elementwise_unary("elu", F.elu),
    elementwise_unary("leaky_relu", lambda x: F.leaky_relu(x, 0.2)),
    elementwise_unary("softplus", F.softplus),
    elementwise_unary("hardswish", F.hardswish),
    elementwise_unary("hardtanh", F.hardtanh),
    elementwise_unary("logsigmoid", F.logsigmoid),
    elementwise_unary("nan_to_num", torch.nan_to_num),
    elementwise_unary("bitwise_not", torch.bitwise_not, dtypes=INTS, differentiable=False),
    OpInfo("clamp", torch.clamp, _clamp_samples),
    OpInfo("pow_scalar", lambda x: torch.pow(x, 3), unary_samples()),
    OpInfo("pow_frac", lambda x: x ** 0.5, unary_samples(0.1, 3.0)),
    # ---- binary elementwise ----
    elementwise_binary("add", torch.add),
    elementwise_binary("add_alpha", lambda a, b: torch.add(a, b, alpha=2), samples=binary_samples(scalar=False)),
    elementwise_binary("sub", torch.sub),
    elementwise_binary("mul", torch.mul),
    elementwise_binary("div", torch.div, sample_kw=dict(rhs_low=0.5, rhs_high=2.0)),
    elementwise_binary("div_floor", lambda a, b: torch.div(a, b, rounding_mode="floor"), differentiable=False,
                       sample_kw=dict(rhs_low=0.5, rhs_high=2.0)),
    elementwise_binary("remainder", torch.remainder, differentiable=False, sample_kw=dict(rhs_low=0.5, rhs_high=2.0)),
    elementwise_binary("fmod", torch.fmod, differentiable=False, sample_kw=dict(rhs_low=0.5, rhs_high=2.0)),
    elementwise_binary("pow", torch.pow, sample_kw=dict(low=0.5, high=2.0, rhs_low=-1.0, rhs_high=2.0)),
    elementwise_binary("maximum", torch.maximum, samples=binary_samples(scalar=False)),
    elementwise_binary("minimum", torch.minimum, samples=binary_samples(scalar=False)),
    elementwise_binary("atan2", torch.atan2, samples=binary_samples(scalar=False)),
    elementwise_binary("copysign", torch.copysign, samples=binary_samples(scalar=False)),
    elementwise_binary("eq", torch.eq, differentiable=False),
    elementwise_binary("ne", torch.ne, differentiable=False),
    elementwise_binary("lt", torch.lt, differentiable=False),
    elementwise_binary("le", torch.le, differentiable=False),
    elementwise_binary("gt", torch.gt, differentiable=False),
    elementwise_binary("ge", torch.ge, differentiable=False),
    elementwise_binary("bitwise_and", torch.bitwise_and, dtypes=INTS, differentiable=False,
                       samples=binary_samples(scalar=False)),
    elementwise_binary("bitwise_xor", torch.bitwise_xor, dtypes=INTS, differentiable=False,
                       samples=binary_samples(scalar=False)),
    elementwise_binary("int_add", torch.add, dtypes=INTS, differentiable=False, samples=binary_samples(scalar=False)),
    OpInfo("lerp", torch.lerp, lambda d, t, r: iter([SampleInput((_t((3, 4), d, t, r), _t((3, 4), d, t, r), 0.3))])),
    OpInfo("addcmul", lambda a, b, c: torch.addcmul(a, b, c, value=0.5),
           lambda d, t, r: iter([SampleInput((_t((3, 4), d, t, r), _t((3, 4), d, t, r), _t((3, 4), d, t, r)))])),
    OpInfo("addcdiv", lambda a, b, c: torch.addcdiv(a, b, c, value=0.5),
           lambda d, t, r: iter([SampleInput((_t((3, 4), d, t, r), _t((3, 4), d, t, r), _t((3, 4), d, t, r, 0.5, 2.0)))])),
    OpInfo("where", torch.where, _where_samples),
    OpInfo("masked_fill", torch.masked_fill, _masked_fill_samples),
    # ---- reductions ----
    OpInfo("sum", torch.sum, reduction_samples()),
    OpInfo("mean", torch.mean, reduction_samples()),
    OpInfo("prod", lambda x, **k: torch.prod(x, **k) if k else torch.prod(x), reduction_samples(dims=(None, 1))),
    OpInfo("amax", torch.amax, reduction_samples(dims=(0, -1, (0, 1)))),
    OpInfo("amin", torch.amin, reduction_samples(dims=(0, -1))),
    OpInfo("var", torch.var, reduction_samples(dims=(None, 0, -1))),
    OpInfo("var_unbiased0", lambda x, **k: torch.var(x, correction=0, **k), reduction_samples(dims=(None, 1))),
    OpInfo("std", torch.std, reduction_samples(dims=(None, 1))),
    OpInfo("logsumexp", lambda x, dim=-1, keepdim=False: torch.logsumexp(x, dim, keepdim), reduction_samples(dims=(0, -1))),
    OpInfo("argmax", torch.argmax, reduction_samples(dims=(0, -1)), differentiable=False),
    OpInfo("argmin", torch.argmin, reduction_samples(dims=(0, -1)), differentiable=False),
    OpInfo("any", lambda x: torch.any(x > 0), unary_samples(), differentiable=False),
    OpInfo("all", lambda x: torch.all(x > -10), unary_samples(), differentiable=False),
    OpInfo("cumsum", torch.cumsum, _cumsum_samples),
    OpInfo("topk_values", lambda x, k, **kw: torch.topk(x, k, **kw).values, _topk_samples),
    OpInfo("sort_values", lambda x: torch.sort(x, -1).values, unary_samples(shapes=[(3, 6)])),
    # ---- shape ops ----
    OpInfo("reshape", torch.reshape, _shape_samples([((3, 4), ((12,),), {}), ((2, 3, 4), ((6, -1),), {})])),
    OpInfo("view", lambda x, s: x.view(s), _shape_samples([((3, 4), ((4, 3),), {})])),
    OpInfo("transpose", torch.transpose, _shape_samples([((3, 4), (0, 1), {}), ((2, 3, 4), (-1, 0), {})])),
    OpInfo("permute", torch.permute, _shape_samples([((2, 3, 4), ((2, 0, 1),), {})])),
    OpInfo("unsqueeze", torch.unsqueeze, _shape_samples([((3, 4), (1,), {}), ((3,), (-1,), {})])),
    OpInfo("squeeze", torch.squeeze, _shape_samples([((3, 1, 4), (1,), {}), ((1, 3, 1), (), {})])),
    OpInfo("flatten", torch.flatten, _shape_samples([((2, 3, 4), (1,), {}), ((2, 3, 4), (), {})])),
    OpInfo("expand", lambda x, *s: x.expand(*s), _shape_samples([((3, 1), (3, 4), {}), ((4,), (2, 4), {})])),
    OpInfo("repeat", lambda x, *s: x.repeat(*s), _shape_samples([((2, 3), (2, 1), {})])),
    OpInfo("flip", torch.flip, _shape_samples([((3, 4), ((0,),), {}), ((3, 4), ((0, 1),), {})])),
    OpInfo("roll", torch.roll, _shape_samples([((3, 4), (1, 1), {})])),
    OpInfo("narrow", torch.narrow, _shape_samples([((4, 5), (1, 1, 3), {})])),
    OpInfo("movedim", torch.movedim, _shape_samples([((2, 3, 4), (0, 2), {})])),
    OpInfo("tril", torch.tril, unary_samples(shapes=[(4, 4), (3, 5)])),
    OpInfo("triu", lambda x: torch.triu(x, 1), unary_samples(shapes=[(4, 4)])),
    OpInfo("cat", torch.cat, _cat_samples),
    OpInfo("stack", torch.stack, _stack_samples),
    OpInfo("split", lambda x, s, **k: torch.split(x, s, **k), _split_samples),
    OpInfo("chunk", lambda x: torch.chunk(x, 3, 0), unary_samples(shapes=[(6, 2)])),
    OpInfo("unbind", lambda x: torch.unbind(x, 1), unary_samples(shapes=[(2, 3)])),
    OpInfo("getitem", lambda x, k: x[k], _getitem_samples),
    OpInfo("pad", F.pad, _pad_samples),
    OpInfo("contiguous_T", lambda x: x.t().contiguous().view(-1), unary_samples(shapes=[(3, 4)])),
    OpInfo("to_dtype", lambda x: x.to(torch.float64).sum(-1), unary_samples()),
    # ---- indexing ----
    OpInfo("gather", torch.gather, _gather_samples),
    OpInfo("index_select", torch.index_select, _index_select_samples),
    OpInfo("take_along_dim", lambda x, i: torch.take_along_dim(x, i, 1),
           lambda d, t, r: iter([SampleInput((_t((3, 5), d, t, r), torch.randint(0, 5, (3, 2), device=d)))])),
    OpInfo("scatter_add", torch.scatter_add, _scatter_add_samples),
    OpInfo("index_add", torch.index_add, _index_add_samples),
    OpInfo("embedding", F.embedding, _embedding_samples),
    OpInfo("one_hot", lambda i: F.one_hot(i, 7), lambda d, t, r: iter([SampleInput((torch.randint(0, 7, (3, 4), device=d),))]),
           dtypes=(torch.int64,), differentiable=False),
    # ---- linear algebra ----
    OpInfo("matmul", torch.matmul, _matmul_samples, atol=1e-2, rtol=1e-2),
    OpInfo("linear", F.linear, _linear_samples, atol=1e-2, rtol=1e-2),
    OpInfo("bmm", torch.bmm, lambda d, t, r: iter([SampleInput((_t((2, 3, 4), d, t, r), _t((2, 4, 5), d, t, r)))]),
           atol=1e-2, rtol=1e-2),
    OpInfo("addmm", torch.addmm, lambda d, t, r: iter([SampleInput((_t((3, 5), d, t, r), _t((3, 4), d, t, r), _t((4, 5), d, t, r)))]),
           atol=1e-2, rtol=1e-2),
    OpInfo("outer", torch.outer, lambda d, t, r: iter([SampleInput((_t((3,), d, t, r), _t((4,), d, t, r)))])),
    OpInfo("einsum", torch.einsum, _einsum_samples, atol=1e-2, rtol=1e-2),
    # ---- nn ----
    OpInfo("softmax", F.softmax, _softmax_samples),
    OpInfo("log_softmax", F.log_softmax, _softmax_samples),
    OpInfo("layer_norm", F.layer_norm, _norm_samples("layer_norm"), atol=2e-2, rtol=2e-2),
    OpInfo("rms_norm", F.rms_norm, _norm_samples("rms_norm"), atol=2e-2, rtol=2e-2),
    OpInfo("group_norm", F.group_norm, _group_norm_samples, atol=2e-2, rtol=2e-2),
    OpInfo("cross_entropy", F.cross_entropy, _ce_samples, atol=2e-2, rtol=2e-2),
    OpInfo("mse_loss", F.mse_loss, _mse_samples),
    OpInfo("l1_loss", F.l1_loss, _mse_samples),
    OpInfo("bce_with_logits", F.binary_cross_entropy_with_logits, _bce_samples),
    OpInfo("sdpa", F.scaled_dot_product_attention, _sdpa_samples, atol=2e-2, rtol=2e-2),
    OpInfo("normalize", F.normalize, unary_samples(shapes=[(3, 4)])),
]

OPS_BY_NAME = {o.name: o for o in OPS}


# =========================================================================================
# Convolution / pooling / normalization / activations / shape utilities (torch/nn_ops.py)
# =========================================================================================
def _conv_samples(n):
    def gen(device, dtype, requires_grad):
        sp = (7,) * n
        x = _t((2, 4) + sp, device, dtype, requires_grad)
        w = _t((6, 4) + (3,) * n, device, dtype, requires_grad)
        b = _t((6,), device, dtype, requires_grad)
        yield SampleInput((x, w, b))
        yield SampleInput((x, w), {"stride": 2, "padding": 1})
        yield SampleInput((x, w, b), {"padding": "same", "dilation": 2})
        wg = _t((6, 2) + (2,) * n, device, dtype, requires_grad)
        yield SampleInput((x, wg), {"groups": 2, "padding": "same"})  # even kernel: asymmetric 'same'

    return gen


def _pool_samples(n, kind):
    def gen(device, dtype, requires_grad):
        x = _t((2, 3) + (9,) * n, device, dtype, requires_grad)
        yield SampleInput((x, 3))
        yield SampleInput((x, 3), {"stride": 2, "padding": 1})
        if kind == "max":
            yield SampleInput((x, 2), {"stride": 2, "dilation": 2})
            yield SampleInput((x, 3), {"stride": 2, "ceil_mode": True})
        else:
            yield SampleInput((x, 3), {"stride": 2, "padding": 1, "count_include_pad": False})

    return gen


def _bn_samples(training):
    def gen(device, dtype, requires_grad):
        x = _t((4, 3, 5, 5), device, dtype, requires_grad)
        w = _t((3,), device, dtype, requires_grad, 0.5, 1.5)
        b = _t((3,), device, dtype, requires_grad)
        rm = torch.zeros(3, device=device, dtype=dtype)
        rv = torch.ones(3, device=device, dtype=dtype)
        yield SampleInput((x, rm.clone(), rv.clone(), w, b), {"training": training})
        yield SampleInput((x, rm.clone(), rv.clone()), {"training": training, "momentum": 0.2, "eps": 1e-3})

    return gen


def _interp_samples(mode, n):
    def gen(device, dtype, requires_grad):
        x = _t((2, 3) + (5,) * n, device, dtype, requires_grad)
        kw = {"mode": mode}
        yield SampleInput((x,), dict(kw, size=(8,) * n))
        yield SampleInput((x,), dict(kw, scale_factor=2.0))
        yield SampleInput((x,), dict(kw, size=(3,) * n))
        if mode != "nearest":
            yield SampleInput((x,), dict(kw, size=(8,) * n, align_corners=True))

    return gen


def _prelu_samples(device, dtype, requires_grad):
    yield SampleInput((_t((2, 3, 4), device, dtype, requires_grad), _t((3,), device, dtype, requires_grad, 0.1, 0.5)))
    yield SampleInput((_t((2, 3), device, dtype, requires_grad), _t((1,), device, dtype, requires_grad, 0.1, 0.5)))


def _index_copy_samples(device, dtype, requires_grad):
    x = _t((5, 3), device, dtype, requires_grad)
    src = _t((2, 3), device, dtype, requires_grad)
    yield SampleInput((x, 0, torch.tensor([4, 1], device=device), src))
    x2 = _t((3, 5), device, dtype, requires_grad)
    yield SampleInput((x2, 1, torch.tensor([0, 3], device=device), _t((3, 2), device, dtype, requires_grad)))


def _multi_dot_samples(device, dtype, requires_grad):
    yield SampleInput(([_t((3, 4), device, dtype, requires_grad), _t((4, 5), device, dtype, requires_grad),
                        _t((5, 2), device, dtype, requires_grad)],))


OPS += [
    # activations
    elementwise_unary("celu", F.celu),
    OpInfo("celu_alpha", lambda x: F.celu(x, alpha=0.5), unary_samples()),
    elementwise_unary("selu", F.selu),
    elementwise_unary("hardshrink", F.hardshrink),
    elementwise_unary("softshrink", F.softshrink),
    elementwise_unary("hardsigmoid", F.hardsigmoid, low=-4.0, high=4.0),
    elementwise_unary("softsign", F.softsign),
    elementwise_unary("tanhshrink", F.tanhshrink),
    OpInfo("threshold", lambda x: F.threshold(x, 0.3, -1.0), unary_samples()),
    OpInfo("glu", F.glu, unary_samples(shapes=[(3, 4), (2, 6)])),
    OpInfo("glu_dim0", lambda x: F.glu(x, 0), unary_samples(shapes=[(4, 3)])),
    OpInfo("prelu", F.prelu, _prelu_samples),
    OpInfo("rrelu_eval", lambda x: F.rrelu(x, training=False), unary_samples()),
    OpInfo("softmin", lambda x: F.softmin(x, dim=-1), unary_samples(shapes=[(3, 4)])),
    OpInfo("ldexp", torch.ldexp, lambda d, t, r: iter([SampleInput((_t((3, 4), d, t, r), torch.randint(-2, 3, (3, 4), device=d)))]),
           dtypes=FLOAT32),
    # shape utilities
    OpInfo("atleast_1d", torch.atleast_1d, unary_samples(shapes=[(), (3,), (2, 3)])),
    OpInfo("atleast_2d", torch.atleast_2d, unary_samples(shapes=[(), (3,), (2, 3)])),
    OpInfo("atleast_3d", torch.atleast_3d, unary_samples(shapes=[(), (3,), (2, 3), (2, 3, 4)])),
    OpInfo("diagonal", torch.diagonal, _shape_samples([((4, 4), (), {}), ((3, 5), (1,), {}), ((5, 3), (-2,), {}),
                                                        ((2, 3, 4), (0, 1, 2), {})])),
    OpInfo("unfold", lambda x, *a: x.unfold(*a), _shape_samples([((7,), (0, 3, 2), {}), ((2, 8, 3), (1, 4, 1), {})])),
    OpInfo("index_copy", torch.index_copy, _index_copy_samples),
    OpInfo("multi_dot", torch.linalg.multi_dot, _multi_dot_samples, atol=1e-2, rtol=1e-2),
    # convolution
    OpInfo("conv1d", F.conv1d, _conv_samples(1), atol=2e-2, rtol=2e-2),
    OpInfo("conv2d", F.conv2d, _conv_samples(2), atol=2e-2, rtol=2e-2),
    OpInfo("conv3d", F.conv3d, _conv_samples(3), atol=2e-2, rtol=2e-2, dtypes=FLOAT32),
    # pooling
    OpInfo("max_pool1d", F.max_pool1d, _pool_samples(1, "max")),
    OpInfo("max_pool2d", F.max_pool2d, _pool_samples(2, "max")),
    OpInfo("max_pool3d", F.max_pool3d, _pool_samples(3, "max"), dtypes=FLOAT32),
    OpInfo("avg_pool1d", F.avg_pool1d, _pool_samples(1, "avg"), atol=1e-2, rtol=1e-2),
    OpInfo("avg_pool2d", F.avg_pool2d, _pool_samples(2, "avg"), atol=1e-2, rtol=1e-2),
    OpInfo("avg_pool3d", F.avg_pool3d, _pool_samples(3, "avg"), atol=1e-2, rtol=1e-2, dtypes=FLOAT32),
    OpInfo("adaptive_avg_pool2d", F.adaptive_avg_pool2d,
           lambda d, t, r: iter([SampleInput((_t((2, 3, 8, 6), d, t, r), (4, 3))), SampleInput((_t((2, 3, 8, 6), d, t, r), 1))]),
           atol=1e-2, rtol=1e-2),
    # normalization
    OpInfo("batch_norm_train", F.batch_norm, _bn_samples(True), atol=2e-2, rtol=2e-2),
    OpInfo("batch_norm_eval", F.batch_norm, _bn_samples(False), atol=2e-2, rtol=2e-2),
    OpInfo("instance_norm", F.instance_norm,
           lambda d, t, r: iter([SampleInput((_t((2, 3, 6), d, t, r),)),
                                 SampleInput((_t((2, 3, 4, 4), d, t, r),), {"weight": _t((3,), d, t, r, 0.5, 1.5),
                                                                           "bias": _t((3,), d, t, r)})]),
           atol=2e-2, rtol=2e-2),
    # (ATen's CPU kernels do not run LRN / ldexp-with-int in reduced precision: fp32 reference only)
    OpInfo("local_response_norm", lambda x: F.local_response_norm(x, 3), unary_samples(shapes=[(2, 5, 4), (2, 4, 3, 3)]),
           dtypes=FLOAT32),
    # interpolation
    OpInfo("interpolate_nearest", F.interpolate, _interp_samples("nearest", 2)),
    OpInfo("interpolate_bilinear", F.interpolate, _interp_samples("bilinear", 2), atol=2e-2, rtol=2e-2),
    OpInfo("interpolate_linear", F.interpolate, _interp_samples("linear", 1), atol=2e-2, rtol=2e-2),
]

OPS_BY_NAME = {o.name: o for o in OPS}


# =========================================================================================
# More coverage of existing ltorch symbols
# =========================================================================================
def _bool_pair(device, dtype, requires_grad):
    yield SampleInput((torch.rand(3, 4, device=device) > 0.5, torch.rand(3, 4, device=device) > 0.3))


def _scatter_samples(device, dtype, requires_grad):
    x = _t((3, 5), device, dtype, requires_grad)
    idx = torch.tensor([[0, 1, 2], [4, 3, 2], [1, 3, 0]], device=device)  # no duplicates per row
    yield SampleInput((x, 1, idx, _t((3, 3), device, dtype, requires_grad)))


def _index_put_samples(device, dtype, requires_grad):
    x = _t((5, 3), device, dtype, requires_grad)
    yield SampleInput((x, (torch.tensor([0, 3], device=device),), _t((2, 3), device, dtype, requires_grad)))
    yield SampleInput((x, (torch.tensor([1, 1, 4], device=device),), _t((3, 3), device, dtype, requires_grad)),
                      {"accumulate": True})


OPS += [
    OpInfo("clone", torch.clone, unary_samples()),
    OpInfo("floor_divide", torch.floor_divide, binary_samples(low=1.0, high=5.0, scalar=False), differentiable=False),
    OpInfo("clamp_min", lambda x: torch.clamp_min(x, -0.5), unary_samples()),
    OpInfo("clamp_max", lambda x: torch.clamp_max(x, 0.5), unary_samples()),
    OpInfo("logical_and", torch.logical_and, _bool_pair, dtypes=(torch.bool,), differentiable=False),
    OpInfo("logical_or", torch.logical_or, _bool_pair, dtypes=(torch.bool,), differentiable=False),
    OpInfo("logical_xor", torch.logical_xor, _bool_pair, dtypes=(torch.bool,), differentiable=False),
    OpInfo("logical_not", lambda a, b: torch.logical_not(a), _bool_pair, dtypes=(torch.bool,), differentiable=False),
    OpInfo("bitwise_or", torch.bitwise_or, binary_samples(scalar=False), dtypes=INTS, differentiable=False),
    OpInfo("bitwise_left_shift", torch.bitwise_left_shift, binary_samples(low=0, high=4, scalar=False), dtypes=INTS,
           differentiable=False),
    OpInfo("repeat_interleave", lambda x: torch.repeat_interleave(x, 2, 1), unary_samples(shapes=[(3, 4)])),
    OpInfo("tensor_split", lambda x: torch.tensor_split(x, 3, 1), unary_samples(shapes=[(2, 7)])),
    OpInfo("unflatten", lambda x: x.unflatten(1, (2, 3)), unary_samples(shapes=[(4, 6)])),
    OpInfo("select", lambda x: x.select(1, 2), unary_samples(shapes=[(3, 4, 2)])),
    OpInfo("expand_as", lambda x: x.expand_as(torch.empty(4, 3, 5)), unary_samples(shapes=[(3, 1)])),
    OpInfo("sort", lambda x: torch.sort(x, 1, descending=True), unary_samples(shapes=[(3, 6)])),
    OpInfo("argsort", lambda x: torch.argsort(x, -1), unary_samples(shapes=[(3, 6)]), differentiable=False),
    OpInfo("scatter", torch.scatter, _scatter_samples),
    OpInfo("index_put", torch.index_put, _index_put_samples),
    OpInfo("baddbmm", torch.baddbmm, lambda d, t, r: iter([SampleInput((_t((2, 3, 5), d, t, r), _t((2, 3, 4), d, t, r),
                                                                        _t((2, 4, 5), d, t, r)))]),
           atol=1e-2, rtol=1e-2),
    OpInfo("mm", torch.mm, lambda d, t, r: iter([SampleInput((_t((3, 4), d, t, r), _t((4, 5), d, t, r)))]),
           atol=1e-2, rtol=1e-2),
    OpInfo("t", lambda x: x.t(), unary_samples(shapes=[(3, 4)])),
    OpInfo("zeros_like_add", lambda x: torch.zeros_like(x) + x, unary_samples()),
    OpInfo("full_like_mul", lambda x: torch.full_like(x, 2.5) * x, unary_samples()),
    OpInfo("isinf", torch.isinf, unary_samples(), differentiable=False),
    OpInfo("signbit", torch.signbit, unary_samples(), differentiable=False),
    OpInfo("masked_fill_tensor", lambda x: x.masked_fill(x > 0.5, -1.0), unary_samples()),
    OpInfo("cumsum_dim0", lambda x: torch.cumsum(x, 0), unary_samples(shapes=[(4, 3)])),
    OpInfo("logsumexp_dim0", lambda x: torch.logsumexp(x, 0), unary_samples(shapes=[(4, 3)])),
    OpInfo("amax_keepdim", lambda x: torch.amax(x, (0, 2), keepdim=True), unary_samples(shapes=[(2, 3, 4)])),
]

OPS_BY_NAME = {o.name: o for o in OPS}


# =========================================================================================
# torch/more_ops.py: losses, special functions, products, scans and shape utilities
# =========================================================================================
def _pair(shape_a, shape_b, low=-2.0, high=2.0, lb=None, hb=None):
    def gen(device, dtype, requires_grad):
        yield SampleInput((_t(shape_a, device, dtype, requires_grad, low, high),
                           _t(shape_b, device, dtype, requires_grad, low if lb is None else lb,
                              high if hb is None else hb)))

    return gen


def _loss_samples(target="normal", extra=({},)):
    def gen(device, dtype, requires_grad):
        x = _t((3, 5), device, dtype, requires_grad)
        if target == "sign":
            y = torch.where(torch.rand(3, 5, device=device) > 0.5, 1.0, -1.0).to(dtype)
        elif target == "prob":
            y = _t((3, 5), device, dtype, False, 0.05, 0.95)
        elif target == "binary":
            y = (torch.rand(3, 5, device=device) > 0.5).to(dtype)
        else:
            y = _t((3, 5), device, dtype, requires_grad)
        for kw in extra:
            yield SampleInput((x, y), dict(kw))

    return gen


def _prob_input_loss(device, dtype, requires_grad):
    p = _t((3, 5), device, dtype, requires_grad, 0.05, 0.95)
    y = (torch.rand(3, 5, device=device) > 0.5).to(dtype)
    yield SampleInput((p, y))
    yield SampleInput((p, y), {"reduction": "sum"})


def _three(shapes, low=-2.0, high=2.0):
    def gen(device, dtype, requires_grad):
        yield SampleInput(tuple(_t(s, device, dtype, requires_grad, low, high) for s in shapes))

    return gen


def _cosemb_samples(device, dtype, requires_grad):
    a, b = _t((4, 6), device, dtype, requires_grad), _t((4, 6), device, dtype, requires_grad)
    yield SampleInput((a, b, torch.tensor([1.0, -1.0, 1.0, -1.0], device=device, dtype=dtype)), {"margin": 0.1})


def _mrank_samples(device, dtype, requires_grad):
    a, b = _t((6,), device, dtype, requires_grad), _t((6,), device, dtype, requires_grad)
    yield SampleInput((a, b, torch.tensor([1.0, -1.0, 1.0, -1.0, 1.0, 1.0], device=device, dtype=dtype)))


def _gnll_samples(device, dtype, requires_grad):
    x, y = _t((3, 5), device, dtype, requires_grad), _t((3, 5), device, dtype, requires_grad)
    yield SampleInput((x, y, _t((3, 5), device, dtype, requires_grad, 0.2, 2.0)))
    yield SampleInput((x, y, _t((3, 1), device, dtype, requires_grad, 0.2, 2.0)), {"full": True})


def _list_samples(shapes):
    def gen(device, dtype, requires_grad):
        yield SampleInput(([_t(s, device, dtype, requires_grad) for s in shapes],))

    return gen


OPS += [
    # losses / distances
    OpInfo("smooth_l1_loss", F.smooth_l1_loss, _loss_samples(extra=({}, {"beta": 0.5}, {"reduction": "none"}))),
    OpInfo("huber_loss", F.huber_loss, _loss_samples(extra=({}, {"delta": 0.3}, {"reduction": "sum"}))),
    OpInfo("binary_cross_entropy", lambda p, y, **kw: F.binary_cross_entropy(p, (y > 0.5).to(p.dtype), **kw),
           _prob_input_loss, atol=3e-2, rtol=3e-2),
    OpInfo("kl_div", lambda x, y: F.kl_div(x.log_softmax(-1), y, reduction="batchmean"), _loss_samples("prob")),
    OpInfo("kl_div_log_target", lambda x, y: F.kl_div(x, y, reduction="sum", log_target=True), _loss_samples()),
    OpInfo("poisson_nll_loss", F.poisson_nll_loss, _loss_samples("prob", ({}, {"full": True}))),
    OpInfo("soft_margin_loss", lambda x, y: F.soft_margin_loss(x, y.sign().detach()), _loss_samples("sign")),
    OpInfo("hinge_embedding_loss", lambda x, y: F.hinge_embedding_loss(x, y.sign()), _loss_samples("sign")),
    OpInfo("multilabel_soft_margin_loss", F.multilabel_soft_margin_loss, _loss_samples("binary")),
    OpInfo("margin_ranking_loss", lambda a, b, t: F.margin_ranking_loss(a, b, t.sign()), _mrank_samples),
    OpInfo("cosine_embedding_loss", lambda a, b, t, **kw: F.cosine_embedding_loss(a, b, t.sign(), **kw), _cosemb_samples, atol=3e-2, rtol=3e-2),
    OpInfo("gaussian_nll_loss", F.gaussian_nll_loss, _gnll_samples, atol=3e-2, rtol=3e-2),
    OpInfo("cosine_similarity", F.cosine_similarity, _pair((4, 6), (4, 6))),
    OpInfo("pairwise_distance", F.pairwise_distance, _pair((4, 6), (4, 6)), atol=3e-2, rtol=3e-2),
    OpInfo("triplet_margin_loss", F.triplet_margin_loss, _three([(4, 6)] * 3), atol=3e-2, rtol=3e-2),
    # elementwise special functions
    elementwise_binary("logaddexp", torch.logaddexp, samples=_pair((3, 4), (3, 4))),
    elementwise_binary("logaddexp2", torch.logaddexp2, samples=_pair((3, 4), (4,))),
    elementwise_binary("xlogy", torch.xlogy, samples=_pair((3, 4), (3, 4), lb=0.1, hb=3.0)),
    elementwise_binary("xlog1py", torch.special.xlog1py, samples=_pair((3, 4), (3, 4), lb=0.1, hb=3.0)),
    elementwise_binary("hypot", torch.hypot, samples=_pair((3, 4), (3, 4))),
    elementwise_binary("fmax", torch.fmax, samples=_pair((3, 4), (3, 4))),
    elementwise_binary("fmin", torch.fmin, samples=_pair((3, 4), (3, 4))),
    elementwise_unary("logit", lambda x: torch.logit(x, 1e-3), 0.05, 0.95),
    elementwise_unary("sinc", torch.sinc),
    elementwise_unary("deg2rad", torch.deg2rad),
    elementwise_unary("rad2deg", torch.rad2deg),
    elementwise_unary("frac", torch.frac),
    elementwise_unary("positive", torch.positive),
    elementwise_unary("erfcx", torch.special.erfcx, 0.0, 2.0, dtypes=FLOAT32),
    elementwise_unary("float_power", lambda x: torch.float_power(x, 2.5), 0.1, 2.0, dtypes=FLOAT32),
    elementwise_unary("isposinf", lambda x: torch.isposinf(1.0 / x.round()), differentiable=False),
    elementwise_unary("isneginf", lambda x: torch.isneginf(1.0 / x.round()), differentiable=False),
    elementwise_binary("isclose", lambda a, b: torch.isclose(a, a + b * 1e-9), samples=_pair((3, 4), (3, 4)),
                       differentiable=False),
    elementwise_binary("heaviside", torch.heaviside, samples=_pair((3, 4), (3, 4)), dtypes=FLOAT32,
                       differentiable=False),
    # reductions / scans
    OpInfo("nansum", torch.nansum, reduction_samples(dims=(None, 1))),
    OpInfo("nanmean", torch.nanmean, reduction_samples(dims=(None, 0)), dtypes=FLOAT32),
    OpInfo("count_nonzero", lambda x: torch.count_nonzero(x.round(), 1), unary_samples(shapes=[(3, 4)]),
           differentiable=False),
    OpInfo("cumprod", lambda x: torch.cumprod(x, 1), unary_samples(shapes=[(3, 5)]), dtypes=FLOAT32),
    OpInfo("logcumsumexp", lambda x: torch.logcumsumexp(x, -1), unary_samples(shapes=[(3, 5), (6,)])),
    OpInfo("diff", lambda x: torch.diff(x, n=2), unary_samples(shapes=[(3, 6)])),
    OpInfo("diff_prepend", lambda x: torch.diff(x, dim=0, prepend=x[:1] * 2), unary_samples(shapes=[(3, 4)])),
    OpInfo("trace", torch.trace, unary_samples(shapes=[(4, 4), (3, 5)]), dtypes=FLOAT32),
    # products
    OpInfo("dot", torch.dot, _pair((6,), (6,))),
    OpInfo("vdot", torch.vdot, _pair((6,), (6,))),
    OpInfo("inner", torch.inner, _pair((3, 4), (5, 4))),
    OpInfo("mv", torch.mv, _pair((3, 4), (4,))),
    OpInfo("addmv", lambda a, m, v: torch.addmv(a, m, v, beta=0.5, alpha=2.0), _three([(3,), (3, 4), (4,)])),
    OpInfo("addr", lambda a, u, v: torch.addr(a, u, v, alpha=0.5), _three([(3, 4), (3,), (4,)])),
    OpInfo("addbmm", torch.addbmm, _three([(3, 5), (2, 3, 4), (2, 4, 5)])),
    OpInfo("kron", torch.kron, _pair((2, 3), (3, 2))),
    OpInfo("tensordot", lambda a, b: torch.tensordot(a, b, dims=([1, 2], [0, 1])), _pair((2, 3, 4), (3, 4, 5))),
    OpInfo("bilinear", F.bilinear, _three([(3, 4), (3, 5), (2, 4, 5)]), atol=3e-2, rtol=3e-2),
    # shape utilities
    OpInfo("column_stack", torch.column_stack, _list_samples([(4,), (4, 2)])),
    OpInfo("row_stack", torch.row_stack, _list_samples([(4,), (2, 4)])),
    OpInfo("dstack", torch.dstack, _list_samples([(3, 4), (3, 4)])),
    OpInfo("hsplit", lambda x: torch.hsplit(x, 2), unary_samples(shapes=[(3, 4)])),
    OpInfo("vsplit", lambda x: torch.vsplit(x, [1, 3]), unary_samples(shapes=[(4, 3)])),
    OpInfo("dsplit", lambda x: torch.dsplit(x, 2), unary_samples(shapes=[(2, 3, 4)])),
    OpInfo("broadcast_tensors", torch.broadcast_tensors, _pair((1, 4), (3, 1))),
    OpInfo("pixel_shuffle", lambda x: F.pixel_shuffle(x, 2), unary_samples(shapes=[(1, 8, 2, 3)])),
    OpInfo("pixel_unshuffle", lambda x: F.pixel_unshuffle(x, 2), unary_samples(shapes=[(1, 2, 4, 6)])),
    OpInfo("rot90", lambda x: torch.rot90(x, 1, (0, 2)), unary_samples(shapes=[(2, 3, 4)])),
    OpInfo("rot90_neg", lambda x: torch.rot90(x, -1), unary_samples(shapes=[(3, 4)])),
    OpInfo("tile", lambda x: torch.tile(x, (2, 1, 2)), unary_samples(shapes=[(3, 4)])),
    OpInfo("block_diag", torch.block_diag, _pair((2, 3), (3, 2))),
    OpInfo("cartesian_prod", torch.cartesian_prod, _pair((3,), (2,))),
    OpInfo("meshgrid", lambda a, b: torch.meshgrid(a, b, indexing="ij"), _pair((3,), (2,))),
    OpInfo("meshgrid_xy", lambda a, b: torch.meshgrid(a, b, indexing="xy"), _pair((3,), (2,))),
    OpInfo("vander", lambda x: torch.vander(x, 4, increasing=True), unary_samples(shapes=[(5,)]),
           differentiable=False),
    OpInfo("eye_mul", lambda x: torch.eye(3, 4, dtype=x.dtype, device=x.device) * x, unary_samples(shapes=[(3, 4)])),
]

OPS_BY_NAME = {o.name: o for o in OPS}

OPS += [
    elementwise_unary("special_ndtri", torch.special.ndtri, 0.02, 0.98, dtypes=FLOAT32),
    elementwise_unary("special_ndtr", torch.special.ndtr, dtypes=FLOAT32),
    elementwise_unary("special_log_ndtr", torch.special.log_ndtr, -3.0, 3.0, dtypes=FLOAT32),
    elementwise_unary("special_entr", torch.special.entr, 0.05, 2.0, dtypes=FLOAT32),
    elementwise_unary("special_gammaln", torch.special.gammaln, 0.5, 4.0, dtypes=FLOAT32),
    elementwise_unary("special_multigammaln", lambda x: torch.special.multigammaln(x, 3), 1.5, 4.0, dtypes=FLOAT32),
]
OPS_BY_NAME = {o.name: o for o in OPS}
