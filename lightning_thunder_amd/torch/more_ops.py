"""Further ltorch decompositions: losses, distances, elementwise special functions, linear-algebra
products, reductions and shape utilities (parity: the corresponding ``@torchsymbol`` entries of
reference ``thunder/torch/__init__.py`` — e.g. ``smooth_l1_loss``, ``kl_div``, ``cosine_similarity``,
``logaddexp``, ``xlogy``, ``cumprod``, ``kron``, ``tensordot``, ``nansum``, ``count_nonzero``,
``pixel_shuffle``, ``hstack``-family, ``broadcast_tensors``, ``eye``).

Each op is written in terms of existing ltorch symbols, so it gets an analytic VJP through its
parts, its elementwise pieces fuse in hipfuse, and the trace shows the ATen-level name (the torch
executor still runs the whole op as one ATen call when nothing claims its parts).
"""
from __future__ import annotations

import builtins
import math

import torch

from ..core import prims
from ..core.baseutils import check
from ..core.proxies import TensorProxy, pyval
from . import torchsymbol, _tfn
from . import _this as _lt


def _f(name):
    """The ltorch symbol ``name`` (looked up late so ops defined in sibling modules resolve)."""
    return getattr(_lt, name)


def _export(sym):
    setattr(_lt, sym.name, sym)
    return sym


def _reduce(x, reduction: str):
    if reduction == "mean":
        return _f("mean")(x)
    if reduction == "sum":
        return _f("sum")(x)
    check(reduction == "none", f"unknown reduction {reduction!r}")
    return x


# =========================================================================================
# Losses
# =========================================================================================
@_export
@torchsymbol(*_tfn("nn.functional.smooth_l1_loss"), id="torch.nn.functional.smooth_l1_loss")
def smooth_l1_loss(input, target, size_average=None, reduce=None, reduction: str = "mean", beta: float = 1.0):
    d = _f("abs")(_f("sub")(input, target))
    b = pyval(beta)
    if b == 0:
        return _reduce(d, reduction)
    loss = _f("where")(_f("lt")(d, b), _f("true_divide")(_f("mul")(_f("mul")(d, d), 0.5), b), _f("sub")(d, 0.5 * b))
    return _reduce(loss, reduction)


@_export
@torchsymbol(*_tfn("nn.functional.huber_loss"), id="torch.nn.functional.huber_loss")
def huber_loss(input, target, reduction: str = "mean", delta: float = 1.0, weight=None):
    d = _f("abs")(_f("sub")(input, target))
    dl = pyval(delta)
    loss = _f("where")(_f("lt")(d, dl), _f("mul")(_f("mul")(d, d), 0.5), _f("mul")(_f("sub")(d, 0.5 * dl), dl))
    if weight is not None:
        loss = _f("mul")(loss, weight)
    return _reduce(loss, reduction)


@_export
@torchsymbol(*_tfn("nn.functional.binary_cross_entropy"), id="torch.nn.functional.binary_cross_entropy")
def binary_cross_entropy(input, target, weight=None, size_average=None, reduce=None, reduction: str = "mean"):
    # torch clamps the logs at -100
    lx = _f("clamp")(_f("log")(input), -100.0, None)
    l1x = _f("clamp")(_f("log")(_f("sub")(1.0, input)), -100.0, None)
    loss = _f("neg")(_f("add")(_f("mul")(target, lx), _f("mul")(_f("sub")(1.0, target), l1x)))
    if weight is not None:
        loss = _f("mul")(loss, weight)
    return _reduce(loss, reduction)


@_export
@torchsymbol(*_tfn("nn.functional.kl_div"), id="torch.nn.functional.kl_div")
def kl_div(input, target, size_average=None, reduce=None, reduction: str = "mean", log_target: bool = False):
    if log_target:
        loss = _f("mul")(_f("exp")(target), _f("sub")(target, input))
    else:
        loss = _f("sub")(xlogy(target, target), _f("mul")(target, input))
    if reduction == "batchmean":
        return _f("true_divide")(_f("sum")(loss), input.shape[0] if input.ndim else 1)
    return _reduce(loss, reduction)


@_export
@torchsymbol(*_tfn("nn.functional.poisson_nll_loss"), id="torch.nn.functional.poisson_nll_loss")
def poisson_nll_loss(input, target, log_input: bool = True, full: bool = False, size_average=None, eps: float = 1e-8,
                     reduce=None, reduction: str = "mean"):
    if log_input:
        loss = _f("sub")(_f("exp")(input), _f("mul")(target, input))
    else:
        loss = _f("sub")(input, _f("mul")(target, _f("log")(_f("add")(input, eps))))
    if full:
        st = _f("add")(_f("sub")(_f("mul")(target, _f("log")(target)), target),
                       _f("mul")(_f("log")(_f("mul")(target, 2 * math.pi)), 0.5))
        loss = _f("add")(loss, _f("where")(_f("gt")(target, 1), st, _f("zeros_like")(st)))
    return _reduce(loss, reduction)


@_export
@torchsymbol(*_tfn("nn.functional.soft_margin_loss"), id="torch.nn.functional.soft_margin_loss")
def soft_margin_loss(input, target, size_average=None, reduce=None, reduction: str = "mean"):
    return _reduce(_f("log1p")(_f("exp")(_f("neg")(_f("mul")(target, input)))), reduction)


@_export
@torchsymbol(*_tfn("nn.functional.margin_ranking_loss"), id="torch.nn.functional.margin_ranking_loss")
def margin_ranking_loss(input1, input2, target, margin: float = 0.0, size_average=None, reduce=None,
                        reduction: str = "mean"):
    v = _f("add")(_f("mul")(_f("neg")(target), _f("sub")(input1, input2)), margin)
    return _reduce(_f("clamp")(v, 0.0, None), reduction)


@_export
@torchsymbol(*_tfn("nn.functional.hinge_embedding_loss"), id="torch.nn.functional.hinge_embedding_loss")
def hinge_embedding_loss(input, target, margin: float = 1.0, size_average=None, reduce=None, reduction: str = "mean"):
    zero = _f("zeros_like")(input)
    pos = _f("where")(_f("ne")(target, -1), input, zero)
    neg_ = _f("where")(_f("ne")(target, 1), _f("clamp")(_f("sub")(margin, input), 0.0, None), zero)
    return _reduce(_f("add")(pos, neg_), reduction)


@_export
@torchsymbol(*_tfn("nn.functional.gaussian_nll_loss"), id="torch.nn.functional.gaussian_nll_loss")
def gaussian_nll_loss(input, target, var, full: bool = False, eps: float = 1e-6, reduction: str = "mean"):
    if var.ndim != input.ndim:  # a trailing singleton var dim was dropped
        var = _f("unsqueeze")(var, -1)
    v = _f("clamp")(var, eps, None)
    loss = _f("mul")(_f("add")(_f("log")(v), _f("true_divide")(_f("square")(_f("sub")(input, target)), v)), 0.5)
    if full:
        loss = _f("add")(loss, 0.5 * math.log(2 * math.pi))
    return _reduce(loss, reduction)


@_export
@torchsymbol(*_tfn("nn.functional.multilabel_soft_margin_loss"), id="torch.nn.functional.multilabel_soft_margin_loss")
def multilabel_soft_margin_loss(input, target, weight=None, size_average=None, reduce=None, reduction: str = "mean"):
    ls = _f("logsigmoid")
    loss = _f("neg")(_f("add")(_f("mul")(target, ls(input)), _f("mul")(_f("sub")(1.0, target), ls(_f("neg")(input)))))
    if weight is not None:
        loss = _f("mul")(loss, weight)
    loss = _f("mean")(loss, -1)
    return _reduce(loss, reduction)


@_export
@torchsymbol(*_tfn("nn.functional.cosine_similarity"), id="torch.nn.functional.cosine_similarity")
def cosine_similarity(x1, x2, dim: int = 1, eps: float = 1e-8):
    num = _f("sum")(_f("mul")(x1, x2), dim)
    n1 = _f("sqrt")(_f("sum")(_f("mul")(x1, x1), dim))
    n2 = _f("sqrt")(_f("sum")(_f("mul")(x2, x2), dim))
    return _f("true_divide")(num, _f("clamp")(_f("mul")(n1, n2), eps, None))


@_export
@torchsymbol(*_tfn("nn.functional.pairwise_distance"), id="torch.nn.functional.pairwise_distance")
def pairwise_distance(x1, x2, p: float = 2.0, eps: float = 1e-6, keepdim: bool = False):
    d = _f("abs")(_f("add")(_f("sub")(x1, x2), eps))
    p = pyval(p)
    if p == 2.0:
        return _f("sqrt")(_f("sum")(_f("mul")(d, d), -1, keepdim))
    if p == 1.0:
        return _f("sum")(d, -1, keepdim)
    return _f("pow")(_f("sum")(_f("pow")(d, p), -1, keepdim), 1.0 / p)


@_export
@torchsymbol(*_tfn("nn.functional.cosine_embedding_loss"), id="torch.nn.functional.cosine_embedding_loss")
def cosine_embedding_loss(input1, input2, target, margin: float = 0.0, size_average=None, reduce=None,
                          reduction: str = "mean"):
    cos = cosine_similarity(input1, input2, 1 if input1.ndim > 1 else 0, 1e-12)
    pos = _f("sub")(1.0, cos)
    neg_ = _f("clamp")(_f("sub")(cos, margin), 0.0, None)
    loss = _f("where")(_f("eq")(target, 1), pos, _f("where")(_f("eq")(target, -1), neg_, _f("zeros_like")(cos)))
    return _reduce(loss, reduction)


@_export
@torchsymbol(*_tfn("nn.functional.triplet_margin_loss"), id="torch.nn.functional.triplet_margin_loss")
def triplet_margin_loss(anchor, positive, negative, margin: float = 1.0, p: float = 2.0, eps: float = 1e-6,
                        swap: bool = False, size_average=None, reduce=None, reduction: str = "mean"):
    dp = pairwise_distance(anchor, positive, p, eps)
    dn = pairwise_distance(anchor, negative, p, eps)
    if swap:
        dn = _f("minimum")(dn, pairwise_distance(positive, negative, p, eps))
    return _reduce(_f("clamp")(_f("add")(_f("sub")(dp, dn), margin), 0.0, None), reduction)


# =========================================================================================
# Elementwise special functions
# =========================================================================================
@_export
@torchsymbol(*_tfn("logaddexp", "Tensor.logaddexp"), id="torch.logaddexp")
def logaddexp(a, b):
    m = _f("maximum")(a, b)
    return _f("add")(m, _f("log1p")(_f("exp")(_f("neg")(_f("abs")(_f("sub")(a, b))))))


@_export
@torchsymbol(*_tfn("logaddexp2", "Tensor.logaddexp2"), id="torch.logaddexp2")
def logaddexp2(a, b):
    m = _f("maximum")(a, b)
    return _f("add")(m, _f("true_divide")(_f("log1p")(_f("exp2")(_f("neg")(_f("abs")(_f("sub")(a, b))))), math.log(2)))


@_export
@torchsymbol(*_tfn("xlogy", "special.xlogy", "Tensor.xlogy"), id="torch.xlogy")
def xlogy(a, b):
    r = _f("mul")(a, _f("log")(b))
    r = _f("where")(_f("eq")(a, 0), _f("zeros_like")(r), r)
    return _f("where")(_f("isnan")(b), b if isinstance(b, TensorProxy) else r, r)


@_export
@torchsymbol(*_tfn("special.xlog1py"), id="torch.special.xlog1py")
def xlog1py(a, b):
    r = _f("mul")(a, _f("log1p")(b))
    r = _f("where")(_f("eq")(a, 0), _f("zeros_like")(r), r)
    return _f("where")(_f("isnan")(b), b if isinstance(b, TensorProxy) else r, r)


@_export
@torchsymbol(*_tfn("hypot", "Tensor.hypot"), id="torch.hypot")
def hypot(a, b):
    return _f("sqrt")(_f("add")(_f("mul")(a, a), _f("mul")(b, b)))


@_export
@torchsymbol(*_tfn("logit", "special.logit", "Tensor.logit"), id="torch.logit")
def logit(a, eps=None):
    if eps is not None:
        a = _f("clamp")(a, pyval(eps), 1.0 - pyval(eps))
    return _f("log")(_f("true_divide")(a, _f("sub")(1.0, a)))


@_export
@torchsymbol(*_tfn("sinc", "special.sinc", "Tensor.sinc"), id="torch.sinc")
def sinc(a):
    pa = _f("mul")(a, math.pi)
    r = _f("true_divide")(_f("sin")(pa), pa)
    return _f("where")(_f("eq")(a, 0), _f("ones_like")(r), r)


@_export
@torchsymbol(*_tfn("deg2rad", "Tensor.deg2rad"), id="torch.deg2rad")
def deg2rad(a):
    return _f("mul")(a, math.pi / 180.0)


@_export
@torchsymbol(*_tfn("rad2deg", "Tensor.rad2deg"), id="torch.rad2deg")
def rad2deg(a):
    return _f("mul")(a, 180.0 / math.pi)


@_export
@torchsymbol(*_tfn("frac", "Tensor.frac"), id="torch.frac")
def frac(a):
    return _f("sub")(a, _f("trunc")(a))


@_export
@torchsymbol(*_tfn("heaviside", "Tensor.heaviside"), id="torch.heaviside")
def heaviside(a, values):
    z = _f("zeros_like")(a)
    return _f("where")(_f("eq")(a, 0), _f("add")(z, values), _f("where")(_f("gt")(a, 0), _f("ones_like")(a), z))


@_export
@torchsymbol(*_tfn("fmax", "Tensor.fmax"), id="torch.fmax")
def fmax(a, b):
    # NaN-ignoring maximum: a NaN loses against a number
    m = _f("maximum")(a, b)
    return _f("where")(_f("isnan")(a), b, _f("where")(_f("isnan")(b), a, m))


@_export
@torchsymbol(*_tfn("fmin", "Tensor.fmin"), id="torch.fmin")
def fmin(a, b):
    m = _f("minimum")(a, b)
    return _f("where")(_f("isnan")(a), b, _f("where")(_f("isnan")(b), a, m))


@_export
@torchsymbol(*_tfn("float_power", "Tensor.float_power"), id="torch.float_power")
def float_power(a, b):
    a = _f("to")(a, torch.float64) if isinstance(a, TensorProxy) else float(pyval(a))
    b = _f("to")(b, torch.float64) if isinstance(b, TensorProxy) else float(pyval(b))
    return _f("pow")(a, b)


@_export
@torchsymbol(*_tfn("positive", "Tensor.positive"), id="torch.positive")
def positive(a):
    return a


@_export
@torchsymbol(*_tfn("isposinf"), id="torch.isposinf")
def isposinf(a):
    return _f("eq")(a, float("inf"))


@_export
@torchsymbol(*_tfn("isneginf"), id="torch.isneginf")
def isneginf(a):
    return _f("eq")(a, float("-inf"))


@_export
@torchsymbol(*_tfn("isreal", "Tensor.isreal"), id="torch.isreal")
def isreal(a):
    return _f("ne")(_f("zeros_like")(a), 1)  # real dtypes only: all True


@_export
@torchsymbol(*_tfn("isclose", "Tensor.isclose"), id="torch.isclose")
def isclose(a, b, rtol: float = 1e-05, atol: float = 1e-08, equal_nan: bool = False):
    close = _f("le")(_f("abs")(_f("sub")(a, b)), _f("add")(_f("mul")(_f("abs")(b), pyval(rtol)), pyval(atol)))
    close = _f("logical_or")(close, _f("eq")(a, b))
    if equal_nan:
        close = _f("logical_or")(close, _f("logical_and")(_f("isnan")(a), _f("isnan")(b)))
    return close


@_export
@torchsymbol(*_tfn("special.erfcx"), id="torch.special.erfcx")
def erfcx(a):
    return _f("mul")(_f("exp")(_f("mul")(a, a)), _f("erfc")(a))


@_export
@torchsymbol(*_tfn("special.logsumexp"), id="torch.special.logsumexp")
def special_logsumexp(a, dim, keepdim: bool = False):
    return _f("logsumexp")(a, dim, keepdim)


@_export
@torchsymbol(*_tfn("special.softmax"), id="torch.special.softmax")
def special_softmax(a, dim, dtype=None):
    return _f("softmax")(a, dim, dtype=dtype)


@_export
@torchsymbol(*_tfn("special.log_softmax"), id="torch.special.log_softmax")
def special_log_softmax(a, dim, dtype=None):
    return _f("log_softmax")(a, dim, dtype=dtype)


# =========================================================================================
# Reductions / scans
# =========================================================================================
@_export
@torchsymbol(*_tfn("nansum", "Tensor.nansum"), id="torch.nansum")
def nansum(a, dim=None, keepdim: bool = False, *, dtype=None):
    z = _f("where")(_f("isnan")(a), _f("zeros_like")(a), a)
    return _f("sum")(z, dim, keepdim, dtype=dtype)


@_export
@torchsymbol(*_tfn("nanmean", "Tensor.nanmean"), id="torch.nanmean")
def nanmean(a, dim=None, keepdim: bool = False, *, dtype=None):
    nn = _f("logical_not")(_f("isnan")(a))
    s = nansum(a, dim, keepdim, dtype=dtype)
    c = _f("sum")(_f("to")(nn, s.dtype), dim, keepdim)
    return _f("true_divide")(s, c)


@_export
@torchsymbol(*_tfn("count_nonzero", "Tensor.count_nonzero"), id="torch.count_nonzero")
def count_nonzero(a, dim=None):
    return _f("sum")(_f("to")(_f("ne")(a, 0), torch.int64), dim)


@_export
@torchsymbol(*_tfn("aminmax", "Tensor.aminmax"), id="torch.aminmax")
def aminmax(a, *, dim=None, keepdim: bool = False):
    return torch.return_types.aminmax((_f("amin")(a, dim, keepdim) if dim is not None else _f("amin")(a, ()),
                                       _f("amax")(a, dim, keepdim) if dim is not None else _f("amax")(a, ())))


@_export
@torchsymbol(*_tfn("cumprod", "Tensor.cumprod"), id="torch.cumprod")
def cumprod(a, dim, *, dtype=None):
    # exp(cumsum(log|a|)) with the sign tracked as a cumulative parity and exact zeros propagated
    d = pyval(dim) % a.ndim if a.ndim else 0
    x = _f("to")(a, dtype) if dtype is not None else a
    if not x.dtype.is_floating_point:
        x = _f("to")(x, torch.float64)
    zero = _f("eq")(x, 0)
    mag = _f("exp")(_f("cumsum")(_f("log")(_f("where")(zero, _f("ones_like")(x), _f("abs")(x))), d))
    negc = _f("cumsum")(_f("to")(_f("lt")(x, 0), torch.int64), d)
    sign = _f("sub")(1.0, _f("mul")(_f("remainder")(negc, 2), 2.0))
    anyzero = _f("gt")(_f("cumsum")(_f("to")(zero, torch.int64), d), 0)
    r = _f("where")(anyzero, _f("zeros_like")(mag), _f("mul")(mag, sign))
    return _f("to")(r, dtype or a.dtype)


@_export
@torchsymbol(*_tfn("logcumsumexp", "Tensor.logcumsumexp"), id="torch.logcumsumexp")
def logcumsumexp(a, dim):
    d = pyval(dim) % a.ndim if a.ndim else 0
    m = _f("amax")(a, (d,), True)
    m = _f("where")(_f("isinf")(m), _f("zeros_like")(m), m)
    return _f("add")(_f("log")(_f("cumsum")(_f("exp")(_f("sub")(a, m)), d)), m)


@_export
@torchsymbol(*_tfn("diff", "Tensor.diff"), id="torch.diff")
def diff(a, n: int = 1, dim: int = -1, prepend=None, append=None):
    d = pyval(dim) % a.ndim
    if prepend is not None:
        a = _f("cat")([prepend, a], d)
    if append is not None:
        a = _f("cat")([a, append], d)
    for _ in range(pyval(n)):
        L = a.shape[d]
        hi = _f("narrow")(a, d, 1, L - 1)
        lo = _f("narrow")(a, d, 0, L - 1)
        a = _f("logical_xor")(hi, lo) if a.dtype == torch.bool else _f("sub")(hi, lo)
    return a


@_export
@torchsymbol(*_tfn("trace", "Tensor.trace"), id="torch.trace")
def trace(a):
    return _f("sum")(_f("diagonal")(a))


# =========================================================================================
# Products
# =========================================================================================
@_export
@torchsymbol(*_tfn("dot", "Tensor.dot"), id="torch.dot")
def dot(a, b):
    return _f("sum")(_f("mul")(a, b))


@_export
@torchsymbol(*_tfn("vdot", "Tensor.vdot"), id="torch.vdot")
def vdot(a, b):
    return _f("sum")(_f("mul")(a, b))


@_export
@torchsymbol(*_tfn("inner", "Tensor.inner"), id="torch.inner")
def inner(a, b):
    if a.ndim == 0 or b.ndim == 0:
        return _f("mul")(a, b)
    return _f("matmul")(a, _f("movedim")(b, -1, 0)) if b.ndim <= 2 else tensordot(a, b, ([a.ndim - 1], [b.ndim - 1]))


@_export
@torchsymbol(*_tfn("mv", "Tensor.mv"), id="torch.mv")
def mv(a, v):
    return _f("matmul")(a, v)


@_export
@torchsymbol(*_tfn("addmv", "Tensor.addmv"), id="torch.addmv")
def addmv(input, mat, vec, *, beta=1, alpha=1):
    r = _f("mul")(_f("matmul")(mat, vec), alpha) if pyval(alpha) != 1 else _f("matmul")(mat, vec)
    return _f("add")(_f("mul")(input, beta) if pyval(beta) != 1 else input, r)


@_export
@torchsymbol(*_tfn("addr", "Tensor.addr"), id="torch.addr")
def addr(input, vec1, vec2, *, beta=1, alpha=1):
    r = _f("mul")(_f("unsqueeze")(vec1, 1), _f("unsqueeze")(vec2, 0))
    if pyval(alpha) != 1:
        r = _f("mul")(r, alpha)
    return _f("add")(_f("mul")(input, beta) if pyval(beta) != 1 else input, r)


@_export
@torchsymbol(*_tfn("addbmm", "Tensor.addbmm"), id="torch.addbmm")
def addbmm(input, batch1, batch2, *, beta=1, alpha=1):
    r = _f("sum")(_f("matmul")(batch1, batch2), 0)
    if pyval(alpha) != 1:
        r = _f("mul")(r, alpha)
    return _f("add")(_f("mul")(input, beta) if pyval(beta) != 1 else input, r)


@_export
@torchsymbol(*_tfn("kron", "Tensor.kron"), id="torch.kron")
def kron(a, b):
    n = builtins.max(a.ndim, b.ndim)
    a = _f("reshape")(a, (1,) * (n - a.ndim) + tuple(a.shape))
    b = _f("reshape")(b, (1,) * (n - b.ndim) + tuple(b.shape))
    ai = []
    bi = []
    for i in range(n):
        ai += [a.shape[i], 1]
        bi += [1, b.shape[i]]
    r = _f("mul")(_f("reshape")(a, tuple(ai)), _f("reshape")(b, tuple(bi)))
    return _f("reshape")(r, tuple(a.shape[i] * b.shape[i] for i in range(n)))


@_export
@torchsymbol(*_tfn("tensordot"), id="torch.tensordot")
def tensordot(a, b, dims=2, out=None):
    dims = pyval(dims) if not isinstance(dims, (tuple, list)) else dims
    if isinstance(dims, int):
        da = list(range(a.ndim - dims, a.ndim))
        db = list(range(dims))
    else:
        da, db = list(dims[0]), list(dims[1])
        da = [d if isinstance(d, int) else pyval(d) for d in (da if isinstance(da, list) else [da])]
        db = [d if isinstance(d, int) else pyval(d) for d in (db if isinstance(db, list) else [db])]
    da = [d % a.ndim for d in da]
    db = [d % b.ndim for d in db]
    fa = [i for i in range(a.ndim) if i not in da]
    fb = [i for i in range(b.ndim) if i not in db]
    K = 1
    for d in da:
        K *= a.shape[d]
    at = _f("reshape")(_f("permute")(a, fa + da), (-1, K))
    bt = _f("reshape")(_f("permute")(b, db + fb), (K, -1))
    return _f("reshape")(_f("matmul")(at, bt), tuple(a.shape[i] for i in fa) + tuple(b.shape[i] for i in fb))


@_export
@torchsymbol(*_tfn("nn.functional.bilinear"), id="torch.nn.functional.bilinear")
def bilinear(input1, input2, weight, bias=None):
    # y[..., o] = sum_ij x1[..., i] W[o, i, j] x2[..., j] + b[o]
    lead = tuple(input1.shape[:-1])
    O, I, J = weight.shape
    x1 = _f("reshape")(input1, (-1, 1, 1, I))
    x2 = _f("reshape")(input2, (-1, 1, J))
    t = _f("reshape")(_f("matmul")(x1, weight), (-1, O, J))  # [N, O, 1, J] -> [N, O, J]
    y = _f("reshape")(_f("sum")(_f("mul")(t, x2), -1), lead + (O,))
    return _f("add")(y, bias) if bias is not None else y


# =========================================================================================
# Shape utilities
# =========================================================================================
@_export
@torchsymbol(*_tfn("column_stack"), id="torch.column_stack")
def column_stack(tensors):
    ts = [(_f("reshape")(t, (-1, 1)) if t.ndim <= 1 else t) for t in tensors]
    return _f("cat")(ts, 1)


@_export
@torchsymbol(*_tfn("row_stack"), id="torch.row_stack")
def row_stack(tensors):
    return _f("vstack")(tensors)


@_export
@torchsymbol(*_tfn("dstack"), id="torch.dstack")
def dstack(tensors):
    ts = []
    for t in tensors:
        if t.ndim == 0:
            t = _f("reshape")(t, (1, 1, 1))
        elif t.ndim == 1:
            t = _f("reshape")(t, (1, t.shape[0], 1))
        elif t.ndim == 2:
            t = _f("unsqueeze")(t, -1)
        ts.append(t)
    return _f("cat")(ts, 2)


def _split_n(a, sections, dim):
    return _f("tensor_split")(a, sections, dim)


@_export
@torchsymbol(*_tfn("hsplit", "Tensor.hsplit"), id="torch.hsplit")
def hsplit(a, sections):
    return _split_n(a, sections, 1 if a.ndim > 1 else 0)


@_export
@torchsymbol(*_tfn("vsplit", "Tensor.vsplit"), id="torch.vsplit")
def vsplit(a, sections):
    return _split_n(a, sections, 0)


@_export
@torchsymbol(*_tfn("dsplit", "Tensor.dsplit"), id="torch.dsplit")
def dsplit(a, sections):
    return _split_n(a, sections, 2)


@_export
@torchsymbol(*_tfn("broadcast_tensors"), id="torch.broadcast_tensors")
def broadcast_tensors(*tensors):
    from ..clang import compute_broadcast_shape

    shape = compute_broadcast_shape(*(tuple(t.shape) for t in tensors))
    return tuple(_f("expand")(t, shape) for t in tensors)


@_export
@torchsymbol(*_tfn("nn.functional.pixel_shuffle"), id="torch.nn.functional.pixel_shuffle")
def pixel_shuffle(a, upscale_factor: int):
    r = pyval(upscale_factor)
    *lead, C, H, W = a.shape
    x = _f("reshape")(a, tuple(lead) + (C // (r * r), r, r, H, W))
    n = len(lead)
    x = _f("permute")(x, list(range(n)) + [n, n + 3, n + 1, n + 4, n + 2])
    return _f("reshape")(x, tuple(lead) + (C // (r * r), H * r, W * r))


@_export
@torchsymbol(*_tfn("nn.functional.pixel_unshuffle"), id="torch.nn.functional.pixel_unshuffle")
def pixel_unshuffle(a, downscale_factor: int):
    r = pyval(downscale_factor)
    *lead, C, H, W = a.shape
    x = _f("reshape")(a, tuple(lead) + (C, H // r, r, W // r, r))
    n = len(lead)
    x = _f("permute")(x, list(range(n)) + [n, n + 2, n + 4, n + 1, n + 3])
    return _f("reshape")(x, tuple(lead) + (C * r * r, H // r, W // r))


@_export
@torchsymbol(*_tfn("rot90", "Tensor.rot90"), id="torch.rot90")
def rot90(a, k: int = 1, dims=(0, 1)):
    k = pyval(k) % 4
    d0, d1 = (pyval(d) % a.ndim for d in dims)
    if k == 0:
        return a
    if k == 1:
        return _f("transpose")(_f("flip")(a, (d1,)), d0, d1)
    if k == 2:
        return _f("flip")(a, (d0, d1))
    return _f("flip")(_f("transpose")(a, d0, d1), (d1,))


@_export
@torchsymbol(*_tfn("tile", "Tensor.tile"), id="torch.tile")
def tile(a, dims):
    dims = tuple(pyval(d) for d in dims)
    if len(dims) < a.ndim:
        dims = (1,) * (a.ndim - len(dims)) + dims
    return _f("repeat")(a, dims)


@_export
@torchsymbol(*_tfn("block_diag"), id="torch.block_diag")
def block_diag(*tensors):
    ts = [(_f("reshape")(t, (1, -1)) if t.ndim < 2 else t) for t in tensors]
    R = builtins.sum(t.shape[0] for t in ts)
    C = builtins.sum(t.shape[1] for t in ts)
    rows, c0 = [], 0
    for t in ts:
        c1 = c0 + t.shape[1]
        rows.append(_f("pad")(t, (c0, C - c1)))
        c0 = c1
    return _f("cat")(rows, 0)


@_export
@torchsymbol(*_tfn("cartesian_prod"), id="torch.cartesian_prod")
def cartesian_prod(*tensors):
    if len(tensors) == 1:
        return tensors[0]
    grids = meshgrid(*tensors, indexing="ij")
    return _f("stack")([_f("reshape")(g, (-1,)) for g in grids], 1)


@_export
@torchsymbol(*_tfn("meshgrid"), id="torch.meshgrid")
def meshgrid(*tensors, indexing: str = "ij"):
    if len(tensors) == 1 and isinstance(tensors[0], (tuple, list)):
        tensors = tuple(tensors[0])
    ts = list(tensors)
    swap = indexing == "xy" and len(ts) >= 2
    if swap:
        ts[0], ts[1] = ts[1], ts[0]
    shape = tuple(t.shape[0] if t.ndim else 1 for t in ts)
    out = []
    for i, t in enumerate(ts):
        view = [1] * len(ts)
        view[i] = shape[i]
        out.append(_f("expand")(_f("reshape")(t, tuple(view)), shape))
    if swap:  # the ij grids of (b, a, ...) are the xy grids of (a, b, ...)
        out[0], out[1] = out[1], out[0]
    return tuple(out)


@_export
@torchsymbol(*_tfn("vander"), id="torch.vander")
def vander(x, N=None, increasing: bool = False):
    n = x.shape[0] if N is None else pyval(N)
    p = _f("arange")(n, device=x.device, dtype=x.dtype)
    if not increasing:
        p = _f("flip")(p, (0,))
    return _f("pow")(_f("unsqueeze")(x, 1), _f("unsqueeze")(p, 0))


@_export
@torchsymbol(*_tfn("eye"), id="torch.eye")
def eye(n, m=None, *, dtype=None, layout=None, device=None, pin_memory=False, requires_grad=False):
    n = pyval(n)
    m = n if m is None else pyval(m)
    r = _f("arange")(n, device=device)
    c = _f("arange")(m, device=device)
    e = _f("eq")(_f("unsqueeze")(r, 1), _f("unsqueeze")(c, 0))
    return _f("to")(e, dtype or torch.get_default_dtype())


# =========================================================================================
# In-place samplers (functionalized: a fresh sample copied into the tensor)
# =========================================================================================
def _u01(a, lo=0.0, hi=1.0):
    dt = a.dtype if a.dtype.is_floating_point else torch.float32
    return prims.uniform(a.shape, lo, hi, device=a.device, dtype=dt)


def _fill(a, v):
    return prims.copy_(_f("to")(v, a.dtype), a)


@_export
@torchsymbol(torch.Tensor.normal_, is_method=True, id="torch.Tensor.normal_")
def normal_(a, mean: float = 0.0, std: float = 1.0, *, generator=None):
    z = prims.randn(a.shape, device=a.device, dtype=a.dtype)
    return _fill(a, _f("add")(_f("mul")(z, std), mean))


@_export
@torchsymbol(torch.Tensor.log_normal_, is_method=True, id="torch.Tensor.log_normal_")
def log_normal_(a, mean: float = 1.0, std: float = 2.0, *, generator=None):
    z = prims.randn(a.shape, device=a.device, dtype=a.dtype)
    return _fill(a, _f("exp")(_f("add")(_f("mul")(z, std), mean)))


@_export
@torchsymbol(torch.Tensor.exponential_, is_method=True, id="torch.Tensor.exponential_")
def exponential_(a, lambd: float = 1.0, *, generator=None):
    # inverse CDF on (0, 1]: -log(1 - u) / lambda
    return _fill(a, _f("true_divide")(_f("neg")(_f("log1p")(_f("neg")(_u01(a)))), lambd))


@_export
@torchsymbol(torch.Tensor.cauchy_, is_method=True, id="torch.Tensor.cauchy_")
def cauchy_(a, median: float = 0.0, sigma: float = 1.0, *, generator=None):
    return _fill(a, _f("add")(_f("mul")(_f("tan")(_f("mul")(_f("sub")(_u01(a), 0.5), math.pi)), sigma), median))


@_export
@torchsymbol(torch.Tensor.geometric_, is_method=True, id="torch.Tensor.geometric_")
def geometric_(a, p: float, *, generator=None):
    # number of Bernoulli(p) trials to the first success: ceil(log(1-u) / log(1-p)), at least 1
    k = _f("ceil")(_f("true_divide")(_f("log1p")(_f("neg")(_u01(a))), math.log1p(-pyval(p))))
    return _fill(a, _f("clamp")(k, 1.0, None))


@_export
@torchsymbol(torch.Tensor.random_, is_method=True, id="torch.Tensor.random_")
def random_(a, from_=0, to=None, *, generator=None):
    if to is None and from_ != 0:
        from_, to = 0, from_
    if to is None:
        to = 2 ** (torch.finfo(a.dtype).nmant + 1) if a.dtype.is_floating_point else (
            2 if a.dtype == torch.bool else torch.iinfo(a.dtype).max)
    u = prims.uniform(a.shape, 0.0, 1.0, device=a.device, dtype=torch.float64)
    v = _f("floor")(_f("add")(_f("mul")(u, float(pyval(to) - pyval(from_))), float(pyval(from_))))
    return _fill(a, v)


# =========================================================================================
# torch.special: normal-distribution functions and friends
# =========================================================================================
@_export
@torchsymbol(*_tfn("special.ndtri"), id="torch.special.ndtri")
def ndtri(a):
    from .. import clang

    return clang.ndtri(a)


@_export
@torchsymbol(*_tfn("special.ndtr"), id="torch.special.ndtr")
def ndtr(a):
    a = _f("to")(a, torch.get_default_dtype()) if not a.dtype.is_floating_point else a
    return _f("mul")(_f("erfc")(_f("mul")(a, -1.0 / math.sqrt(2.0))), 0.5)


@_export
@torchsymbol(*_tfn("special.log_ndtr"), id="torch.special.log_ndtr")
def log_ndtr(a):
    # log(0.5 erfc(-x/sqrt2)); for x < -5 the erfc underflows in fp32: use log(erfcx(t)) - t^2 there
    a = _f("to")(a, torch.get_default_dtype()) if not a.dtype.is_floating_point else a
    t = _f("mul")(a, -1.0 / math.sqrt(2.0))
    direct = _f("log")(_f("mul")(_f("erfc")(t), 0.5))
    tail = _f("sub")(_f("log")(_f("mul")(_erfcx_impl(t), 0.5)), _f("mul")(t, t))
    return _f("where")(_f("lt")(a, -5.0), tail, direct)


def _erfcx_impl(a):
    return _f("mul")(_f("exp")(_f("mul")(a, a)), _f("erfc")(a))


@_export
@torchsymbol(*_tfn("special.entr"), id="torch.special.entr")
def entr(a):
    r = _f("neg")(_f("mul")(a, _f("log")(a)))
    r = _f("where")(_f("eq")(a, 0), _f("zeros_like")(r), r)
    return _f("where")(_f("lt")(a, 0), _f("full_like")(r, float("-inf")), r)


@_export
@torchsymbol(*_tfn("special.gammaln"), id="torch.special.gammaln")
def gammaln(a):
    return _f("lgamma")(a)


@_export
@torchsymbol(*_tfn("special.multigammaln", "mvlgamma", "Tensor.mvlgamma"), id="torch.special.multigammaln")
def multigammaln(a, p: int):
    p = pyval(p)
    acc = _f("lgamma")(a)
    for j in range(1, p):
        acc = _f("add")(acc, _f("lgamma")(_f("sub")(a, j / 2.0)))
    return _f("add")(acc, p * (p - 1) / 4.0 * math.log(math.pi))


@_export
@torchsymbol(*_tfn("special.expm1"), id="torch.special.expm1")
def special_expm1(a):
    return _f("expm1")(a)


@_export
@torchsymbol(*_tfn("special.log1p"), id="torch.special.log1p")
def special_log1p(a):
    return _f("log1p")(a)
