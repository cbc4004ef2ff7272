"""VJP rule registry and DAG utilities (parity: reference ``thunder/core/transforms.py``:
``register_grad`` :620, ``augmented_forward_impls``/``backward_impls`` :1634-1728,
DAG utilities :103-429, ``add_transform`` :430-467).

A VJP rule is ``rule(*args, **kwargs) -> (output, backward)``: it runs in the
forward trace (recording whatever forward ops it needs) and returns a closure
``backward(*cotangents) -> grads`` that runs later in the backward trace.  Proxies
captured by the closure become saved-for-backward tensors automatically.
``grads`` mirrors the structure of ``args`` (``None`` for no gradient).
"""
from __future__ import annotations

import math
from enum import Enum, auto
from typing import Any, Callable

import torch

from . import dtypes, prims
from .prims import PrimIDs
from .proxies import TensorProxy, Proxy, NumberProxy, pyval
from .pytree import tree_flatten, tree_unflatten, tree_map

_vjp_rules: dict[Any, Callable] = {}


def register_vjp(*ids):
    def deco(fn):
        for i in ids:
            key = i.id if hasattr(i, "id") else i
            _vjp_rules[key] = fn
        return fn

    return deco


def get_vjp_rule(sym_id):
    return _vjp_rules.get(sym_id)


# -----------------------------------------------------------------------------------------
# Helpers
# -----------------------------------------------------------------------------------------
def _ltorch():
    from .. import torch as ltorch

    return ltorch


def _clang():
    from .. import clang

    return clang


def sum_to_shape(g: TensorProxy, shape) -> TensorProxy:
    """Reduces a broadcast gradient back to ``shape``."""
    shape = tuple(shape)
    if tuple(g.shape) == shape:
        return g
    lead = g.ndim - len(shape)
    dims = list(range(lead))
    for i, s in enumerate(shape):
        if s == 1 and g.shape[lead + i] != 1:
            dims.append(lead + i)
    out = g
    if dims:
        out = _ltorch().sum(g, dims)
    return _clang().reshape(out, shape)


def grad_like(g, a):
    """Cast/reduce gradient ``g`` to match input ``a`` (or None for non-tensors)."""
    if not isinstance(a, TensorProxy) or g is None:
        return None
    if not dtypes.is_inexact_dtype(a.dtype):
        return None
    if tuple(g.shape) != tuple(a.shape):
        g = sum_to_shape(g, a.shape)
    if g.dtype != a.dtype:
        g = _clang().maybe_convert_to_dtype(g, a.dtype)
    return g


def _requires(x):
    return isinstance(x, TensorProxy) and x.requires_grad


def zeros_like_proxy(p: TensorProxy):
    return prims.full(tuple(p.shape), 0, device=p.device, dtype=p.dtype)


# =========================================================================================
# Prim rules
# =========================================================================================
def _unary_rule(fwd_prim, dfn):
    """dfn(a, out, g) -> grad for a (in a's compute dtype)."""

    def rule(a):
        out = fwd_prim(a)

        def bwd(g):
            return (dfn(a, out, g),)

        return out, bwd

    return rule


P = prims

register_vjp(PrimIDs.NEG)(_unary_rule(P.neg, lambda a, o, g: P.neg(g)))
register_vjp(PrimIDs.EXP)(_unary_rule(P.exp, lambda a, o, g: P.mul(g, o)))
register_vjp(PrimIDs.EXP2)(_unary_rule(P.exp2, lambda a, o, g: P.mul(P.mul(g, o), math.log(2.0))))
register_vjp(PrimIDs.EXPM1)(_unary_rule(P.expm1, lambda a, o, g: P.mul(g, P.add(o, 1.0))))
register_vjp(PrimIDs.LOG)(_unary_rule(P.log, lambda a, o, g: P.div(g, a)))
register_vjp(PrimIDs.LOG1P)(_unary_rule(P.log1p, lambda a, o, g: P.div(g, P.add(a, 1.0))))
register_vjp(PrimIDs.LOG2)(_unary_rule(P.log2, lambda a, o, g: P.div(g, P.mul(a, math.log(2.0)))))
register_vjp(PrimIDs.LOG10)(_unary_rule(P.log10, lambda a, o, g: P.div(g, P.mul(a, math.log(10.0)))))
register_vjp(PrimIDs.SQRT)(_unary_rule(P.sqrt, lambda a, o, g: P.div(g, P.mul(o, 2.0))))
register_vjp(PrimIDs.RSQRT)(_unary_rule(P.rsqrt, lambda a, o, g: P.mul(P.mul(g, -0.5), P.div(o, a))))
register_vjp(PrimIDs.RECIPROCAL)(_unary_rule(P.reciprocal, lambda a, o, g: P.neg(P.mul(g, P.mul(o, o)))))
register_vjp(PrimIDs.SIN)(_unary_rule(P.sin, lambda a, o, g: P.mul(g, P.cos(a))))
register_vjp(PrimIDs.COS)(_unary_rule(P.cos, lambda a, o, g: P.neg(P.mul(g, P.sin(a)))))
register_vjp(PrimIDs.TAN)(_unary_rule(P.tan, lambda a, o, g: P.mul(g, P.add(P.mul(o, o), 1.0))))
register_vjp(PrimIDs.TANH)(_unary_rule(P.tanh, lambda a, o, g: P.mul(g, P.sub(1.0, P.mul(o, o)))))
register_vjp(PrimIDs.SINH)(_unary_rule(P.sinh, lambda a, o, g: P.mul(g, P.cosh(a))))
register_vjp(PrimIDs.COSH)(_unary_rule(P.cosh, lambda a, o, g: P.mul(g, P.sinh(a))))
register_vjp(PrimIDs.ASIN)(_unary_rule(P.asin, lambda a, o, g: P.mul(g, P.rsqrt(P.sub(1.0, P.mul(a, a))))))
register_vjp(PrimIDs.ACOS)(_unary_rule(P.acos, lambda a, o, g: P.neg(P.mul(g, P.rsqrt(P.sub(1.0, P.mul(a, a)))))))
register_vjp(PrimIDs.ATAN)(_unary_rule(P.atan, lambda a, o, g: P.div(g, P.add(P.mul(a, a), 1.0))))
register_vjp(PrimIDs.ASINH)(_unary_rule(P.asinh, lambda a, o, g: P.mul(g, P.rsqrt(P.add(P.mul(a, a), 1.0)))))
register_vjp(PrimIDs.ACOSH)(_unary_rule(P.acosh, lambda a, o, g: P.mul(g, P.rsqrt(P.sub(P.mul(a, a), 1.0)))))
register_vjp(PrimIDs.ATANH)(_unary_rule(P.atanh, lambda a, o, g: P.div(g, P.sub(1.0, P.mul(a, a)))))
register_vjp(PrimIDs.ERF)(
    _unary_rule(P.erf, lambda a, o, g: P.mul(g, P.mul(P.exp(P.neg(P.mul(a, a))), 2.0 / math.sqrt(math.pi))))
)
register_vjp(PrimIDs.ERFC)(
    _unary_rule(P.erfc, lambda a, o, g: P.mul(g, P.mul(P.exp(P.neg(P.mul(a, a))), -2.0 / math.sqrt(math.pi))))
)
register_vjp(PrimIDs.ABS)(_unary_rule(P.abs, lambda a, o, g: P.mul(g, P.sign(a))))
register_vjp(PrimIDs.ERFINV)(
    _unary_rule(P.erfinv, lambda a, o, g: P.mul(g, P.mul(P.exp(P.mul(o, o)), math.sqrt(math.pi) / 2.0)))
)

register_vjp(PrimIDs.ERFCINV)(
    _unary_rule(P.erfcinv, lambda a, o, g: P.mul(g, P.mul(P.exp(P.mul(o, o)), -math.sqrt(math.pi) / 2.0)))
)
register_vjp(PrimIDs.NDTRI)(
    _unary_rule(P.ndtri, lambda a, o, g: P.mul(g, P.mul(P.exp(P.mul(P.mul(o, o), 0.5)), math.sqrt(2.0 * math.pi))))
)


def _trigamma(x):
    """psi_1(x) = sum_{k<6} 1/(x+k)^2 + asymptotic series at x+6 (accurate to ~1e-10 for x > 0)."""
    acc = None
    for k in range(6):
        xk = P.add(x, float(k)) if k else x
        t = P.reciprocal(P.mul(xk, xk))
        acc = t if acc is None else P.add(acc, t)
    z = P.add(x, 6.0)
    iz = P.reciprocal(z)
    iz2 = P.mul(iz, iz)
    # 1/z + 1/(2z^2) + 1/(6z^3) - 1/(30z^5) + 1/(42z^7) - 1/(30z^9)
    poly = P.add(1.0 / 6.0, P.mul(iz2, P.add(-1.0 / 30.0, P.mul(iz2, P.add(1.0 / 42.0, P.mul(iz2, -1.0 / 30.0))))))
    series = P.add(P.add(iz, P.mul(iz2, 0.5)), P.mul(P.mul(iz2, iz), poly))
    return P.add(acc, series)


register_vjp(PrimIDs.DIGAMMA)(_unary_rule(P.digamma, lambda a, o, g: P.mul(g, _trigamma(a))))
register_vjp(PrimIDs.LGAMMA)(_unary_rule(P.lgamma, lambda a, o, g: P.mul(g, P.digamma(a))))

for _zero_grad_prim in (P.sign, P.floor, P.ceil, P.round, P.trunc):
    register_vjp(_zero_grad_prim)(_unary_rule(_zero_grad_prim, lambda a, o, g: P.mul(g, 0.0)))


def _binary(fwd, dfa, dfb):
    def rule(a, b):
        out = fwd(a, b)

        def bwd(g):
            ga = dfa(a, b, out, g) if _requires(a) else None
            gb = dfb(a, b, out, g) if _requires(b) else None
            return ga, gb

        return out, bwd

    return rule


register_vjp(PrimIDs.ADD)(_binary(P.add, lambda a, b, o, g: g, lambda a, b, o, g: g))
register_vjp(PrimIDs.SUB)(_binary(P.sub, lambda a, b, o, g: g, lambda a, b, o, g: P.neg(g)))
register_vjp(PrimIDs.MUL)(_binary(P.mul, lambda a, b, o, g: P.mul(g, b), lambda a, b, o, g: P.mul(g, a)))
register_vjp(PrimIDs.DIV)(
    _binary(P.div, lambda a, b, o, g: P.div(g, b), lambda a, b, o, g: P.neg(P.div(P.mul(g, o), b)))
)


def _pow_da(a, b, o, g):
    if isinstance(b, TensorProxy):
        return P.mul(g, P.mul(b, P.pow(a, P.sub(b, 1.0))))
    bv = pyval(b)
    return P.mul(g, P.mul(P.pow(a, bv - 1.0), bv))


def _pow_db(a, b, o, g):
    la = P.log(a) if isinstance(a, TensorProxy) else math.log(pyval(a))
    return P.mul(g, P.mul(o, la))


register_vjp(PrimIDs.POW)(_binary(P.pow, _pow_da, _pow_db))


def _maxmin_rule(fwd, cmp):
    def rule(a, b):
        out = fwd(a, b)

        def bwd(g):
            # ties split evenly like torch
            if isinstance(a, TensorProxy) and isinstance(b, TensorProxy):
                mask_a = P.convert_element_type(cmp(a, b), g.dtype)
                eq = P.convert_element_type(P.eq(a, b), g.dtype)
                wa = P.add(mask_a, P.mul(eq, 0.5))
                wb = P.sub(1.0, wa)
                return (P.mul(g, wa) if _requires(a) else None, P.mul(g, wb) if _requires(b) else None)
            if isinstance(a, TensorProxy):
                m = P.convert_element_type(P.eq(out, a), g.dtype)
                return P.mul(g, m), None
            m = P.convert_element_type(P.eq(out, b), g.dtype)
            return None, P.mul(g, m)

        return out, bwd

    return rule


register_vjp(PrimIDs.MAXIMUM)(_maxmin_rule(P.maximum, P.gt))
register_vjp(PrimIDs.MINIMUM)(_maxmin_rule(P.minimum, P.lt))


@register_vjp(PrimIDs.COPYSIGN)
def _copysign_rule(a, b):
    out = P.copysign(a, b)

    def bwd(g):
        # d/da |a|*sign(b) = sign(a)*sign(out); b only contributes its sign (zero gradient)
        return P.mul(g, P.mul(P.sign(a), P.sign(out))), None

    return out, bwd


@register_vjp(PrimIDs.ATAN2)
def _atan2_rule(a, b):
    out = P.atan2(a, b)

    def bwd(g):
        denom = P.add(P.mul(a, a), P.mul(b, b))
        return P.div(P.mul(g, b), denom), P.neg(P.div(P.mul(g, a), denom))

    return out, bwd


@register_vjp(PrimIDs.REMAINDER)
def _remainder_rule(a, b):
    out = P.remainder(a, b)

    def bwd(g):
        gb = None
        if _requires(b):
            gb = P.neg(P.mul(g, P.floor(P.div(a, b))))
        return g, gb

    return out, bwd


@register_vjp(PrimIDs.FMOD)
def _fmod_rule(a, b):
    out = P.fmod(a, b)

    def bwd(g):
        gb = None
        if _requires(b):
            gb = P.neg(P.mul(g, P.trunc(P.div(a, b))))
        return g, gb

    return out, bwd


@register_vjp(PrimIDs.WHERE)
def _where_rule(pred, a, b):
    out = P.where(pred, a, b)

    def bwd(g):
        ga = P.where(pred, g, 0.0) if _requires(a) else None
        gb = P.where(pred, 0.0, g) if _requires(b) else None
        return None, ga, gb

    return out, bwd


@register_vjp(PrimIDs.CONVERT_ELEMENT_TYPE)
def _convert_rule(a, dtype):
    out = P.convert_element_type(a, dtype)

    def bwd(g):
        if not isinstance(a, TensorProxy):
            return None, None
        return P.convert_element_type(g, a.dtype) if g.dtype != a.dtype else g, None

    return out, bwd


@register_vjp(PrimIDs.DEVICE_PUT)
def _device_put_rule(a, device):
    out = P.device_put(a, device)

    def bwd(g):
        return P.device_put(g, a.device), None

    return out, bwd


@register_vjp(PrimIDs.SHALLOW_COPY)
def _shallow_copy_rule(a):
    out = P.shallow_copy(a)
    return out, lambda g: (g,)


@register_vjp(PrimIDs.BROADCAST_IN_DIM)
def _broadcast_in_dim_rule(a, shape, broadcast_dimensions):
    out = P.broadcast_in_dim(a, shape, broadcast_dimensions)

    def bwd(g):
        bd = list(broadcast_dimensions)
        # sum over dims not in broadcast_dimensions, and over dims where a had size 1 but out didn't
        reduce_dims = [i for i in range(len(shape)) if i not in bd]
        keep_reduce = [bd[i] for i in range(a.ndim) if a.shape[i] == 1 and shape[bd[i]] != 1]
        gg = g
        all_dims = sorted(set(reduce_dims + keep_reduce))
        if all_dims:
            gg = P.sum(gg, tuple(all_dims))
        return _clang().reshape(gg, a.shape), None, None

    return out, bwd


@register_vjp(PrimIDs.RESHAPE)
def _reshape_rule(a, shape):
    out = P.reshape(a, shape)
    return out, lambda g: (P.reshape(g, a.shape), None)


@register_vjp(PrimIDs.TRANSPOSE)
def _transpose_rule(a, permutation):
    out = P.transpose(a, permutation)
    inv = [0] * len(permutation)
    for i, p in enumerate(permutation):
        inv[p] = i
    return out, lambda g: (P.transpose(g, tuple(inv)), None)


@register_vjp(PrimIDs.SQUEEZE)
def _squeeze_rule(a, dims):
    out = P.squeeze(a, dims)
    return out, lambda g: (_clang().reshape(g, a.shape), None)


@register_vjp(PrimIDs.SLICE)
def _slice_rule(a, start_indices, end_indices, strides=None):
    out = P.slice_prim(a, start_indices, end_indices, strides)

    def bwd(g):
        st = strides if strides is not None else [1] * a.ndim
        cfg = []
        for s, e, stride, dimlen, gl in zip(start_indices, end_indices, st, a.shape, g.shape):
            interior = stride - 1
            used = s + (gl - 1) * stride + 1 if gl > 0 else s
            cfg.append((s, dimlen - used, interior))
        return P.pad(g, 0.0, cfg), None, None, None

    return out, bwd


@register_vjp(PrimIDs.PAD)
def _pad_rule(a, padding_value, padding_config):
    out = P.pad(a, padding_value, padding_config)

    def bwd(g):
        starts, ends, strides = [], [], []
        for (lo, hi, it), s in zip(padding_config, a.shape):
            starts.append(lo)
            ends.append(lo + s + max(s - 1, 0) * it)
            strides.append(it + 1)
        return P.slice_prim(g, starts, ends, strides), None, None

    return out, bwd


@register_vjp(PrimIDs.CAT)
def _cat_rule(tensors, dim):
    out = P.cat(tensors, dim)

    def bwd(g):
        grads = []
        start = 0
        for t in tensors:
            n = t.shape[dim]
            grads.append(_clang().slice_in_dim(g, start, start + n, 1, dim))
            start += n
        return grads, None

    return out, bwd


@register_vjp(PrimIDs.FLIP)
def _flip_rule(a, dims):
    out = P.flip(a, dims)
    return out, lambda g: (P.flip(g, dims), None)


@register_vjp(PrimIDs.TAKE)
def _take_rule(a, indices, dim):
    out = P.take(a, indices, dim)

    def bwd(g):
        z = zeros_like_proxy(a) if g.dtype == a.dtype else P.full(tuple(a.shape), 0, device=a.device, dtype=g.dtype)
        gi = g
        if indices.ndim != 1:
            shape = list(a.shape)
            shape[dim] = math.prod(indices.shape)
            gi = _clang().reshape(g, tuple(shape))
            idx = _clang().reshape(indices, (math.prod(indices.shape),))
        else:
            idx = indices
        return P.index_add(z, idx, gi, dim), None, None

    return out, bwd


@register_vjp(PrimIDs.TAKE_ALONG_AXIS)
def _take_along_axis_rule(a, indices, dim):
    out = P.take_along_axis(a, indices, dim)

    def bwd(g):
        z = P.full(tuple(a.shape), 0, device=a.device, dtype=g.dtype)
        return P.scatter_add(z, indices, g, dim), None, None

    return out, bwd


@register_vjp(PrimIDs.INDEX_ADD)
def _index_add_rule(a, indices, value, dim):
    out = P.index_add(a, indices, value, dim)

    def bwd(g):
        gv = P.take(g, indices, dim) if _requires(value) else None
        return g, None, gv, None

    return out, bwd


@register_vjp(PrimIDs.INDEX_PUT)
def _index_put_rule(a, indices, values, accumulate):
    """``out = a; out[indices] (+)= values`` (advanced indexing on the leading dims).  The values'
    gradient is the cotangent gathered at the same indices (summed back to a broadcast value's shape);
    with ``accumulate=False`` the overwritten positions get no gradient in ``a``."""
    out = P.index_put(a, indices, values, accumulate)

    def bwd(g):
        ga = g
        if not accumulate:
            zero = P.full(tuple(values.shape), 0, device=g.device, dtype=g.dtype)
            ga = P.index_put(g, indices, zero, False)
        gv = None
        if _requires(values):
            gv = _ltorch().getitem(g, tuple(indices))
            if tuple(gv.shape) != tuple(values.shape):
                gv = sum_to_shape(gv, values.shape)
            if gv.dtype != values.dtype:
                gv = _clang().maybe_convert_to_dtype(gv, values.dtype)
        return ga, None, gv, None

    return out, bwd


@register_vjp(PrimIDs.SCATTER)
def _scatter_rule(a, index, src, dim):
    """``out = a; out[index] = src`` along ``dim``: overwritten positions get no gradient in ``a``;
    ``src`` receives the cotangent gathered at ``index``."""
    out = P.scatter(a, index, src, dim)

    def bwd(g):
        zero = P.full(tuple(index.shape), 0, device=g.device, dtype=g.dtype)
        ga = P.scatter(g, index, zero, dim)
        gs = P.take_along_axis(g, index, dim) if _requires(src) else None
        return ga, None, gs, None

    return out, bwd


@register_vjp(PrimIDs.SCATTER_ADD)
def _scatter_add_rule(a, index, value, dim):
    out = P.scatter_add(a, index, value, dim)

    def bwd(g):
        gv = P.take_along_axis(g, index, dim) if _requires(value) else None
        return g, None, gv, None

    return out, bwd


def _restore_reduced(g, a, dims):
    shape = [1 if i in dims else s for i, s in enumerate(a.shape)]
    g = _clang().reshape(g, tuple(shape))
    return _clang().expand(g, a.shape)


@register_vjp(PrimIDs.SUM)
def _sum_rule(a, dims, *, output_dtype=None):
    out = P.sum(a, dims, output_dtype=output_dtype) if output_dtype else P.sum(a, dims)

    def bwd(g):
        gg = _restore_reduced(g, a, tuple(dims))
        if gg.dtype != a.dtype:
            gg = P.convert_element_type(gg, a.dtype)
        return gg, None

    return out, bwd


def _amax_like(fwd):
    def rule(a, dims, *, output_dtype=None):
        out = fwd(a, dims)

        def bwd(g):
            ob = _restore_reduced(out, a, tuple(dims))
            mask = P.convert_element_type(P.eq(a, ob), g.dtype)
            cnt = _restore_reduced(P.sum(mask, tuple(dims)), a, tuple(dims))
            gg = _restore_reduced(g, a, tuple(dims))
            return P.div(P.mul(gg, mask), cnt), None

        return out, bwd

    return rule


register_vjp(PrimIDs.AMAX)(_amax_like(P.amax))
register_vjp(PrimIDs.AMIN)(_amax_like(P.amin))


@register_vjp(PrimIDs.PROD)
def _prod_rule(a, dims, *, output_dtype=None):
    out = P.prod(a, dims)

    def bwd(g):
        ob = _restore_reduced(out, a, tuple(dims))
        gg = _restore_reduced(g, a, tuple(dims))
        return P.div(P.mul(gg, ob), a), None

    return out, bwd


@register_vjp(PrimIDs.VAR)
def _var_rule(a, dims, *, correction):
    out = P.var(a, dims, correction=correction)

    def bwd(g):
        n = math.prod(a.shape[d] for d in dims)
        mean = _restore_reduced(P.div(P.sum(a, tuple(dims)), float(n)), a, tuple(dims))
        gg = _restore_reduced(g, a, tuple(dims))
        return P.mul(P.mul(gg, P.sub(a, mean)), 2.0 / max(n - correction, 1)), None

    return out, bwd


@register_vjp(PrimIDs.VAR_MEAN)
def _var_mean_rule(a, dims, *, correction):
    v, m = P.var_mean(a, dims, correction=correction)

    def bwd(gv, gm):
        n = math.prod(a.shape[d] for d in dims)
        res = None
        if gv is not None:
            mb = _restore_reduced(m, a, tuple(dims))
            res = P.mul(P.mul(_restore_reduced(gv, a, tuple(dims)), P.sub(a, mb)), 2.0 / max(n - correction, 1))
        if gm is not None:
            t = P.div(_restore_reduced(gm, a, tuple(dims)), float(n))
            res = t if res is None else P.add(res, t)
        return res, None

    return (v, m), bwd


@register_vjp(PrimIDs.CUMSUM)
def _cumsum_rule(a, dim, *, dtype=None):
    out = P.cumsum(a, dim)

    def bwd(g):
        return P.flip(P.cumsum(P.flip(g, (dim,)), dim), (dim,)), None

    return out, bwd


@register_vjp(PrimIDs.MATMUL)
def _matmul_rule(a, b):
    out = P.matmul(a, b)

    def bwd(g):
        ltorch = _ltorch()
        ga = gb = None
        if a.ndim == 1 and b.ndim == 1:
            ga = P.mul(g, b) if _requires(a) else None
            gb = P.mul(g, a) if _requires(b) else None
            return ga, gb
        if a.ndim == 1:
            # (k) @ (..., k, n) -> (..., n)
            if _requires(a):
                ga = sum_to_shape(ltorch.squeeze(P.matmul(ltorch.unsqueeze(g, -2), ltorch.transpose(b, -1, -2)), -2), a.shape)
            if _requires(b):
                gb = sum_to_shape(P.matmul(ltorch.unsqueeze(a, -1), ltorch.unsqueeze(g, -2)), b.shape)
            return ga, gb
        if b.ndim == 1:
            if _requires(a):
                ga = sum_to_shape(P.matmul(ltorch.unsqueeze(g, -1), ltorch.unsqueeze(b, 0)), a.shape)
            if _requires(b):
                gb = sum_to_shape(ltorch.squeeze(P.matmul(ltorch.transpose(a, -1, -2), ltorch.unsqueeze(g, -1)), -1), b.shape)
            return ga, gb
        if _requires(a):
            ga = sum_to_shape(P.matmul(g, ltorch.transpose(b, -1, -2)), a.shape)
        if _requires(b):
            gb = sum_to_shape(P.matmul(ltorch.transpose(a, -1, -2), g), b.shape)
        return ga, gb

    return out, bwd


def linear_backward(a, w, bias, g):
    """dgrad = g @ W ; wgrad = g^T @ a (flattened over leading dims) ; bgrad = sum(g)."""
    ltorch = _ltorch()
    ga = gw = gb = None
    if _requires(a):
        ga = P.matmul(g, w)
    if _requires(w):
        g2 = _clang().reshape(g, (-1, g.shape[-1]))
        a2 = _clang().reshape(a, (-1, a.shape[-1]))
        gw = P.matmul(ltorch.transpose(g2, 0, 1), a2)
    if bias is not None and _requires(bias):
        # summed over g's own leading dims (no flattening reshape): a fusion region producing g (an
        # activation / dropout backward) then also emits the bias gradient as its column reduction
        gb = ltorch.sum(g, tuple(range(g.ndim - 1))) if g.ndim > 1 else g
    return ga, gw, gb


@register_vjp(PrimIDs.LINEAR)
def _linear_rule(a, w, bias=None):
    out = P.linear(a, w, bias)
    return out, lambda g: linear_backward(a, w, bias, g)


@register_vjp(PrimIDs.EMBEDDING)
def _embedding_rule(a, weight, *, padding_idx=-1, max_norm=None, norm_type=2.0, scale_grad_by_freq=False, sparse=False):
    out = P.embedding(a, weight, padding_idx=padding_idx, max_norm=max_norm, norm_type=norm_type,
                      scale_grad_by_freq=scale_grad_by_freq, sparse=sparse)

    def bwd(g):
        gw = P.embedding_backward(g, a, weight.shape[0], padding_idx, scale_grad_by_freq, sparse)
        return None, gw

    return out, bwd


@register_vjp(PrimIDs.COPY_)
def _copy_rule(copy_from, copy_to):
    out = P.copy_(copy_from, copy_to)
    return out, lambda g: (g, None)


for _nd in (PrimIDs.FULL, PrimIDs.IOTA, PrimIDs.UNIFORM, PrimIDs.UNIFORM_PHILOX, PrimIDs.RANDN, PrimIDs.EMPTY,
            PrimIDs.EQ, PrimIDs.NE, PrimIDs.LT, PrimIDs.LE, PrimIDs.GT, PrimIDs.GE, PrimIDs.ISFINITE,
            PrimIDs.SIGNBIT, PrimIDs.ARGMAX, PrimIDs.ARGMIN, PrimIDs.BITWISE_AND, PrimIDs.BITWISE_OR,
            PrimIDs.BITWISE_XOR, PrimIDs.BITWISE_NOT, PrimIDs.ITEM, PrimIDs.TENSOR_FROM_SEQUENCE, PrimIDs.BITCAST):
    _vjp_rules[_nd] = None  # explicitly non-differentiable


@register_vjp(PrimIDs.TOPK)
def _topk_rule(a, k, dim, largest, sorted):
    v, i = P.topk(a, k, dim, largest, sorted)

    def bwd(gv, gi=None):
        z = P.full(tuple(a.shape), 0, device=a.device, dtype=gv.dtype)
        return P.scatter_add(z, i, gv, dim), None, None, None, None

    return (v, i), bwd


@register_vjp(PrimIDs.SORT)
def _sort_rule(a, dim, descending, stable):
    v, i = P.sort(a, dim, descending, stable)

    def bwd(gv, gi=None):
        z = P.full(tuple(a.shape), 0, device=a.device, dtype=gv.dtype)
        return P.scatter_add(z, i, gv, dim), None, None, None

    return (v, i), bwd


NON_DIFFERENTIABLE = object()


def add_transform(cfn, *, transform, disable_torch_autograd_support=False, _legacy_copy_params=False):
    """Re-jits ``cfn`` with an additional transform (reference :430-467)."""
    from ..common import compile_data_of
    from .. import jit

    cd = compile_data_of(cfn)
    if cd is None:
        raise ValueError("add_transform expects a function/module compiled with lightning_thunder_amd.jit")
    transforms = list(cd.transforms) + (list(transform) if isinstance(transform, (list, tuple)) else [transform])
    return jit(
        cd.fn,
        executors=cd.executors_list,
        cache=cd.cache_option,
        disable_torch_autograd=cd.disable_torch_autograd or disable_torch_autograd_support,
        transforms=transforms,
        debug_options=cd.debug_options,
        **cd.compile_options,
    )


# -----------------------------------------------------------------------------------------
# Joint-style gradient registration (reference ``register_grad`` :620 with ``get_grad`` /
# ``put_grad``): ``gradfn(*args)`` computes the forward, reads output cotangents with
# ``get_grad(out)`` and deposits input gradients with ``put_grad(arg, g)`` -- one function for both
# directions.  Here it is converted into a VJP rule by recording what gradfn traces: the ops that
# depend on a ``get_grad`` placeholder (transitively) are the backward and are replayed, with the
# real cotangents substituted, when autodiff reaches the op; the rest stay in the forward trace.
# -----------------------------------------------------------------------------------------
import threading as _threading

_joint = _threading.local()


def get_grad(x):
    """The cotangent of forward value ``x`` (only inside a ``register_grad`` gradient function)."""
    st = getattr(_joint, "state", None)
    if st is None:
        raise RuntimeError("get_grad is only valid inside a gradient function registered with register_grad")
    if not isinstance(x, TensorProxy):
        return None
    ph = TensorProxy(like=x, requires_grad=False, prefix="gct")
    st["get"][ph.name] = x
    return ph


def put_grad(x, g) -> None:
    """Accumulates ``g`` into the gradient of ``x`` (only inside a ``register_grad`` gradient function)."""
    st = getattr(_joint, "state", None)
    if st is None:
        raise RuntimeError("put_grad is only valid inside a gradient function registered with register_grad")
    if isinstance(x, TensorProxy) and g is not None:
        st["put"].append((x, g))


def register_grad(sym_or_id, gradfn: Callable) -> None:
    """Registers a joint forward/backward gradient function for a symbol (see ``get_grad`` /
    ``put_grad``); it takes precedence like any registered VJP rule."""
    from .trace import get_tracectx

    def rule(*args, **kwargs):
        trc = get_tracectx()
        scope = trc.scopes[-1]
        n0 = len(scope)
        prev = getattr(_joint, "state", None)
        _joint.state = st = {"get": {}, "put": []}
        try:
            out = gradfn(*args, **kwargs)
        finally:
            _joint.state = prev
        recorded = scope[n0:]
        del scope[n0:]
        # split: backward = ops reached from a get_grad placeholder
        tainted = set(st["get"])
        fwd, bwd_ops = [], []
        for b in recorded:
            if any(a.name in tainted for a in b.flat_proxy_args):
                bwd_ops.append(b)
                tainted.update(o.name for o in b.flat_proxy_outs)
            else:
                fwd.append(b)
        scope.extend(fwd)
        flat_out = [o for o in tree_flatten(out)[0] if isinstance(o, TensorProxy)]
        puts = st["put"]
        placeholders = dict(st["get"])

        def backward(*cts):
            swap = {}
            for ph_name, x in placeholders.items():
                ct = None
                for o, c in zip(flat_out, cts):
                    if o is x or o.name == x.name:
                        ct = c
                        break
                if ct is None:
                    ct = P.full(tuple(x.shape), 0, device=x.device, dtype=x.dtype)
                swap[ph_name] = ct
            cur = get_tracectx()
            for b in bwd_ops:
                cur.scopes[-1].append(b.swap_proxies(swap, skip_output=True))
            grads = {}
            for x, g in puts:
                if isinstance(g, Proxy) and g.name in swap:
                    g = swap[g.name]
                grads[x.name] = g if x.name not in grads else _ltorch().add(grads[x.name], g)
            return tuple(grads.get(a.name) if isinstance(a, TensorProxy) else None for a in args)

        return out, backward

    register_vjp(sym_or_id)(rule)


# -----------------------------------------------------------------------------------------
# Functional transforms (reference ``vjp`` :3041, ``value_and_grad`` :3068, ``grad`` :1518):
# evaluated through the compiled program's own forward/backward traces.
# -----------------------------------------------------------------------------------------
def _diff_inputs(primals):
    out = []
    for p in primals:
        if isinstance(p, torch.Tensor) and (p.is_floating_point() or p.is_complex()):
            out.append(p.detach().requires_grad_(True))
        else:
            out.append(p)
    return out


def _vjp_run(jf, primals, kwargs, make_cotangents):
    ins = _diff_inputs(primals)
    out = jf(*ins, **kwargs)
    cotangents = make_cotangents(out)
    flat_out = [o for o in tree_flatten(out)[0] if isinstance(o, torch.Tensor)]
    flat_ct = tree_flatten(cotangents)[0] if cotangents is not None else []
    pairs = [(o, c) for o, c in zip(flat_out, flat_ct) if c is not None and o.requires_grad]
    diff = [p for p in ins if isinstance(p, torch.Tensor) and p.requires_grad]
    if pairs and diff:
        grads = torch.autograd.grad([o for o, _ in pairs], diff, [c for _, c in pairs], allow_unused=True)
    else:
        grads = [None] * len(diff)
    it = iter(grads)
    full = tuple(next(it) if isinstance(p, torch.Tensor) and p.requires_grad else None for p in ins)
    return out, full


def vjp(func):
    """``vjp(func)(primals, cotangents, **kwargs) -> (outputs, grads)``: outputs of ``func(*primals)``
    and the vector-Jacobian products of ``cotangents`` w.r.t. each primal (None where not
    differentiable), computed by the compiled forward and backward programs."""
    from .. import jit

    jf = jit(func)

    def _vjp(primals, cotangents, **kwargs):
        if not isinstance(primals, (tuple, list)):
            primals = (primals,)
        return _vjp_run(jf, primals, kwargs, lambda out: cotangents)

    return _vjp


def value_and_grad(func):
    """``value_and_grad(func)(*args, **kwargs) -> (value, grads)``: all-ones cotangents."""
    from .. import jit

    jf = jit(func)

    def ones(out):
        return tree_map(lambda o: torch.ones_like(o) if isinstance(o, torch.Tensor) and o.is_floating_point() else None, out)

    def _value_and_grad(*args, **kwargs):
        return _vjp_run(jf, args, kwargs, ones)

    return _value_and_grad


def eval_trace(trace, *args, symbol_mapper=None, with_env: bool = False, **kwargs):
    """Evaluates ``trace`` on ``args`` bound symbol by bound symbol, each through
    ``symbol_mapper(bsym)`` (default: the symbol itself) — reference ``core/transforms.py``
    ``eval_trace``; see ``core/trace_interpreter.interpret_trace``."""
    from .trace_interpreter import interpret_trace

    return interpret_trace(trace, *args, symbol_mapper=symbol_mapper, with_env=with_env, **kwargs)
