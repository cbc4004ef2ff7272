"""Autocast inside traces (parity: reference ``thunder/transforms/autocast.py:23-310``;
hook in ``Symbol.__call__`` as at reference ``thunder/core/symbol.py:294-298``).

When ``torch.autocast`` is active at call time the cache key records it and the
trace is acquired with an autocast dtype: matmul-like ops (linear, matmul, bmm,
SDPA, conv) are rewritten to cast their floating inputs to that dtype, matching
PyTorch's autocast op lists.  ``autocast(fn, dtype)`` returns a function traced
as if under autocast.
"""
from __future__ import annotations

import contextlib
import functools
from typing import Callable

import torch

from ..core.proxies import TensorProxy
from ..core import dtypes

_rules: dict = {}


def _cast(x, dtype):
    from .. import clang

    if isinstance(x, TensorProxy) and dtypes.is_float_dtype(x.dtype) and x.dtype != dtype:
        return clang.maybe_convert_to_dtype(x, dtype)
    return x


def _install_rules():
    if _rules:
        return
    from .. import torch as ltorch

    def lin(a, w, bias=None, *, dtype):
        return ltorch.linear(_cast(a, dtype), _cast(w, dtype), _cast(bias, dtype))

    def mm(a, b, *, dtype):
        return ltorch.matmul(_cast(a, dtype), _cast(b, dtype))

    def bmm(a, b, *, dtype):
        return ltorch.bmm(_cast(a, dtype), _cast(b, dtype))

    def sdpa(q, k, v, attn_mask=None, dropout_p=0.0, is_causal=False, *, scale=None, enable_gqa=False, dtype):
        return ltorch.scaled_dot_product_attention(_cast(q, dtype), _cast(k, dtype), _cast(v, dtype), attn_mask, dropout_p,
                                                   is_causal, scale=scale, enable_gqa=enable_gqa)

    _rules[ltorch.linear.id] = lin
    _rules[ltorch.matmul.id] = mm
    _rules[ltorch.mm.id] = mm
    _rules[ltorch.bmm.id] = bmm
    _rules[ltorch.scaled_dot_product_attention.id] = sdpa


def maybe_autocast(sym):
    _install_rules()
    rule = _rules.get(sym.id)
    if rule is None:
        return None

    def apply(*args, dtype, **kwargs):
        from ..core.trace import get_tracectx

        trc = get_tracectx()
        prev = trc.autocast_dtype
        trc.autocast_dtype = None  # avoid re-entry while the rule calls the op
        try:
            return rule(*args, dtype=dtype, **kwargs)
        finally:
            trc.autocast_dtype = prev

    return apply


_active_autocast = [None]


@contextlib.contextmanager
def autocast_ctx(key):
    """Sets the autocast dtype seen by traces acquired in this context (key from the cache info)."""
    prev = _active_autocast[0]
    _active_autocast[0] = key[1] if key is not None else None
    try:
        yield
    finally:
        _active_autocast[0] = prev


def current_autocast_dtype():
    return _active_autocast[0]


def autocast(fn: Callable, dtype: torch.dtype = torch.bfloat16) -> Callable:
    """Functional autocast: ``jit(autocast(f, torch.bfloat16))`` traces ``f`` with autocast rules."""

    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        from ..core.trace import get_tracectx

        trc = get_tracectx()
        if trc is None:
            with torch.autocast("cuda" if torch.cuda.is_available() else "cpu", dtype=dtype):
                return fn(*args, **kwargs)
        prev = trc.autocast_dtype
        trc.autocast_dtype = dtype
        try:
            return fn(*args, **kwargs)
        finally:
            trc.autocast_dtype = prev

    return wrapper
