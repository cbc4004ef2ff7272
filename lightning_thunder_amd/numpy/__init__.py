"""Minimal NumPy language context (reference ``thunder/numpy/__init__.py``: ``npsymbol``, ``size``,
``len``, ``add``): lets programs written against NumPy-style calls be traced into the same
prims as the torch language."""
from __future__ import annotations

import builtins
from numbers import Number

from .. import clang
from ..core.proxies import TensorProxy
from ..core.symbol import Symbol

_np_symbols: dict[str, Symbol] = {}


class npsymbol:
    def __init__(self, *, method_name: str | None = None):
        self.method_name = method_name

    def __call__(self, fn):
        sym = Symbol(fn.__name__, fn, id=f"numpy.{fn.__name__}", module="numpy")
        _np_symbols[self.method_name or fn.__name__] = sym
        return sym


@npsymbol(method_name="len")
def compute_len(a: TensorProxy, /) -> int:
    if a.ndim == 0:
        raise TypeError("len() of a 0-d tensor")
    return a.shape[0]


@npsymbol(method_name="size")
def size(a: TensorProxy, /) -> int:
    n = 1
    for s in a.shape:
        n *= s
    return n


@npsymbol(method_name="add")
def add(a: Number | TensorProxy, b: Number | TensorProxy, /, *, where: None | Number | TensorProxy = None):
    if where is not None:
        return clang.where(where, clang.add(a, b), a)
    return clang.add(a, b)


def get_method(name: str):
    return _np_symbols.get(name)
