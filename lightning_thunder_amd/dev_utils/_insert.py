"""Helpers for transforms that insert host-side calls between bound symbols."""
from __future__ import annotations

import itertools

from ..core.symbol import Symbol, BoundSymbol

_ids = itertools.count()


def host_call(name: str, fn, args=(), output=None) -> BoundSymbol:
    """A bound symbol that calls ``fn(*args)`` on the host (python executor)."""
    from ..executors.pythonex import ex as pyex

    nm = f"{name}_{next(_ids)}"
    sym = Symbol(nm, meta=None, is_prim=True, executor=pyex)
    return BoundSymbol(sym, args=tuple(args), kwargs={}, output=output, _call_ctx={nm: fn})


SKIP = ("unpack_trivial", "unpack_sequence", "python_return", "python_del", "unpack_key", "unpack_attr")
