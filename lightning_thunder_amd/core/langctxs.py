"""Language contexts (reference ``thunder/core/langctxs.py``): which language resolves method
calls on proxies (``t.sum()`` -> ``ltorch.sum`` under TORCH, ``numpy.size`` under NUMPY)."""
from __future__ import annotations

import contextlib
from contextvars import ContextVar
from enum import Enum, auto


class Languages(Enum):
    TORCH = auto()
    CLANG = auto()
    PRIMS = auto()
    NUMPY = auto()


_langctx: ContextVar = ContextVar("langctx", default=Languages.TORCH)


def get_langctx() -> Languages:
    return _langctx.get()


def set_langctx(lang: Languages):
    return _langctx.set(lang)


def reset_langctx(tok) -> None:
    _langctx.reset(tok)


@contextlib.contextmanager
def langctx(lang: Languages):
    tok = _langctx.set(lang)
    try:
        yield
    finally:
        _langctx.reset(tok)


def resolve_method(name: str):
    """The symbol implementing method ``name`` in the active language."""
    lang = get_langctx()
    if lang is Languages.NUMPY:
        from ..numpy import get_method

        return get_method(name)
    if lang in (Languages.TORCH,):
        from ..torch import get_method

        return get_method(name)
    from .. import clang

    return getattr(clang, name, None)
