"""Printing of values into trace source (parity: reference ``thunder/core/codeutils.py:44,144,314,403``).

Values that are not representable as Python literals (process groups, callables,
arbitrary objects) are registered into the trace's object context and printed
by name, so every trace stays executable Python.
"""
from __future__ import annotations

import math
from contextlib import contextmanager
from contextvars import ContextVar
from enum import Enum
from numbers import Number
from typing import Any

import torch

from .proxies import Proxy, NumberProxy
from .symbolic import SymInt

# symbols the program being printed binds from its arguments (None: not printing a program — show
# every expression); a SymInt over any other symbol is printed as its value and specialized
_bindable: ContextVar = ContextVar("lta_bindable_syms", default=None)


_used: ContextVar = ContextVar("lta_used_syms", default=None)


@contextmanager
def bindable_symbols(names, used: set | None = None):
    """Prints SymInts over ``names`` as expressions (collecting the symbols printed into ``used``)."""
    tok = _bindable.set(set(names))
    tok2 = _used.set(used)
    try:
        yield
    finally:
        _used.reset(tok2)
        _bindable.reset(tok)


def _print_symint(x: SymInt) -> str:
    ok = _bindable.get()
    free = x.free_symbols()
    expr = x.expr
    if ok is not None and not free <= ok:
        # a symbol the program cannot bind may equal (a recorded guard) one it can
        from .symbolic import current_env
        import re

        env = current_env()
        for s in free - ok:
            alt = next((e for e in (env.equivalents(s) if env is not None else ()) if e in ok), None)
            if alt is None:
                return repr(int(x))  # int() specializes the program on this value
            expr = re.sub(rf"\b{s}\b", alt, expr)
        free = set(re.findall(r"\bs\d+\b", expr))
    used = _used.get()
    if used is not None:
        used.update(free)
    return expr


class ContextObject:
    """A named object placed in the generated program's globals."""

    def __init__(self, name: str, obj: Any):
        self.name = name
        self.obj = obj

    def __repr__(self):
        return self.name


def is_literal(x) -> bool:
    if x is None or isinstance(x, (bool, int, str, torch.dtype, torch.device, slice, type(Ellipsis))):
        return True
    if isinstance(x, float):
        return True
    if isinstance(x, complex):
        return True
    if isinstance(x, (tuple, list)):
        return all(is_literal(v) or isinstance(v, Proxy) for v in x)
    return False


def prettyprint(x: Any, obj_ctx: dict[str, Any] | None = None, *, with_type: bool = False) -> str:
    """Returns python source that evaluates to ``x`` in a trace program."""
    if isinstance(x, ContextObject):
        if obj_ctx is not None:
            obj_ctx[x.name] = x.obj
        return x.name
    if isinstance(x, Proxy):
        return x.name
    if x is None:
        return "None"
    if x is Ellipsis:
        return "..."
    if isinstance(x, bool):
        return repr(x)
    if isinstance(x, SymInt):
        return _print_symint(x)
    if isinstance(x, int):
        return repr(x)
    if isinstance(x, float):
        if math.isnan(x):
            return "float('nan')"
        if math.isinf(x):
            return "float('inf')" if x > 0 else "-float('inf')"
        return repr(x)
    if isinstance(x, complex):
        return f"complex({prettyprint(x.real)}, {prettyprint(x.imag)})"
    if isinstance(x, str):
        return repr(x)
    if isinstance(x, torch.dtype):
        return str(x)  # "torch.float32"
    if isinstance(x, torch.device):
        return f'torch.device("{x}")'
    if isinstance(x, torch.Size):
        return "(" + "".join(prettyprint(v, obj_ctx) + ", " for v in x) + ")"
    if isinstance(x, slice):
        return f"slice({prettyprint(x.start, obj_ctx)}, {prettyprint(x.stop, obj_ctx)}, {prettyprint(x.step, obj_ctx)})"
    if isinstance(x, tuple):
        if hasattr(type(x), "_fields"):
            return _register(x, obj_ctx)
        if len(x) == 1:
            return "(" + prettyprint(x[0], obj_ctx) + ",)"
        return "(" + ", ".join(prettyprint(v, obj_ctx) for v in x) + ")"
    if isinstance(x, list):
        return "[" + ", ".join(prettyprint(v, obj_ctx) for v in x) + "]"
    if isinstance(x, dict):
        return "{" + ", ".join(f"{prettyprint(k, obj_ctx)}: {prettyprint(v, obj_ctx)}" for k, v in x.items()) + "}"
    if isinstance(x, type) and x in (bool, int, float, complex):
        return x.__name__
    if isinstance(x, Enum):
        return _register(x, obj_ctx, hint=f"{type(x).__name__}_{x.name}")
    if isinstance(x, Number):
        return repr(x)
    return _register(x, obj_ctx)


_obj_names: dict[int, str] = {}
_obj_counter = [0]


def _register(x, obj_ctx, hint: str | None = None) -> str:
    key = id(x)
    name = _obj_names.get(key)
    if name is None:
        base = hint or type(x).__name__
        base = "".join(c if c.isalnum() else "_" for c in base)
        name = f"_{base}_{_obj_counter[0]}"
        _obj_counter[0] += 1
        _obj_names[key] = name
    if obj_ctx is not None:
        obj_ctx[name] = x
    return name


def print_output_target(out: Any) -> str:
    """Assignment target for a bound symbol's output structure."""
    if isinstance(out, Proxy):
        return out.name
    if isinstance(out, (tuple, list)):
        if len(out) == 0:
            return "_"
        inner = ", ".join(print_output_target(o) for o in out)
        if len(out) == 1:
            inner += ","
        return f"({inner})"
    return "_"


def has_proxy_output(out: Any) -> bool:
    if isinstance(out, Proxy):
        return True
    if isinstance(out, (tuple, list)):
        return any(has_proxy_output(o) for o in out)
    return False


def type_comment(out: Any) -> str:
    from .pytree import tree_flatten

    leaves, _ = tree_flatten(out)
    parts = [f'{p.name}: "{p.type_string()}"' for p in leaves if isinstance(p, Proxy) and not isinstance(p, NumberProxy)]
    return ", ".join(parts)


def sanitize_name(s: str) -> str:
    out = "".join(c if c.isalnum() else "_" for c in s)
    if not out or out[0].isdigit():
        out = "_" + out
    return out
