"""Small base utilities (parity: reference ``thunder/core/baseutils.py:151,497-523,621``).

``build_callable`` compiles generated trace source, registering it with
``linecache`` so tracebacks and ``inspect.getsource`` point at the generated
program — traces are debuggable Python, as in the reference.
"""
from __future__ import annotations

import functools
import itertools
import linecache
import os
from typing import Any, Callable


class ThunderError(RuntimeError):
    pass


def check(cond: bool, msg: Callable[[], str] | str, exception_type=RuntimeError) -> None:
    if not cond:
        raise exception_type(msg() if callable(msg) else msg)


def check_type(x, types, name: str = "value") -> None:
    if not isinstance(x, types):
        raise ValueError(f"{name} has type {type(x)}, expected {types}")


def check_valid_length(n: int) -> None:
    check(isinstance(n, int) and n >= 0, lambda: f"Invalid length {n}")


def check_valid_shape(shape) -> None:
    for s in shape:
        check_valid_length(s)


_callable_counter = itertools.count()


def build_callable(name: str, python_str: str, ctx: dict[str, Any], file_name: str | None = None) -> Callable:
    """Compiles ``python_str`` (which defines ``name``) with globals ``ctx`` and returns the function."""
    if file_name is None:
        file_name = f"thunder.{name}_{next(_callable_counter)}"
    code = compile(python_str, file_name, mode="exec")
    lines = python_str.splitlines(keepends=True)
    linecache.cache[file_name] = (len(python_str), None, lines, file_name)
    glbs = dict(ctx)
    exec(code, glbs)
    fn = glbs[name]
    fn.__thunder_source__ = python_str
    return fn


def run_once(fn: Callable) -> Callable:
    done = False
    result = None

    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        nonlocal done, result
        if not done:
            result = fn(*args, **kwargs)
            done = True
        return result

    return wrapper


def env_flag(name: str, default: bool = False) -> bool:
    v = os.environ.get(name)
    if v is None:
        return default
    return v not in ("0", "", "false", "False", "no")


class TagBase:
    """Tags are singletons identified by name; used for OpTags/ProxyTags/BoundSymbolTags."""

    _registry: dict[str, "TagBase"] = {}

    def __init__(self, name: str):
        self.name = name

    def __repr__(self):
        return f"{type(self).__name__}.{self.name}"


def sequencify(x):
    if isinstance(x, (list, tuple)):
        return x
    return (x,)


def indent(level: int) -> str:
    return "  " * level
