"""Traces: straight-line programs of bound symbols (parity: reference ``thunder/core/trace.py:46-503``,
``python`` :349, ``python_callable`` :461, ``from_trace`` :507, ``tracectx`` :573).

A ``TraceCtx`` owns a list of ``BoundSymbol`` s, a flat signature of input
proxies and a name table.  ``python()`` prints the program and
``python_callable()`` compiles it.  An optional execution-file hook lets a
user inspect and edit generated programs before they run.
"""
from __future__ import annotations

import contextlib
import os
import time
from collections import defaultdict
from contextvars import ContextVar
from typing import Any, Callable

from .baseutils import build_callable
from .codeutils import prettyprint, sanitize_name, bindable_symbols
from .proxies import Proxy, TensorProxy

_tracectx: ContextVar = ContextVar("tracectx", default=None)


def get_tracectx() -> "TraceCtx | None":
    return _tracectx.get()


def set_tracectx(trc):
    return _tracectx.set(trc)


def reset_tracectx(tok):
    _tracectx.reset(tok)


@contextlib.contextmanager
def tracectx(trc: "TraceCtx | None"):
    tok = _tracectx.set(trc)
    try:
        yield trc
    finally:
        _tracectx.reset(tok)


@contextlib.contextmanager
def detached_trace():
    """Runs code under a throwaway trace (used when probing metas)."""
    trc = TraceCtx()
    with tracectx(trc):
        yield trc


class TraceProvenance:
    def __init__(self, pss: str):
        self.pss = pss

    def __repr__(self):
        return f"# Constructed by {self.pss}"


class TraceTag:
    AUGMENTED_FORWARD = "augmented_forward"
    BACKWARD = "backward"
    PROLOGUE = "prologue"
    EPILOGUE = "epilogue"


_execution_file: str | None = None


def _set_execution_file(path: str | None) -> None:
    """If set, programs are written to ``path`` before running; if the user edited it, the edited program runs."""
    global _execution_file
    _execution_file = path


class TraceCtx:
    def __init__(self, fn: Callable | None = None, *, prologue: "TraceCtx | None" = None):
        self.fn = fn
        self.args: list = []
        self.kwargs: dict = {}
        self.bound_symbols: list = []
        self.scopes: list[list] = [self.bound_symbols]
        self.names: set[str] = set()
        self._counters: dict[str, int] = defaultdict(int)
        self._provenance: TraceProvenance | None = None
        self.fn_name = getattr(fn, "__name__", None) if fn is not None and not isinstance(fn, str) else None
        if self.fn_name is None or not self.fn_name.isidentifier() or self.fn_name == "<lambda>":
            self.fn_name = "computation"
        self.prologue = prologue
        self.tags: set = set()
        self.decorators: list[str] = []
        self.extra_imports: dict[str, Any] = {}
        self.obj_ctx: dict[str, Any] = {}
        # Autocast / compile data snapshot that Symbol.__call__ consults while tracing
        self.autocast_dtype = None
        self.ignored_names: set[str] = set()
        self.unpack_list_arg = False
        # set by the acquisition frontend (core/functionalization.AliasTracker)
        self.alias_tracker = None

    # --- names ------------------------------------------------------------------------
    def add_name(self, name: str) -> None:
        if name in self.names:
            raise RuntimeError(f"Trying to add the name {name} to a trace, but that name is already used")
        self.names.add(name)

    def has_name(self, name: str) -> bool:
        return name in self.names

    def make_name(self, prefix: str = "t") -> str:
        while True:
            n = self._counters[prefix]
            self._counters[prefix] = n + 1
            name = f"{prefix}{n}"
            if name not in self.names:
                self.names.add(name)
                return name

    def make_unique_name(self, base: str) -> str:
        """A fresh name derived from ``base`` (not yet registered: the proxy constructor adds it)."""
        base = sanitize_name(base)
        if base not in self.names:
            return base
        i = 0
        while f"{base}_{i}" in self.names:
            i += 1
        return f"{base}_{i}"

    # --- scopes -------------------------------------------------------------------------
    def add_bound_symbol(self, bsym) -> None:
        self.scopes[-1].append(bsym)

    def push_scope(self, scope: list) -> None:
        self.scopes.append(scope)

    def pop_scope(self) -> list:
        return self.scopes.pop()

    # --- provenance -------------------------------------------------------------------------
    def set_provenance(self, provenance: TraceProvenance | str) -> None:
        if isinstance(provenance, str):
            provenance = TraceProvenance(provenance)
        self._provenance = provenance

    def get_provenance(self):
        return self._provenance

    # --- signature ----------------------------------------------------------------------------
    def set_signature(self, args: list, fn_name: str | None = None) -> None:
        self.args = list(args)
        if fn_name is not None:
            self.fn_name = fn_name

    @property
    def output(self):
        from . import prims

        for bsym in reversed(self.bound_symbols):
            if bsym.sym.id == prims.PrimIDs.RETURN:
                return bsym.args[0] if len(bsym.args) == 1 else bsym.args
        return None

    # --- printing ------------------------------------------------------------------------------
    def python_ctx(self) -> dict[str, Any]:
        import torch

        from . import prims
        from .. import torch as ltorch
        from .. import clang

        ctx = {"torch": torch, "prims": prims, "ltorch": ltorch, "clang": clang, "inf": float("inf"), "nan": float("nan")}
        ctx.update(self.extra_imports)
        ctx.update(self.obj_ctx)
        return ctx

    def python(self, *, print_depth: int = 1, include_decorators: bool = True) -> str:
        obj_ctx: dict[str, Any] = {}
        lines: list[str] = []
        if self._provenance is not None:
            lines.append(repr(self._provenance))
        lines.append("import torch")
        if include_decorators:
            lines.extend(self.decorators)
        arg_names = []
        for a in self.args:
            arg_names.append(a.name if isinstance(a, Proxy) else prettyprint(a, obj_ctx))
        if self.unpack_list_arg:
            # Takes one mutable list and clears it, so the caller's references (e.g. saved-for-backward
            # tensors) die as soon as this frame drops them (reference: torch_autograd.py:95-115).
            lines.append(f"def {self.fn_name}(args):")
            if arg_names:
                lines.append(f"  ({', '.join(arg_names)},) = args")
            lines.append("  args.clear()")
        else:
            lines.append(f"def {self.fn_name}({', '.join(arg_names)}):")
        for a in self.args:
            if isinstance(a, Proxy):
                lines.append(f'  # {a.name}: "{a.type_string()}"')
        # symbolic dims (cache="symbolic values"): bound from this program's own tensor arguments
        binds = _symbol_bindings(self.args)
        body = []
        used: set = set()
        with bindable_symbols(binds.keys(), used):
            for bsym in self.bound_symbols:
                body.extend(bsym.python(indent=1, print_depth=print_depth, obj_ctx=obj_ctx))
        for sym, (arg, d) in binds.items():
            if sym in used:
                lines.append(f"  {sym} = {arg}" if d is None else f"  {sym} = {arg}.shape[{d}]")
        if not body:
            body = ["  pass"]
        lines.extend(body)
        self.obj_ctx.update(obj_ctx)
        return "\n".join(lines) + "\n"

    def save_trace(self, filename) -> None:
        """Writes the program (``python()``) to ``filename`` (reference ``TraceCtx.save_trace``)."""
        import os

        with open(os.fspath(filename), "w") as f:
            f.write(self.python())

    def python_callable(self, *, global_dicts: dict | None = None, **kwargs) -> Callable:
        src = self.python(**kwargs)
        ctx = self.python_ctx()
        for bsym in _iter_all_bsyms(self.bound_symbols):
            if bsym._call_ctx:
                ctx.update(bsym._call_ctx)
        if global_dicts:
            ctx.update(global_dicts)
        if _execution_file is not None:
            src = _maybe_replace_with_user_program(src, self.fn_name)
        fn = build_callable(self.fn_name, src, ctx)
        fn.__thunder_trace__ = self
        return fn

    def __repr__(self) -> str:
        return self.python()

    def __str__(self) -> str:
        return self.python()


def _symbol_bindings(args) -> dict:
    """symbol -> (argument name, dim) for every symbolic dim a tensor argument carries bare."""
    from .symbolic import SymInt

    out: dict = {}
    for a in args:
        if isinstance(a, TensorProxy):
            for d, s in enumerate(a._shape):
                if isinstance(s, SymInt) and s.expr.isidentifier() and s.expr not in out:
                    out[s.expr] = (a.name, d)
        elif getattr(a, "_sym", None) is not None and a._sym not in out:  # an int size argument
            out[a._sym] = (a.name, None)
    return out


def _iter_all_bsyms(bsyms):
    for b in bsyms:
        yield b


def _maybe_replace_with_user_program(src: str, name: str) -> str:
    path = _execution_file
    key = f"{path}.{name}.orig"
    if os.path.exists(path) and os.path.exists(key):
        with open(key) as f:
            orig = f.read()
        with open(path) as f:
            cur = f.read()
        if orig == src and cur != src:
            return cur
    with open(path, "w") as f:
        f.write(src)
    with open(key, "w") as f:
        f.write(src)
    return src


def from_trace(trace: TraceCtx) -> TraceCtx:
    """A new, empty trace with the same signature and name table."""
    t = TraceCtx(trace.fn)
    t.args = list(trace.args)
    t.kwargs = dict(trace.kwargs)
    t.names = set(trace.names)
    t._counters = defaultdict(int, trace._counters)
    t.fn_name = trace.fn_name
    t.prologue = trace.prologue
    t.tags = set(trace.tags)
    t.decorators = list(trace.decorators)
    t.extra_imports = dict(trace.extra_imports)
    t.obj_ctx = dict(trace.obj_ctx)
    t.unpack_list_arg = trace.unpack_list_arg
    t.autocast_dtype = trace.autocast_dtype
    return t


class TraceResults:
    def __init__(self, prologue, computation, epilogue, interpreter_log=None):
        self.prologue_trace = prologue
        self.computation_trace = computation
        self.epilogue_trace = epilogue
        self.interpreter_log = interpreter_log


class Timer:
    def __init__(self):
        self.start = time.perf_counter_ns()

    def ms(self) -> float:
        return (time.perf_counter_ns() - self.start) / 1e6
