"""Re-executing traces (parity: reference ``thunder/core/trace_interpreter.py`` —
``interpret_trace`` :23-60, ``interpret_trace_to_trace`` :63-131, ``TraceSubstitutionProcessor``
:134-277).

* :func:`interpret_trace` evaluates a trace's bound symbols on concrete values (or on proxies of
  the *current* trace, which re-records them there), optionally through a ``symbol_mapper`` that
  swaps a bound symbol's callable (e.g. the executor implementation, or a decomposition).
* :func:`interpret_trace_to_trace` does the same into a fresh trace and returns it.
* :class:`TraceSubstitutionProcessor` is the work-list rewriter: subclasses override
  :meth:`process_bsym` and call :meth:`add_processed_bsyms` / :meth:`add_unprocessed_bsyms` /
  :meth:`set_result`; outputs of replaced bound symbols are swapped onto the new proxies.
"""
from __future__ import annotations

from collections import deque
from typing import Any, Callable

from .proxies import Proxy
from .pytree import tree_flatten, tree_map
from .symbol import BoundSymbol, from_bsym_swap_proxies
from .trace import TraceCtx, from_trace, tracectx, TraceProvenance
from .prims import PrimIDs


def _read(env: dict, x):
    if isinstance(x, Proxy):
        try:
            return env[x.name]
        except KeyError:
            raise KeyError(f"interpret_trace: {x.name} is used before it is defined") from None
    return x


def _write(env: dict, target, value) -> None:
    if isinstance(target, Proxy):
        env[target.name] = value
        return
    if isinstance(target, (tuple, list)):
        vals = value if isinstance(value, (tuple, list)) else tuple(value)
        for t, v in zip(target, vals):
            _write(env, t, v)
    elif isinstance(target, dict):
        for k, t in target.items():
            _write(env, t, value[k])


def interpret_trace(trace: TraceCtx, *args, symbol_mapper: Callable | None = None, with_env: bool = False, **kwargs):
    """Evaluates ``trace`` on ``args``; ``symbol_mapper(bsym)`` returns the callable to use (or ``None``
    to run the bound symbol's own symbol)."""
    from .trace import get_tracectx

    if get_tracectx() is None and symbol_mapper is None and not with_env:
        # concrete values: run the trace the way the runtime does (claimed by the default executors)
        from ..executors.passes import transform_for_execution
        from ..extend import get_default_executors

        return transform_for_execution(trace, list(get_default_executors()))[-1].python_callable()(*args, **kwargs)
    env: dict[str, Any] = {}
    flat_params, _ = tree_flatten((trace.args, trace.kwargs))
    flat_vals, _ = tree_flatten((args, kwargs))
    for p, v in zip(flat_params, flat_vals):
        if isinstance(p, Proxy):
            env[p.name] = v
    result = None
    for bsym in trace.bound_symbols:
        sid = bsym.sym.id
        if sid in (PrimIDs.DEL, PrimIDs.COMMENT):
            continue
        a = tree_map(lambda x: _read(env, x), bsym.args)
        k = tree_map(lambda x: _read(env, x), bsym.kwargs)
        if sid == PrimIDs.RETURN:
            result = a[0] if len(a) == 1 else a
            break
        fn = symbol_mapper(bsym) if symbol_mapper is not None else None
        if fn is None:
            fn = bsym.sym
        out = fn(*a, **k)
        _write(env, bsym.output, out)
    return (env, result) if with_env else result


def interpret_trace_to_trace(trace: TraceCtx, *args, symbol_mapper: Callable | None = None, **kwargs) -> TraceCtx:
    """Re-records ``trace`` (through ``symbol_mapper``) into a new trace with fresh input proxies."""
    from .proxies import TensorProxy

    new = from_trace(trace)
    new.bound_symbols = []
    new.scopes = [new.bound_symbols]
    new.names = set()
    with tracectx(new):
        def fresh(p):
            return p.replace(name=p.name) if isinstance(p, TensorProxy) else p

        pargs = tree_map(fresh, tuple(trace.args))
        pkw = tree_map(fresh, dict(trace.kwargs))
        new.args, new.kwargs = list(pargs), pkw
        out = interpret_trace(trace, *pargs, symbol_mapper=symbol_mapper, **pkw)
        from . import prims

        prims.python_return(out)
    new.set_provenance(TraceProvenance("interpret_trace_to_trace"))
    return new


class TraceSubstitutionProcessor:
    """Work-list trace rewriter (reference ``TraceSubstitutionProcessor``)."""

    NULL = object()

    def __init__(self, trace: TraceCtx, *args, **kwargs):
        self.trace = trace
        self.new_trace = from_trace(trace)
        self.new_trace.bound_symbols = []
        self.new_trace.scopes = [self.new_trace.bound_symbols]
        self.new_trace.names = set(trace.names)
        self.swap_map: dict[str, Proxy] = {}
        self.have_processed_args = False
        self._pending: deque = deque()
        self._current: BoundSymbol | None = None
        self._result = self.NULL

    # --- API for process_bsym --------------------------------------------------------------------
    def add_processed_bsyms(self, bsyms: list[BoundSymbol]) -> None:
        self.new_trace.bound_symbols.extend(bsyms)

    def add_unprocessed_bsyms(self, bsyms: list[BoundSymbol]) -> None:
        self._pending.extendleft(reversed(list(bsyms)))

    def add_to_swap_map(self, old, new) -> None:
        if isinstance(old, Proxy) and isinstance(new, Proxy) and old.name != new.name:
            self.swap_map[old.name] = new

    def set_result(self, result) -> None:
        self._result = result

    def add_bsyms_from_function(self, fn: Callable, *args, **kwargs):
        """Traces ``fn`` into the new trace (as processed bound symbols) and returns its result."""
        scope: list = []
        with tracectx(self.new_trace):
            self.new_trace.push_scope(scope)
            try:
                res = fn(*args, **kwargs)
            finally:
                self.new_trace.pop_scope()
        self.add_processed_bsyms(scope)
        return res

    def process_bsym(self, bsym: BoundSymbol) -> None:  # override
        self.add_processed_bsyms([bsym])
        self.set_result(bsym.output)

    # --- driver ----------------------------------------------------------------------------
    def __call__(self) -> tuple[TraceCtx, list]:
        self._pending = deque(self.trace.bound_symbols)
        while self._pending:
            bsym = self._pending.popleft()
            bsym = from_bsym_swap_proxies(bsym, self.swap_map, skip_output=True) if self.swap_map else bsym
            self._current = bsym
            self._result = self.NULL
            self.process_bsym(bsym)
            if self._result is not self.NULL:
                outs, _ = tree_flatten(bsym.output)
                news, _ = tree_flatten(self._result)
                for o, n in zip(outs, news):
                    self.add_to_swap_map(o, n)
        self.new_trace.bound_symbols = [
            from_bsym_swap_proxies(b, self.swap_map, skip_output=True) if self.swap_map else b
            for b in self.new_trace.bound_symbols
        ]
        self.new_trace.scopes = [self.new_trace.bound_symbols]
        return self.new_trace, list(self.new_trace.bound_symbols)
