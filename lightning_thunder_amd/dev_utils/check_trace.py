"""Structural validation of traces (reference ``thunder/dev_utils/check_trace.py``).

Enabled per compilation with ``DebugOptions(check_traces=True)``: every trace produced while
compiling is checked for (1) use-before-definition and redefinition of proxy names, (2) bound
symbols whose subsymbols do not produce the parent's outputs, (3) a return that is not last.
"""
from __future__ import annotations

from ..core.prims import PrimIDs
from ..core.proxies import Proxy, TensorProxy

CHECK_VERSION = 1


class TraceCheckError(RuntimeError):
    pass


def check_subsymbols(parent) -> None:
    if not parent.subsymbols or parent.sym.is_fusion:
        return
    produced = set()
    for s in parent.subsymbols:
        produced |= {o.name for o in s.flat_proxy_outs}
        check_subsymbols(s)
    ins = {a.name for a in parent.flat_proxy_args}
    for o in parent.flat_proxy_outs:
        if o.name not in produced and o.name not in ins:
            raise TraceCheckError(f"{parent.sym.name}: output {o.name} is not produced by its subsymbols")


def check_trace(trace, *, version: int = CHECK_VERSION) -> None:
    defined: set[str] = set()
    for a in trace.args:
        for p in (a if isinstance(a, (list, tuple)) else [a]):
            if isinstance(p, Proxy):
                defined.add(p.name)
    for k, v in (trace.kwargs or {}).items():
        if isinstance(v, Proxy):
            defined.add(v.name)
    deleted: set[str] = set()
    n = len(trace.bound_symbols)
    for i, b in enumerate(trace.bound_symbols):
        if b.sym.id == PrimIDs.RETURN and i != n - 1:
            raise TraceCheckError(f"return is bound symbol {i} of {n}")
        if b.sym.id == PrimIDs.DEL:
            for p in b.flat_proxy_args:
                deleted.add(p.name)
            continue
        for a in b.flat_proxy_args:
            if a.name not in defined and not a.name.startswith("_"):
                raise TraceCheckError(f"{b.sym.name} (bsym {i}) uses {a.name} before it is defined")
            if a.name in deleted:
                raise TraceCheckError(f"{b.sym.name} (bsym {i}) uses {a.name} after it was deleted")
        if b.sym.id == PrimIDs.RETURN:
            continue
        for o in b.flat_proxy_outs:
            if o.name in defined and o.name not in {a.name for a in b.flat_proxy_args}:
                if not (b.sym.name.startswith("unpack") or b.sym.name == "__getitem__"):
                    raise TraceCheckError(f"{b.sym.name} (bsym {i}) redefines {o.name}")
            defined.add(o.name)
            if isinstance(o, TensorProxy) and any((not isinstance(s, int)) or s < 0 for s in o.shape
                                                  if isinstance(s, int) or not hasattr(s, "name")):
                raise TraceCheckError(f"{o.name} has an invalid shape {o.shape}")
        check_subsymbols(b)


class CheckedListOfTraces(list):
    def append(self, trace):
        check_trace(trace)
        super().append(trace)

    def extend(self, traces):
        for t in traces:
            check_trace(t)
        super().extend(traces)
