"""Bound-symbol DAG utilities: build the def-use DAG of a trace, topologically sort it with a
pluggable selector, and rewrite traces by visiting or splicing bound symbols.

Parity: reference ``thunder/core/transforms.py`` ``Node`` / ``bsym_list_to_dag`` :103-205,
``TOPOSORT_ORDER`` / ``toposort_bsym_dag`` :207-276, ``insert_inplace`` / ``replace_inplace``
:278-357, ``VISIT_TYPE`` / ``visitor_transform`` :359-428.  Scheduling passes (``sort_waits``,
the FSDP all-gather window, the fusion partitioner's dataflow order) are selectors over this one
toposort instead of private re-implementations.

Beyond plain data dependencies the DAG keeps the program order of side-effecting bound symbols
(in-place ops and ``del``): reordering two of them could change what a later reader observes.
"""
from __future__ import annotations

import heapq
from enum import Enum, auto
from typing import Callable, Sequence

from .prims import OpTags, PrimIDs
from .proxies import Proxy
from .pytree import tree_flatten
from .trace import TraceCtx, TraceProvenance, from_trace, tracectx


class Node:
    """One bound symbol in the DAG; ``index`` is its position in the source list."""

    __slots__ = ("bsym", "index", "parents", "children", "pending")

    def __init__(self, bsym, index: int):
        self.bsym = bsym
        self.index = index
        self.parents: list[Node] = []
        self.children: list[Node] = []
        self.pending = 0  # parents not yet emitted during a toposort

    def __repr__(self) -> str:
        return f"Node({self.index}: {self.bsym.sym.name})"

    def __lt__(self, other: "Node") -> bool:
        return self.index < other.index


def _proxy_names(x) -> list[str]:
    return [p.name for p in tree_flatten(x)[0] if isinstance(p, Proxy)]


def _has_effect(b) -> bool:
    return OpTags.IN_PLACE in b.sym.tags or b.sym.id == PrimIDs.DEL


def bsym_list_to_dag(bsyms: Sequence, *, keep_effect_order: bool = True) -> tuple[list[Node], list[Node], list[Node]]:
    """(roots, leaves, all nodes).  An edge p -> c means c reads a value p produced (or, with
    ``keep_effect_order``, both have side effects and p comes first)."""
    nodes = [Node(b, i) for i, b in enumerate(bsyms)]
    producer: dict[str, Node] = {}
    last_effect: Node | None = None
    for n in nodes:
        b = n.bsym
        seen: set[int] = set()

        def link(p: Node):
            if p is not n and p.index not in seen:
                seen.add(p.index)
                p.children.append(n)
                n.parents.append(p)

        for name in _proxy_names((b.args, b.kwargs)):
            p = producer.get(name)
            if p is not None:
                link(p)
        if keep_effect_order and _has_effect(b):
            if last_effect is not None:
                link(last_effect)
            last_effect = n
        for name in _proxy_names(b.output):
            producer.setdefault(name, n)
    roots = [n for n in nodes if not n.parents]
    leaves = [n for n in nodes if not n.children]
    return roots, leaves, nodes


class TOPOSORT_ORDER(Enum):
    TOP_DOWN = auto()  # from the inputs: a node is eligible once all its parents are emitted
    BOTTOM_UP = auto()  # from the outputs: eligible once all its children are emitted


def _default_selector(eligible: list[Node]) -> int:
    """Program order: the eligible node that came first in the source list."""
    best = 0
    for i, n in enumerate(eligible):
        if n.index < eligible[best].index:
            best = i
    return best


def toposort_bsym_dag(nodes: Sequence[Node], order: TOPOSORT_ORDER = TOPOSORT_ORDER.TOP_DOWN,
                      selector: Callable[[list[Node]], int] | None = None) -> list:
    """Topologically sorted bound symbols.  ``selector(eligible)`` returns the position of the node
    to emit next (it may inspect ``node.pending`` of other nodes); the default keeps program order.
    BOTTOM_UP sorts from the leaves and returns the result in execution order."""
    top = order is TOPOSORT_ORDER.TOP_DOWN
    for n in nodes:
        n.pending = len(n.parents) if top else len(n.children)
    eligible = [n for n in nodes if n.pending == 0]
    out: list[Node] = []
    while eligible:
        if selector is None and top:
            eligible.sort()
            k = 0
        else:
            k = (selector or _default_selector)(eligible)
        n = eligible.pop(k)
        out.append(n)
        for m in (n.children if top else n.parents):
            m.pending -= 1
            if m.pending == 0:
                eligible.append(m)
    if len(out) != len(nodes):
        raise RuntimeError("toposort_bsym_dag: the bound symbols form a cycle")
    if not top:
        out.reverse()
    return [n.bsym for n in out]


def toposort_with_priority(bsyms: Sequence, priority: Callable) -> list:
    """Convenience: TOP_DOWN toposort emitting the eligible node with the smallest
    ``priority(node)`` (ties by program order), in O(n log n) with a heap."""
    _, _, nodes = bsym_list_to_dag(bsyms)
    for n in nodes:
        n.pending = len(n.parents)
    heap = [(priority(n), n.index, n) for n in nodes if n.pending == 0]
    heapq.heapify(heap)
    out = []
    while heap:
        _, _, n = heapq.heappop(heap)
        out.append(n.bsym)
        for m in n.children:
            m.pending -= 1
            if m.pending == 0:
                heapq.heappush(heap, (priority(m), m.index, m))
    if len(out) != len(nodes):
        raise RuntimeError("toposort_with_priority: cycle")
    return out


def _record(trace: TraceCtx, fn: Callable, *args, **kwargs) -> tuple[list, object]:
    scope: list = []
    with tracectx(trace):
        trace.push_scope(scope)
        try:
            res = fn(*args, **kwargs)
        finally:
            trace.pop_scope()
    return scope, res


def insert_inplace(trace: TraceCtx, idx: int, fn: Callable, *args, **kwargs):
    """Trace ``fn(*args, **kwargs)`` and splice its bound symbols into ``trace`` before position
    ``idx`` (mutates the trace).  Returns ``fn``'s result (proxies)."""
    scope, res = _record(trace, fn, *args, **kwargs)
    trace.bound_symbols[idx:idx] = scope
    return res


def replace_inplace(trace: TraceCtx, idx: int, fn: Callable, *args, **kwargs):
    """Replace the bound symbol at ``idx`` by the bound symbols ``fn(*args, **kwargs)`` records."""
    scope, res = _record(trace, fn, *args, **kwargs)
    trace.bound_symbols[idx:idx + 1] = scope
    return res


class VISIT_TYPE(Enum):
    NO_OP = auto()  # keep the visited bound symbol; nothing may have been recorded
    INSERT_BEFORE = auto()  # recorded bound symbols go before the visited one
    INSERT_AFTER = auto()  # ... after it
    REPLACE = auto()  # recorded bound symbols replace it


def visitor_transform(trace_from: TraceCtx, visit: Callable, *, provenance: str | None = None) -> TraceCtx:
    """New trace built by calling ``visit(bsym)`` for every bound symbol inside a recording context:
    whatever the visitor traces is placed according to the ``VISIT_TYPE`` it returns."""
    trc = from_trace(trace_from)
    out: list = []
    trc.bound_symbols = out
    trc.scopes = [out]
    for b in trace_from.bound_symbols:
        scope, vt = _record(trc, visit, b)
        if vt is None or vt is VISIT_TYPE.NO_OP:
            if scope:
                raise RuntimeError(f"visitor recorded {len(scope)} bound symbols for {b.sym.name} but returned NO_OP")
            out.append(b)
        elif vt is VISIT_TYPE.INSERT_BEFORE:
            out.extend(scope)
            out.append(b)
        elif vt is VISIT_TYPE.INSERT_AFTER:
            out.append(b)
            out.extend(scope)
        elif vt is VISIT_TYPE.REPLACE:
            out.extend(scope)
        else:
            raise ValueError(f"visitor returned {vt!r}")
    trc.bound_symbols = out
    trc.scopes = [out]
    if provenance is not None:
        trc.set_provenance(TraceProvenance(provenance))
    return trc
