"""Communication scheduling (parity: reference ``thunder/distributed/utils.py:15-298``: ``sort_waits``,
``sort_communication_ops``, ``limit_in_flight_allgathers``).

``sort_waits`` reorders a trace (respecting data dependencies) so that collectives are
issued as early as possible and their ``wait`` s as late as possible — RCCL on its own
stream then overlaps with compute.  ``limit_in_flight_allgathers`` bounds how many
FSDP all-gathers are outstanding (memory vs overlap; with 288 GB of HBM the default is
unbounded).
"""
from __future__ import annotations

from ..core.prims import PrimIDs
from ..core.proxies import Proxy
from ..core.symbol import BoundSymbol
from ..core.trace import TraceCtx, from_trace, TraceProvenance


def _is_collective(b: BoundSymbol) -> bool:
    n = b.sym.name
    return any(x in n for x in ("all_gather", "all_reduce", "reduce_scatter", "broadcast")) and "wait" not in n


def _is_wait(b: BoundSymbol) -> bool:
    return b.sym.name.endswith("wait")


def sort_waits(trace: TraceCtx) -> TraceCtx:
    """List scheduling: among ready bound symbols prefer collectives, then regular ops, waits last."""
    bsyms = list(trace.bound_symbols)
    if not any(_is_wait(b) for b in bsyms):
        return trace
    ret = bsyms[-1] if bsyms and bsyms[-1].sym.id == PrimIDs.RETURN else None
    body = bsyms[:-1] if ret is not None else bsyms
    producers: dict[str, int] = {}
    for i, b in enumerate(body):
        for o in b.flat_proxy_outs:
            producers[o.name] = i
    deps = []
    users: list[list[int]] = [[] for _ in body]
    for i, b in enumerate(body):
        d = set()
        for a in b.flat_proxy_args:
            j = producers.get(a.name)
            if j is not None and j != i:
                d.add(j)
        # keep side-effecting ops (in-place copies, deletes) in original relative order
        deps.append(d)
        for j in d:
            users[j].append(i)
    # side effects: keep relative order among DONT_DCE / IN_PLACE ops
    from ..core.prims import OpTags

    last_effect = None
    for i, b in enumerate(body):
        if OpTags.IN_PLACE in b.sym.tags or b.sym.id == PrimIDs.DEL:
            if last_effect is not None:
                deps[i].add(last_effect)
                users[last_effect].append(i)
            last_effect = i
    indeg = [len(d) for d in deps]
    import heapq

    def prio(i):
        b = body[i]
        if _is_collective(b):
            return (0, i)
        if _is_wait(b):
            return (2, i)
        return (1, i)

    ready = [prio(i) for i in range(len(body)) if indeg[i] == 0]
    heapq.heapify(ready)
    order = []
    while ready:
        # waits only when nothing else is ready
        p, i = heapq.heappop(ready)
        order.append(i)
        for u in users[i]:
            indeg[u] -= 1
            if indeg[u] == 0:
                heapq.heappush(ready, prio(u))
    if len(order) != len(body):  # cycle guard (should not happen)
        return trace
    new = from_trace(trace)
    new.bound_symbols = [body[i] for i in order] + ([ret] if ret is not None else [])
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance("Sort waits (collectives early, waits late)"))
    return new


def maybe_sort_waits(trace: TraceCtx) -> TraceCtx:
    if any(_is_wait(b) for b in trace.bound_symbols):
        return sort_waits(trace)
    return trace


def limit_in_flight_allgathers(trace: TraceCtx, max_in_flight: int = 4) -> TraceCtx:
    """Reorders so at most ``max_in_flight`` all-gathers are outstanding (their waits pulled earlier)."""
    bsyms = list(trace.bound_symbols)
    out = []
    inflight: list[BoundSymbol] = []
    waits_by_future = {}
    for b in bsyms:
        if _is_wait(b):
            waits_by_future[b.args[0].name] = b
    emitted_waits = set()
    for b in bsyms:
        if _is_wait(b) and id(b) in emitted_waits:
            continue
        if _is_collective(b) and "all_gather" in b.sym.name and len(inflight) >= max_in_flight:
            oldest = inflight.pop(0)
            w = waits_by_future.get(oldest.output.name) if isinstance(oldest.output, Proxy) else None
            if w is not None and id(w) not in emitted_waits:
                out.append(w)
                emitted_waits.add(id(w))
        out.append(b)
        if _is_wait(b):
            emitted_waits.add(id(b))
            inflight = [c for c in inflight if not (isinstance(c.output, Proxy) and c.output.name == b.args[0].name)]
        elif _is_collective(b) and "all_gather" in b.sym.name:
            inflight.append(b)
    new = from_trace(trace)
    new.bound_symbols = out
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance(f"Limit in-flight all-gathers ({max_in_flight})"))
    return new
