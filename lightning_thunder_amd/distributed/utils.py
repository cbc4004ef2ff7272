"""Communication scheduling (parity: reference ``thunder/distributed/utils.py:15-298``: ``sort_waits``,
``sort_communication_ops``, ``limit_in_flight_allgathers``).

``sort_waits`` reorders a trace (respecting data dependencies) so that collectives are
issued as early as possible and their ``wait`` s as late as possible — RCCL on its own
stream then overlaps with compute.  ``schedule_allgathers`` / ``limit_in_flight_allgathers``
then re-place the parameter all-gathers in a sliding window (ZeRO-3: bounded gathered-parameter
memory; ZeRO-2 keeps every gathered block for the backward anyway, so there the window is off
and all gathers are issued at the start — 288 GB of HBM holds them).
"""
from __future__ import annotations

from ..core.prims import PrimIDs
from ..core.proxies import Proxy
from ..core.symbol import BoundSymbol
from ..core.trace import TraceCtx, from_trace, TraceProvenance


# ops that always hand back a freshly allocated tensor (never their input or a view of it): the only
# producers whose output a tensor-parallel all-reduce may reduce in place (skip_clone)
_FRESH_PRODUCERS = frozenset({
    "linear", "matmul", "mm", "bmm", "embedding", "add", "sub", "mul", "div", "true_divide", "neg", "silu", "gelu",
    "relu", "tanh", "sigmoid", "exp", "sum", "where", "scaled_dot_product_attention", "cat", "rms_norm",
    "layer_norm", "softmax", "baddbmm", "addmm",
})


def allocates_fresh(b: BoundSymbol) -> bool:
    """True when ``b`` is known to allocate its outputs (allowlist, so an unknown op — a future
    conversion or identity op that may return its input — is never reduced in place)."""
    nm = str(getattr(b.sym, "name", ""))
    base = nm[:-5] if nm.endswith("_prim") else nm
    base = base.rsplit(".", 1)[-1]
    return base in _FRESH_PRODUCERS


def lower_tp_syncs(trace: TraceCtx) -> TraceCtx:
    """Tensor-parallel syncs -> explicit async collectives + ``wait`` (reference: the TP prims issue
    ``all_reduce(..., do_async=True, skip_clone=True).wait()`` / ``all_gather(..., True).wait()``,
    thunder/distributed/prims.py:433-551), so that :func:`sort_waits` can move each wait past
    independent work — e.g. a column-parallel linear's input-gradient all-reduce runs under the same
    layer's weight-gradient GEMM.

    * all-reduce syncs (row-parallel output, vocab-parallel embedding output, and the column-parallel
      input gradient, which the VJP expresses as the same sync) -> ``all_reduce(a, SUM, group, True,
      skip_clone)`` + ``wait``; the all-reduce runs in place (no clone) when ``a`` is a fresh tensor
      nothing else reads: not a trace input or output, read only by this sync, and made by an op on
      the :func:`allocates_fresh` allowlist (GEMMs, embedding, elementwise math);
    * last-dim all-gather syncs (column-parallel output) -> ``all_gather(a, group, True, -1)`` + ``wait``;
    * the input-side syncs (identity / local slice) stay as they are.
    Run on the traces right after autodiff, before the executors claim them."""
    from .prims import (synchronize_tensor_parallel_output as tp_out, TPLayerType, all_reduce, all_gather, wait,
                        DistributedReduceOps)
    from ..core.trace import tracectx

    bsyms = list(trace.bound_symbols)
    if not any(b.sym is tp_out for b in bsyms):
        return trace
    readers: dict[str, int] = {}
    producer: dict[str, BoundSymbol] = {}
    for b in bsyms:
        for a in b.flat_proxy_args:
            readers[a.name] = readers.get(a.name, 0) + 1
        for o in b.flat_proxy_outs:
            producer.setdefault(o.name, b)
    from ..core.pytree import tree_flatten

    inputs = {a.name for a in tree_flatten((trace.args, trace.kwargs))[0] if isinstance(a, Proxy)}
    new = from_trace(trace)
    out: list = []
    n = 0
    with tracectx(new):
        for b in bsyms:
            if b.sym is not tp_out:
                out.append(b)
                continue
            a, group, kind = b.args[0], b.args[1], b.args[2]
            if kind in (TPLayerType.ROW_LINEAR, TPLayerType.COLUMN_EMBED):
                prod = producer.get(a.name)
                fresh = (a.name not in inputs and readers.get(a.name, 0) == 1 and prod is not None
                         and allocates_fresh(prod))
                fut = all_reduce.bind(a, DistributedReduceOps.SUM, group, True, fresh,
                                      output=all_reduce.meta(a, DistributedReduceOps.SUM, group, True, fresh))
            else:
                dim = len(a.shape) - 1
                fut = all_gather.bind(a, group, True, dim, output=all_gather.meta(a, group, True, dim))
            out.append(fut)
            out.append(wait.bind(fut.output, output=b.output))
            n += 1
    new.bound_symbols = out
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance(f"Lower tensor-parallel syncs ({n} -> async collective + wait)"))
    return new


def _is_collective(b: BoundSymbol) -> bool:
    n = b.sym.name
    return any(x in n for x in ("all_gather", "all_reduce", "reduce_scatter", "broadcast")) and "wait" not in n


def _is_wait(b: BoundSymbol) -> bool:
    return b.sym.name.endswith("wait")


def hoist_collective_inputs(bsyms: list) -> list:
    """Issue every collective as soon as its inputs CAN exist: in the stretch of program since the
    previous collective, the ops the collective (transitively) depends on move before it, the
    independent ops after it.  Autodiff emits a linear's dgrad and wgrad together, so a
    tensor-parallel input-gradient all-reduce (fed by the dgrads of fc_1 and fc_2) would otherwise
    be issued only after both wgrads, with nothing left to overlap; hoisted, the wgrad GEMMs run
    while it is in flight (list scheduling alone keeps program order among ready ops)."""
    coll = [i for i, b in enumerate(bsyms) if _is_collective(b)]
    if not coll:
        return bsyms
    out: list = []
    prev = 0
    for c in coll:
        window = bsyms[prev:c]
        made = {}
        for k, b in enumerate(window):
            for o in b.flat_proxy_outs:
                made.setdefault(o.name, k)
        need = {a.name for a in bsyms[c].flat_proxy_args}
        anc = set()
        for k in range(len(window) - 1, -1, -1):
            b = window[k]
            if any(o.name in need for o in b.flat_proxy_outs):
                anc.add(k)
                need.update(a.name for a in b.flat_proxy_args)
        out.extend(window[k] for k in range(len(window)) if k in anc)
        out.append(bsyms[c])
        out.extend(window[k] for k in range(len(window)) if k not in anc)
        prev = c + 1
    out.extend(bsyms[prev:])
    return out


def sort_waits(trace: TraceCtx) -> TraceCtx:
    """List scheduling over the bound-symbol DAG (:func:`core.dag.toposort_bsym_dag`): among the
    eligible bound symbols prefer collectives, then regular ops (both in program order), waits
    last; among ready waits, the one that completes the inputs of some consumer ("useful") goes
    first, so the compute stream is not made to wait for collectives whose results are needed only
    later (e.g. the backward's ZeRO-3 re-gathers, consumed in reverse layer order)."""
    from ..core.dag import bsym_list_to_dag, toposort_bsym_dag

    bsyms = list(trace.bound_symbols)
    if not any(_is_wait(b) for b in bsyms):
        return trace
    ret = bsyms[-1] if bsyms and bsyms[-1].sym.id == PrimIDs.RETURN else None
    body = bsyms[:-1] if ret is not None else bsyms
    body = hoist_collective_inputs(body)
    _, _, nodes = bsym_list_to_dag(body)

    def rank(n) -> tuple:
        b = n.bsym
        if _is_collective(b):
            return (0, n.index)
        if not _is_wait(b):
            return (1, n.index)
        useful = any(c.pending == 1 for c in n.children)
        return (2 if useful else 3, n.index)

    def selector(eligible) -> int:
        return min(range(len(eligible)), key=lambda i: rank(eligible[i]))

    try:
        order = toposort_bsym_dag(nodes, selector=selector)
    except RuntimeError:  # cycle guard (should not happen)
        return trace
    new = from_trace(trace)
    new.bound_symbols = order + ([ret] if ret is not None else [])
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance("Sort waits (collectives early, waits late)"))
    return new


def maybe_sort_waits(trace: TraceCtx) -> TraceCtx:
    if any(_is_wait(b) for b in trace.bound_symbols):
        return sort_waits(trace)
    return trace


def _flat_futures(b: BoundSymbol) -> list[str]:
    from ..core.pytree import tree_flatten

    return [o.name for o in tree_flatten(b.output)[0] if isinstance(o, Proxy)]


def schedule_allgathers(trace: TraceCtx, prefetch: int = 2) -> TraceCtx:
    """Sliding-window placement of the (coalesced) parameter all-gathers (reference
    ``sort_communication_ops`` + ``limit_in_flight_allgathers``, thunder/distributed/utils.py:61-117,
    197-298).  Gathers are ordered by their first ``wait``; gather i is issued right after the last
    wait of gather i - ``prefetch`` (the first ``prefetch`` ones at the program start), so while block
    k computes, the gathers of blocks k+1 .. k+prefetch-1 are in flight and at most ``prefetch``
    gathered blocks are live: ZeRO-3 memory stays bounded without serializing RCCL behind compute.
    Every other op keeps its relative order."""
    bsyms = list(trace.bound_symbols)
    gathers = [b for b in bsyms if _is_collective(b) and "all_gather" in b.sym.name]
    if len(gathers) <= prefetch or prefetch < 1:
        return trace
    fut_owner: dict[str, int] = {}
    for gi, g in enumerate(gathers):
        for n in _flat_futures(g):
            fut_owner[n] = gi
    first_wait: dict[int, int] = {}
    last_wait: dict[int, int] = {}
    for pos, b in enumerate(bsyms):
        if _is_wait(b) and b.args and isinstance(b.args[0], Proxy) and b.args[0].name in fut_owner:
            gi = fut_owner[b.args[0].name]
            first_wait.setdefault(gi, pos)
            last_wait[gi] = pos
    if len(first_wait) != len(gathers):
        return trace  # a gather without waits (or a non-gather future): leave the program alone
    order = sorted(range(len(gathers)), key=lambda gi: first_wait[gi])
    gather_ids = {id(g) for g in gathers}
    after: dict[int, list] = {}  # position of a wait -> gathers to issue right after it
    before: dict[int, list] = {}  # position of a wait -> gathers to issue right before it
    head = []
    for k, gi in enumerate(order):
        if k < prefetch:
            head.append(gathers[gi])
            continue
        p = last_wait[order[k - prefetch]]
        if p < first_wait[gi]:
            after.setdefault(p, []).append(gathers[gi])
        else:
            # the earlier bucket stays in use past this one's first wait (e.g. the parameters outside
            # the transformer blocks: embedding at the start, LM head at the end): issue right before
            # the first wait instead, never after it
            before.setdefault(first_wait[gi], []).append(gathers[gi])
    # a gather must also come after whatever produces its inputs (normally trace inputs)
    out = []
    ret = bsyms[-1] if bsyms and bsyms[-1].sym.id == PrimIDs.RETURN else None
    produced_at: dict[str, int] = {}
    for pos, b in enumerate(bsyms):
        for o in b.flat_proxy_outs:
            produced_at.setdefault(o.name, pos)
    late_head = []
    for g in head:
        if any(a.name in produced_at for a in g.flat_proxy_args):
            late_head.append(g)
    head = [g for g in head if g not in late_head]
    out.extend(head)
    pending_late = list(late_head)
    for pos, b in enumerate(bsyms):
        if id(b) in gather_ids:
            continue
        if b is ret:
            break
        out.extend(before.get(pos, ()))
        out.append(b)
        if pending_late:
            ready = [g for g in pending_late
                     if all(produced_at.get(a.name, -1) <= pos for a in g.flat_proxy_args)]
            out.extend(ready)
            pending_late = [g for g in pending_late if g not in ready]
        out.extend(after.get(pos, ()))
    out.extend(pending_late)
    if ret is not None:
        out.append(ret)
    if len(out) != len(bsyms):
        return trace
    new = from_trace(trace)
    new.bound_symbols = out
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance(f"Schedule all-gathers (prefetch window {prefetch})"))
    return new


def limit_in_flight_allgathers(trace: TraceCtx, max_in_flight: int = 2) -> TraceCtx:
    """At most ``max_in_flight`` parameter all-gathers outstanding: ``schedule_allgathers`` with that
    window (reference name, thunder/distributed/utils.py:197-298)."""
    return schedule_allgathers(trace, max_in_flight)
