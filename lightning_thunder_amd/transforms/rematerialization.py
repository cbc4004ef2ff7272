"""Activation rematerialisation between the forward and backward traces (parity: reference
``thunder/core/rematerialization.py`` — ``find_cut`` :239-330, ``rematerialize_forward_and_backward``
:537-620 — which min-cuts between adjacent nvFuser regions).

Here the cut is taken over the whole saved-for-backward frontier right after autodiff, before
claiming, so the recomputed ops join the backward's hipfuse kernels:

* every tensor ``t`` gets an edge ``t_in -> t_out`` whose capacity is the number of bytes kept
  alive if ``t`` is saved (trace inputs cost ~nothing: the caller keeps them alive anyway);
* tensors produced by ops that are not cheap to recompute (GEMMs, attention, reductions,
  RNG-state reads, executor kernels) hang off the source;
* a *recomputable* bound symbol (its decomposition is only elementwise / cast / broadcast /
  reshape prims) links each input's ``_out`` node to its outputs' ``_in`` nodes with infinite
  capacity;
* every currently-saved tensor links to the sink.

The minimum s-t cut is the cheapest set of tensors to save; everything between the cut and the
old saved set is recomputed at the top of the backward.
"""
from __future__ import annotations

import math

from ..core import dtypes
from ..core.prims import PrimIDs, OpTags
from ..core.proxies import Proxy, TensorProxy
from ..core.symbol import BoundSymbol
from ..core.trace import from_trace, TraceProvenance
from ..core.transform_common import dce

_RECOMPUTABLE: set | None = None


def _recomputable_prims() -> set:
    global _RECOMPUTABLE
    if _RECOMPUTABLE is None:
        from ..executors.hipfuse_codegen import ELEMENTWISE, VIEWS

        _RECOMPUTABLE = set(ELEMENTWISE) | set(VIEWS) | {PrimIDs.TRANSPOSE, PrimIDs.FULL, PrimIDs.UNIFORM_PHILOX}
    return _RECOMPUTABLE


def _leaves(b: BoundSymbol):
    if not b.subsymbols:
        yield b
        return
    for s in b.subsymbols:
        yield from _leaves(s)


def is_recomputable(b: BoundSymbol) -> bool:
    if OpTags.DONT_DCE in b.sym.tags or OpTags.RANDOM_OP in b.sym.tags or OpTags.IN_PLACE in b.sym.tags:
        return False
    if getattr(b.sym, "executor", None) is not None and not b.subsymbols:
        return False
    outs = b.flat_proxy_outs
    if not outs or not all(isinstance(o, TensorProxy) for o in outs):
        return False
    allowed = _recomputable_prims()
    for leaf in _leaves(b):
        if leaf.sym.id not in allowed:
            return False
    return True


def _nbytes(t: TensorProxy) -> int:
    return math.prod(t.shape) * dtypes.itemsize(t.dtype)


def rematerialize_forward_and_backward(fb):
    """Returns ``fb`` with a (never larger) saved set and the recomputation moved to the backward."""
    import networkx as nx

    fw, bw = fb.forward_trace, fb.backward_trace
    ret = fw.bound_symbols[-1]
    assert ret.sym.id == PrimIDs.RETURN
    fw_out, saved_t, saved_o = ret.args[0]
    saved_t = list(saved_t)
    if not saved_t:
        return fb

    producer: dict[str, BoundSymbol] = {}
    order: dict[int, int] = {}
    for i, b in enumerate(fw.bound_symbols):
        order[id(b)] = i
        for o in b.flat_proxy_outs:
            producer[o.name] = b
    fw_inputs = {a.name for a in fw.args if isinstance(a, Proxy)}

    # backward closure of the saved set through recomputable producers
    closure: dict[str, TensorProxy] = {}
    stack = list(saved_t)
    while stack:
        t = stack.pop()
        if t.name in closure:
            continue
        closure[t.name] = t
        b = producer.get(t.name)
        if b is not None and t.name not in fw_inputs and is_recomputable(b):
            for a in b.flat_proxy_args:
                if isinstance(a, TensorProxy):
                    stack.append(a)
    if all(not (producer.get(n) is not None and is_recomputable(producer[n])) for n in closure):
        return fb

    g = nx.DiGraph()
    g.add_node("SOURCE")  # saved values recomputable from nothing (e.g. full) leave SOURCE edgeless
    inf = float("inf")
    for n, t in closure.items():
        cost = 1 if n in fw_inputs else max(1, _nbytes(t))
        g.add_edge(n + "_in", n + "_out", capacity=cost)
        b = producer.get(n)
        if n in fw_inputs or b is None or not is_recomputable(b):
            g.add_edge("SOURCE", n + "_in", capacity=inf)
        else:
            for a in b.flat_proxy_args:
                if isinstance(a, TensorProxy):
                    g.add_edge(a.name + "_out", n + "_in", capacity=inf)
    for t in saved_t:
        g.add_edge(t.name + "_out", "SINK", capacity=inf)
    cut_value, (reach, _) = nx.minimum_cut(g, "SOURCE", "SINK")
    old_cost = sum((1 if t.name in fw_inputs else max(1, _nbytes(t))) for t in {t.name: t for t in saved_t}.values())
    if cut_value >= old_cost:
        return fb
    new_saved = [closure[n] for n in closure if n + "_in" in reach and n + "_out" not in reach]
    new_names = {t.name for t in new_saved}

    # bound symbols to replay in the backward (forward order)
    needed: dict[int, BoundSymbol] = {}
    seen: set[str] = set()

    def need(t: TensorProxy):
        if t.name in new_names or t.name in seen:
            return
        seen.add(t.name)
        b = producer[t.name]
        needed[id(b)] = b
        for a in b.flat_proxy_args:
            if isinstance(a, TensorProxy):
                need(a)

    for t in saved_t:
        need(t)
    replay = sorted(needed.values(), key=lambda b: order[id(b)])

    # non-tensor values the replayed ops read must also be saved
    extra_other = []
    have = {p.name for p in saved_o} | new_names
    made = set()
    for b in replay:
        for a in b.flat_proxy_args:
            if not isinstance(a, TensorProxy) and a.name not in have and a.name not in made:
                extra_other.append(a)
                have.add(a.name)
        for o in b.flat_proxy_outs:
            made.add(o.name)

    new_fw = from_trace(fw)
    new_fw.bound_symbols = list(fw.bound_symbols[:-1]) + [
        ret.from_bsym(args=((fw_out, tuple(new_saved), tuple(saved_o) + tuple(extra_other)),))
    ]
    new_fw.scopes = [new_fw.bound_symbols]
    new_fw.args = fw.args
    new_fw = dce(new_fw)
    new_fw.set_provenance(TraceProvenance("Rematerialization (forward)"))

    n_ct = len(bw.args) - len(saved_t) - len(saved_o)
    cotangents = list(bw.args[len(saved_t) + len(saved_o):]) if n_ct > 0 else []
    new_bw = from_trace(bw)
    new_bw.bound_symbols = [b.from_bsym() for b in replay] + list(bw.bound_symbols)
    new_bw.scopes = [new_bw.bound_symbols]
    new_bw.args = list(new_saved) + list(saved_o) + list(extra_other) + cotangents
    new_bw = dce(new_bw)
    new_bw.set_provenance(TraceProvenance(f"Rematerialization (backward): saved {old_cost} -> {int(cut_value)} bytes"))

    fb.forward_trace = new_fw
    fb.backward_trace = new_bw
    fb.saved_tensors = new_saved
    fb.saved_other = list(saved_o) + extra_other
    return fb
