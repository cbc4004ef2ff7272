"""Common trace passes and the Transform ABC (parity: reference ``thunder/core/transform_common.py``:
``dce`` :145, ``cse`` :292, ``Transform`` :376-424, ``_inplace_copy_sanity_check`` :68-109).
"""
from __future__ import annotations

import time
from abc import ABC
from typing import Any, TYPE_CHECKING

from .proxies import Proxy, TensorProxy
from .prims import PrimIDs, OpTags
from .symbol import BoundSymbol, has_tags
from .trace import TraceCtx, from_trace, TraceProvenance
from .pytree import tree_flatten


def _has_side_effects(bsym: BoundSymbol) -> bool:
    if OpTags.DONT_DCE in bsym.sym.tags or OpTags.IN_PLACE in bsym.sym.tags:
        return True
    if bsym.sym.id == PrimIDs.RETURN:
        return True
    tags = getattr(bsym.sym, "tags", ())
    if "dont_dce" in tags:
        return True
    # distributed collectives that are waited on elsewhere are kept via their outputs
    return False


def dce(trace: TraceCtx, *, keep_inputs: bool = False) -> TraceCtx:
    """Removes bound symbols whose outputs are unused (respects DONT_DCE / in-place tags)."""
    start = time.perf_counter_ns()
    needed: set[str] = set()
    kept: list[BoundSymbol] = []
    for bsym in reversed(trace.bound_symbols):
        outs = bsym.flat_proxy_outs
        if _has_side_effects(bsym) or any(o.name in needed for o in outs) or (not outs and bsym.sym.id in (PrimIDs.DEL, PrimIDs.COMMENT)):
            kept.append(bsym)
            for a in bsym.flat_proxy_args:
                needed.add(a.name)
            # subsymbols may reference extra proxies (not needed for liveness)
    kept.reverse()
    new = from_trace(trace)
    new.bound_symbols = kept
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance(f"Dead Code Elimination (took {(time.perf_counter_ns() - start) // 1000000} milliseconds)"))
    return new


def cse(trace: TraceCtx) -> TraceCtx:
    """Common subexpression elimination over side-effect-free bound symbols."""
    from .symbol import from_bsym_swap_proxies

    start = time.perf_counter_ns()
    seen: dict[Any, BoundSymbol] = {}
    swap: dict[str, Proxy] = {}
    out: list[BoundSymbol] = []
    for bsym in trace.bound_symbols:
        b = from_bsym_swap_proxies(bsym, swap, skip_output=True)
        if _has_side_effects(b) or OpTags.RANDOM_OP in b.sym.tags or b.sym.id == PrimIDs.DEL:
            out.append(b)
            continue
        try:
            key = b.rhs()
            hash(key)
        except TypeError:
            out.append(b)
            continue
        prev = seen.get(key)
        if prev is not None and len(prev.flat_outs) == len(b.flat_outs):
            for o_new, o_old in zip(b.flat_outs, prev.flat_outs):
                if isinstance(o_new, Proxy) and isinstance(o_old, Proxy):
                    swap[o_new.name] = o_old
            continue
        seen[key] = b
        out.append(b)
    new = from_trace(trace)
    new.bound_symbols = out
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance(f"Common Subexpression Elimination (took {(time.perf_counter_ns() - start) // 1000000} milliseconds)"))
    return new


def _inplace_copy_sanity_check(trace: TraceCtx) -> None:
    """A fusion must not read a ``copy_`` destination after writing it (aliasing hazard)."""
    for bsym in trace.bound_symbols:
        if not bsym.sym.is_fusion:
            continue
        written: set[str] = set()
        for sub in bsym.subsymbols:
            for a in sub.flat_proxy_args:
                if a.name in written:
                    raise NotImplementedError(
                        f"{bsym.sym.name} reads {a.name} after a copy_ into it; this in-place pattern is unsupported"
                    )
            if sub.sym.id == PrimIDs.COPY_:
                written.add(sub.args[1].name)


class Transform(ABC):
    """Transform hooks (reference :376-424)."""

    def transform_traces_pre_prologue(self, prologue_trace, computation_trace, epilogue_trace, **kwargs):
        return prologue_trace, computation_trace, epilogue_trace

    def transform_module(self, model) -> None:
        pass

    def transform_state_dict_for_submodule(self, model, submodule_name: str, state_dict: dict) -> dict:
        return state_dict

    def reverse_transform_state_dict_for_submodule(self, model, submodule_name: str, state_dict: dict) -> dict:
        return state_dict

    def transform_trace_post_optimization(self, computation_trace, **kwargs):
        return computation_trace

    def __repr__(self) -> str:
        return f"{self.__class__.__module__}.{self.__class__.__name__}()"


def order_proxies(bsyms) -> dict[str, int]:
    order: dict[str, int] = {}
    i = 0
    for b in bsyms:
        for p in b.flat_proxy_args + b.flat_proxy_outs:
            if p.name not in order:
                order[p.name] = i
                i += 1
    return order
