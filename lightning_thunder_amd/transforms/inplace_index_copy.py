"""In-place ``index_copy`` for static caches (parity: reference ``thunder/recipes/hf_transformers.py``
``InplaceIndexCopyTransform`` :26-97).

Functionalization turns ``cache.index_copy_(dim, pos, new)`` into a functional
``t = index_copy(cache, dim, pos, new)`` plus a write-back ``copy_(t, cache)`` at the end of the
program.  For a KV cache that copies the *whole* cache twice per layer per token.  When the cache
is not read between the update and the write-back (other than through ``t``) and nothing is
differentiated through it, the pair is replaced by one in-place ``index_copy_`` whose output
aliases the cache: O(tokens) instead of O(cache) HBM traffic per step.
"""
from __future__ import annotations

import torch

from ..core import prims
from ..core.prims import PrimIDs, OpTags
from ..core.proxies import TensorProxy
from ..core.symbol import Symbol, register_symbol
from ..core.trace import TraceCtx, from_trace, TraceProvenance
from ..core.transform_common import Transform


def _meta(buf, dim, index, src):
    return TensorProxy(like=buf)


index_copy_inplace = Symbol("index_copy_inplace", _meta, id="lta.index_copy_inplace", is_prim=True,
                            tags=(OpTags.DONT_DCE, OpTags.IN_PLACE))
index_copy_inplace.written_args = (0,)
register_symbol(index_copy_inplace)


def _impl(buf, dim, index, src):
    return buf.index_copy_(dim, index, src)


def _register():
    from ..executors import torchex

    op = torchex.ex.register_operator("index_copy_inplace", like=index_copy_inplace, fn=_impl)
    torchex.ex.register_implementation(index_copy_inplace, op)


_register()

_INDEX_COPY_IDS = {"auto.torch.TensorBase.index_copy", "auto.torch.index_copy", "torch.index_copy"}


def _is_index_copy(b) -> bool:
    return b.sym.id in _INDEX_COPY_IDS or b.sym.name in ("index_copy",)


def inplace_index_copy(trace: TraceCtx) -> TraceCtx:
    """Rewrites ``t = index_copy(buf, ...)`` + ``copy_(t, buf)`` into ``t = index_copy_inplace(buf, ...)``."""
    bsyms = list(trace.bound_symbols)
    arg_names = {a.name for a in trace.args if isinstance(a, TensorProxy)}
    consumers: dict[str, list[int]] = {}
    for i, b in enumerate(bsyms):
        for a in b.flat_proxy_args:
            consumers.setdefault(a.name, []).append(i)
    drop: set[int] = set()
    replace: dict[int, object] = {}
    for i, b in enumerate(bsyms):
        if not _is_index_copy(b) or len(b.args) < 4 and not b.kwargs:
            continue
        args = list(b.args) + [b.kwargs.get(k) for k in ("dim", "index", "source") if k in b.kwargs]
        if len(args) != 4:
            continue
        buf, dim, index, src = args
        out = b.output
        if not (isinstance(buf, TensorProxy) and isinstance(out, TensorProxy) and buf.name in arg_names):
            continue
        if buf.requires_grad:
            continue
        # the write-back of the functional result into the buffer
        wb = [j for j in consumers.get(out.name, []) if bsyms[j].sym.id == PrimIDs.COPY_
              and bsyms[j].args[0] is not None and bsyms[j].args[0].name == out.name
              and isinstance(bsyms[j].args[1], TensorProxy) and bsyms[j].args[1].name == buf.name]
        if len(wb) != 1:
            continue
        j = wb[0]
        # no other reader of the old buffer value after the update
        others = [k for k in consumers.get(buf.name, []) if k > i and k != j]
        if others:
            continue
        replace[i] = index_copy_inplace.bind(buf, dim, index, src, output=out)
        drop.add(j)
        # any consumer of the copy_ output is re-pointed at the in-place result
        cj = bsyms[j].output
        if isinstance(cj, TensorProxy) and consumers.get(cj.name):
            drop.discard(j)
            replace.pop(i)
    if not replace:
        return trace
    new = from_trace(trace)
    new.bound_symbols = [replace.get(i, b) for i, b in enumerate(bsyms) if i not in drop]
    new.set_provenance(TraceProvenance(f"In-place index_copy ({len(replace)} cache updates)"))
    return new


class InplaceIndexCopyTransform(Transform):
    """``transform_traces_pre_prologue`` hook running :func:`inplace_index_copy` (use for programs
    that are not differentiated; ``jit`` already applies the pass to every no-grad program)."""

    def transform_traces_pre_prologue(self, prologue_trace, computation_trace, epilogue_trace, **kwargs):
        return prologue_trace, inplace_index_copy(computation_trace), epilogue_trace
