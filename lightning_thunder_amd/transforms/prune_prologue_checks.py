"""Prologue pruning transforms (reference ``thunder/transforms/prune_prologue_checks.py`` and
``extraction_only_prologue_transform.py``).

``PrunePrologueChecks`` drops the metadata guards on module parameters/buffers (they cannot
change between calls without going through the ThunderModule); ``ExtractionOnlyPrologueTransform``
drops every guard, leaving a prologue that only extracts inputs (the caller guarantees that the
cache entry matches)."""
from __future__ import annotations

from ..core import prims
from ..core.trace import from_trace, TraceProvenance
from ..core.transform_common import Transform

_CHECKS = {prims.PrimIDs.CHECK_TENSOR_SHAPE_AND_METADATA, prims.PrimIDs.CHECK_NUMBER_TYPE_AND_VALUE,
           prims.PrimIDs.CHECK_LEN, prims.PrimIDs.CHECK_NONE, prims.PrimIDs.CHECK_STRING_VALUE,
           prims.PrimIDs.CHECK_LITERAL_LIKE}


def _state_proxies(pro) -> set[str]:
    """Names of the values unpacked from the module-state argument (params, buffers, attrs)."""
    names: set[str] = set()
    if len(pro.args) < 2:
        return names
    st = pro.args[1]
    for b in pro.bound_symbols:
        if b.sym.id == prims.PrimIDs.UNPACK_SEQUENCE and b.args and getattr(b.args[0], "name", None) == st.name:
            names |= {o.name for o in b.flat_proxy_outs}
    return names


class PrunePrologueChecks(Transform):
    def __init__(self, prune_all_checks: bool = False):
        self.prune_all_checks = prune_all_checks

    def transform_traces_pre_prologue(self, prologue_trace, computation_trace, epilogue_trace, **kwargs):
        state = _state_proxies(prologue_trace)
        keep = []
        for b in prologue_trace.bound_symbols:
            if b.sym.id in _CHECKS:
                if self.prune_all_checks:
                    continue
                if b.args and getattr(b.args[0], "name", None) in state:
                    continue
            keep.append(b)
        new = from_trace(prologue_trace)
        new.bound_symbols = keep
        new.scopes = [new.bound_symbols]
        new.set_provenance(TraceProvenance("Prune prologue checks"))
        return new, computation_trace, epilogue_trace


class ExtractionOnlyPrologueTransform(PrunePrologueChecks):
    def __init__(self):
        super().__init__(prune_all_checks=True)
