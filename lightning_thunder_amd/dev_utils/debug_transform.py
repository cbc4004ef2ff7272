"""DebugTransform: user callbacks before/after every executed bound symbol
(reference ``thunder/dev_utils/debug_transform.py``; ``debug_execution_trace``)."""
from __future__ import annotations

from typing import Callable

from ..core.trace import from_trace, TraceProvenance
from ..core.transform_common import Transform
from ._insert import host_call, SKIP


class DebugTransform(Transform):
    def __init__(self, pre_callback: Callable | None = None, post_callback: Callable | None = None):
        self.pre_callback = pre_callback
        self.post_callback = post_callback

    def transform_trace_post_optimization(self, trace, **kwargs):
        new = from_trace(trace)
        out = []
        for b in trace.bound_symbols:
            if b.sym.name in SKIP:
                out.append(b)
                continue
            if self.pre_callback is not None:
                pre = self.pre_callback
                out.append(host_call("debug_pre", lambda *a, _b=b, _f=pre: _f(_b, *a), args=b.flat_proxy_args))
            out.append(b)
            if self.post_callback is not None:
                post = self.post_callback
                outs = b.flat_proxy_outs
                out.append(host_call("debug_post", lambda *o, _b=b, _f=post: _f(_b, *o), args=outs))
        new.bound_symbols = out
        new.scopes = [new.bound_symbols]
        new.set_provenance(TraceProvenance("Debug transform"))
        return new


def debug_execution_trace(cfn, pre_callback: Callable | None = None, post_callback: Callable | None = None):
    """Re-jits ``cfn`` with a :class:`DebugTransform` (callbacks get ``(bsym, *tensors)``)."""
    from ..core.transforms import add_transform

    return add_transform(cfn, transform=DebugTransform(pre_callback, post_callback))
