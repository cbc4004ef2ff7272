"""Profiling ranges around every bound symbol of the execution traces (reference:
``thunder/dev_utils/nvtx_profile_transform.py:41-76``).

On ROCm ``torch.cuda.nvtx`` is backed by roctx, so these are roctx ranges: ``rocprofv3
--marker-trace`` shows each range (labelled with the symbol name and, with
``include_shapes=True``, its tensor arguments' shapes / dtypes) next to the HIP kernels the
symbol launched.  ``NvtxProfileTransform`` keeps the reference's name.
"""
from __future__ import annotations

import torch

from ..core.proxies import TensorProxy
from ..core.trace import from_trace, TraceProvenance
from ..core.transform_common import Transform
from ._insert import host_call, SKIP


def _range_push(name):
    if torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)


def _range_pop():
    if torch.cuda.is_available():
        torch.cuda.nvtx.range_pop()


def _label(b, include_shapes: bool) -> str:
    label = str(b.sym.name)
    if include_shapes:
        shapes = [f"{a.dtype}{list(a.shape)}".replace("torch.", "") for a in b.flat_proxy_args
                  if isinstance(a, TensorProxy)]
        if shapes:
            label += "(" + ", ".join(shapes) + ")"
    return label


class RoctxProfileTransform(Transform):
    """Wraps every executed bound symbol in a roctx range."""

    def __init__(self, include_shapes: bool = False):
        self.include_shapes = include_shapes

    def transform_trace_post_optimization(self, trace, **kwargs):
        new = from_trace(trace)
        out = []
        for b in trace.bound_symbols:
            if b.sym.name in SKIP:
                out.append(b)
                continue
            label = _label(b, self.include_shapes)
            out.append(host_call("roctx_push", lambda _l=label: _range_push(_l)))
            out.append(b)
            out.append(host_call("roctx_pop", _range_pop))
        new.bound_symbols = out
        new.scopes = [new.bound_symbols]
        new.set_provenance(TraceProvenance("roctx ranges"))
        return new


NvtxProfileTransform = RoctxProfileTransform

__all__ = ["NvtxProfileTransform", "RoctxProfileTransform"]
