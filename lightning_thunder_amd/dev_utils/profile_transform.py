"""Profiling transforms (reference ``thunder/dev_utils/profile_transform.py`` and
``nvtx_profile_transform.py``).

* ``RoctxProfileTransform``: a roctx range (``torch.cuda.nvtx`` is roctx on ROCm) around every
  bound symbol of the execution traces — the ranges show up in ``rocprofv3 --marker-trace``
  next to the HIP kernels each symbol launched.
* ``ProfileTransform``: run ``torch.profiler`` over a window ``[start, end)`` of the execution
  trace (chosen by index or by regex on input names) for selected calls after warm-up, with a
  ``record_function`` per bound symbol.
"""
from __future__ import annotations

import re

import torch

from ..core.proxies import TensorProxy
from ..core.trace import from_trace, TraceProvenance
from ..core.transform_common import Transform
from ._insert import host_call, SKIP


from .nvtx_profile_transform import RoctxProfileTransform, NvtxProfileTransform, _range_push, _range_pop  # noqa: F401


class ProfileTransform(Transform):
    def __init__(self, *, warmup_runs: int = 3, number_runs: int = 1, start_idx: int = 0, end_idx: int | None = None,
                 input_match: str | None = None, backward: bool = False):
        self.warmup_runs = warmup_runs
        self.number_runs = number_runs
        self.start_idx = start_idx
        self.end_idx = end_idx
        self.input_match = input_match
        self.backward = backward
        self.run_counter = 0
        self.enabled = True
        self.active = False
        self.prof = None

    def start_profile(self):
        self.run_counter += 1
        self.active = self.enabled and self.warmup_runs < self.run_counter <= self.warmup_runs + self.number_runs
        if self.active:
            self.prof = torch.profiler.profile(record_shapes=True)
            self.prof.__enter__()

    def end_profile(self):
        if self.active:
            self.prof.__exit__(None, None, None)
            self.active = False

    def get_profile(self):
        return self.prof

    def _window(self, bsyms):
        if self.input_match is None:
            end = self.end_idx if self.end_idx is not None else len(bsyms)
            return self.start_idx, end
        hits = [i for i, b in enumerate(bsyms) for a in b.flat_proxy_args
                if isinstance(a, TensorProxy) and re.match(self.input_match, a.name)]
        s = hits[self.start_idx] if len(hits) > self.start_idx else 0
        e = hits[self.end_idx] if self.end_idx is not None and len(hits) > self.end_idx else len(bsyms)
        return s, e

    def transform_trace_post_optimization(self, trace, **kwargs):
        is_bw = trace.fn_name == "backward_fn" or bool(trace.unpack_list_arg)
        if is_bw != self.backward:
            return trace
        bsyms = trace.bound_symbols
        start, end = self._window(bsyms)
        out = []
        for i, b in enumerate(bsyms):
            if i == start:
                out.append(host_call("start_profiling", self.start_profile))
            if b.sym.name == "python_return" and start <= i <= end:
                out.append(host_call("end_profiling", self.end_profile))
            elif i == end:
                out.append(host_call("end_profiling", self.end_profile))
            if start <= i < end and b.sym.name not in SKIP:
                label = b.sym.name
                rec = {}

                def enter(_l=label, _r=rec):
                    if self.active:
                        _r["r"] = torch.profiler.record_function(_l)
                        _r["r"].__enter__()

                def leave(_r=rec):
                    r = _r.pop("r", None)
                    if r is not None:
                        r.__exit__(None, None, None)

                out.append(host_call("record_enter", enter))
                out.append(b)
                out.append(host_call("record_exit", leave))
            else:
                out.append(b)
        new = from_trace(trace)
        new.bound_symbols = out
        new.scopes = [new.bound_symbols]
        new.set_provenance(TraceProvenance("Profile transform"))
        return new
