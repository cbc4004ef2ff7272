"""Kernel-level numerics checking (SURVEY §5.2 "MI355X plan": a debug mode that synchronizes after
each fused kernel and compares against the torch executor — numerical bisection).

The reference has no GPU-side checker; its closest tools are ``check_traces`` and nvFuser
optimization fuel (``thunder/dev_utils/check_trace.py``, ``thunder/extend/__init__.py:206-226``).
:class:`NumericsCheckTransform` wraps every executor-claimed bound symbol of the execution trace:

* ``torch.cuda.synchronize()`` after the call, so an asynchronous fault is attributed to the kernel
  that caused it (``DebugOptions(sync_after_each_kernel=True)`` enables just this part);
* non-finite values in floating outputs are reported (unless the inputs already had them);
* hipfuse regions are re-evaluated with the torch implementations of their prims and compared
  (``atol``/``rtol``), which finds a miscompiled fusion without reading any generated code.

Findings go to ``transform.findings``; ``raise_on_error=True`` raises at the first one.
"""
from __future__ import annotations

import torch

from ..core.pytree import tree_flatten
from ..core.trace import from_trace, TraceProvenance
from ..core.transform_common import Transform
from ._insert import SKIP


class NumericsMismatch(RuntimeError):
    pass


def _floats(xs):
    return [x for x in xs if isinstance(x, torch.Tensor) and x.is_floating_point()]


class NumericsCheckTransform(Transform):
    def __init__(self, *, compare_fusions: bool = True, check_finite: bool = True, sync: bool = True,
                 atol: float = 2e-2, rtol: float = 2e-2, raise_on_error: bool = False):
        self.compare_fusions = compare_fusions
        self.check_finite = check_finite
        self.sync = sync
        self.atol = atol
        self.rtol = rtol
        self.raise_on_error = raise_on_error
        self.findings: list[str] = []
        self.checked = 0

    def _report(self, msg: str):
        self.findings.append(msg)
        if self.raise_on_error:
            raise NumericsMismatch(msg)

    def _wrap(self, name: str, fn):
        from ..executors.hipfuse import HipFusion

        def wrapped(*args, **kwargs):
            out = fn(*args, **kwargs)
            if self.sync and torch.cuda.is_available():
                torch.cuda.synchronize()
            self.checked += 1
            flat_out = tree_flatten(out)[0]
            if self.check_finite:
                ins_finite = all(bool(torch.isfinite(t).all()) for t in _floats(tree_flatten((args, kwargs))[0]))
                for i, o in enumerate(_floats(flat_out)):
                    if ins_finite and not bool(torch.isfinite(o).all()):
                        self._report(f"{name}: output {i} has non-finite values (inputs were finite)")
            if self.compare_fusions and isinstance(fn, HipFusion):
                cpu_args = [a.detach().cpu() if isinstance(a, torch.Tensor) else a for a in args]
                ref = fn._run_reference(cpu_args)
                for i, (o, r) in enumerate(zip(_floats(flat_out), _floats(tree_flatten(ref)[0]))):
                    o32, r32 = o.detach().float().cpu(), r.float()
                    if not torch.allclose(o32, r32, atol=self.atol, rtol=self.rtol, equal_nan=True):
                        err = (o32 - r32).abs().max().item()
                        self._report(f"{name}: output {i} differs from the torch reference (max abs err {err:.3e})")
            return out

        return wrapped

    def transform_trace_post_optimization(self, trace, **kwargs):
        new = from_trace(trace)
        out = []
        for b in trace.bound_symbols:
            ctx = b._call_ctx
            if ctx:
                name, fn = next(iter(ctx.items()))
            else:
                name, fn = b.sym.name, getattr(b.sym, "impl_fn", None)
            if b.sym.name in SKIP or fn is None or (b.sym.executor is None and not ctx):
                out.append(b)
                continue
            ident = "checked_" + "".join(c if c.isalnum() else "_" for c in str(b.sym.name))
            out.append(b.from_bsym(_call_ctx={ident: self._wrap(str(name), fn)}))
        new.bound_symbols = out
        new.scopes = [new.bound_symbols]
        new.set_provenance(TraceProvenance("Numerics check (sync + finiteness + fusion-vs-torch)"))
        return new


class SyncAfterEachKernelTransform(NumericsCheckTransform):
    """Only the synchronization part (``DebugOptions(sync_after_each_kernel=True)``)."""

    def __init__(self):
        super().__init__(compare_fusions=False, check_finite=False, sync=True)
