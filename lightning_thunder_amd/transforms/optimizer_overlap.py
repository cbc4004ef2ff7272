"""Optimizer step overlapped with the backward pass (one GPU).

The fused AdamW (``optim.AdamW``, ``ops/csrc/adamw.hip``) streams p, g, m, v at HBM speed, so on one
GPU it is a serial tail after the backward (~16 ms of a Llama-2-7B step).  Nothing in the reference
corresponds: its benchmark runs ``torch.optim.AdamW(fused=True)`` after ``loss.backward()``
(``thunder/benchmarks/benchmark_litgpt.py:275-283``).  Here the update of each parameter is issued
inside the compiled backward as soon as it is safe:

* :func:`insert_grad_ready_hooks` (a pass over the execution backward trace, before the
  last-use ``del`` pass) finds, for every parameter gradient the backward returns, the point after
  which the gradient is final AND the parameter (or any view of it) is no longer read by the
  backward; gradients becoming ready there are grouped into buckets of ``bucket_bytes`` and a host
  call ``optim_grad_ready(positions, *grads)`` is inserted after the bucket's last ready point.
* At run time the call hands the bucket to the optimizer attached with :func:`overlap_with_backward`:
  it records an event on the compute stream and launches the lean (register-capped) AdamW kernel on a
  side stream, whose waves fit next to a running gemm4 workgroup (adamw.hip).  The parameter's
  gradient is then NOT returned to autograd (``p.grad`` stays ``None``).
* ``optimizer.step()`` joins the side stream into the current one and updates whatever was not
  handled during the backward; ``zero_grad`` is unchanged.

Contract: every backward is followed by ``optimizer.step()`` (no gradient accumulation across
backwards and no global-norm gradient clipping between them — both need all gradients before any
update).  Hooks are compiled in only for single-process runs without hipGraph capture.
"""
from __future__ import annotations

import threading
from contextlib import contextmanager

from ..core.prims import PrimIDs, OpTags
from ..core.proxies import TensorProxy
from ..core.trace import from_trace, TraceProvenance

_tls = threading.local()

from ..examine.memory_calculation import is_view_bsym as _is_view  # noqa: E402

# ops that may hand back their input tensor itself at run time (no fresh allocation): torch returns
# ``a`` from contiguous() of a contiguous tensor, from detach()/alias() (new view of the same
# storage), and from to()/type_as()/float()... when nothing changes; in-place ops return ``self``
_MAY_RETURN_INPUT = {"contiguous", "detach", "alias", "shallow_copy", "to", "type_as", "type", "convert_element_type",
                     "float", "double", "half", "bfloat16", "int", "long", "short", "bool", "byte", "char", "cpu",
                     "cuda", "requires_grad_", "data", "clone_if_needed", "view_as_real", "view_as_complex",
                     "resolve_conj", "resolve_neg", "conj", "real", "lift_fresh", "copy_with_setitem", "copy_"}


def may_alias_bsym(b) -> bool:
    """True when an output of ``b`` may share storage with its first tensor input at run time: views,
    the identity-returning conversions above (same dtype / shape out as in), in-place ops (trailing
    ``_``), and composite bound symbols containing any of these."""
    if _is_view(b):
        return True
    nm = str(getattr(b.sym, "name", ""))
    base = nm[:-5] if nm.endswith("_prim") else nm
    base = base.rsplit(".", 1)[-1]
    ins = [a for a in b.flat_proxy_args if isinstance(a, TensorProxy)]
    outs = [o for o in b.flat_proxy_outs if isinstance(o, TensorProxy)]
    if not ins or not outs:
        return False
    if base.endswith("_") and not base.endswith("__"):
        return True
    if base in _MAY_RETURN_INPUT:
        a = ins[0]
        return any(o.dtype == a.dtype and tuple(o.shape) == tuple(a.shape) for o in outs)
    return any(may_alias_bsym(s) for s in (getattr(b, "subsymbols", None) or ()))


def view_aliases(trace, alias_of: dict | None = None) -> dict:
    """name -> root name for every value of ``trace`` that may share storage with another value (views
    and ops that may return their input: :func:`may_alias_bsym`)."""
    alias_of = dict(alias_of or {})
    for b in trace.bound_symbols:
        if not may_alias_bsym(b):
            continue
        srcs = [a.name for a in b.flat_proxy_args if isinstance(a, TensorProxy)]
        if not srcs:
            continue
        root = alias_of.get(srcs[0], srcs[0])
        for o in b.flat_proxy_outs:
            alias_of[o.name] = root
    return alias_of


def insert_grad_ready_hooks(bw, param_names: list, bucket_bytes: int = 128 << 20, fw=None):
    """Returns ``bw`` with ``optim_grad_ready`` host calls; ``param_names[k]`` is the name of the
    forward input whose gradient is output ``k`` of the backward (None: not a candidate).  ``fw``
    (the forward trace) lets views of parameters saved for the backward count as parameter reads."""
    from ..dev_utils._insert import host_call

    bsyms = list(bw.bound_symbols)
    ret_i = next((i for i in range(len(bsyms) - 1, -1, -1) if bsyms[i].sym.id == PrimIDs.RETURN), None)
    if ret_i is None:
        return bw
    outs = bsyms[ret_i].args[0]
    if not isinstance(outs, (tuple, list)):
        return bw
    producer: dict = {}
    last_use: dict = {}
    for i, b in enumerate(bsyms[:ret_i]):
        for a in b.flat_proxy_args:
            last_use[a.name] = i
        for o in b.flat_proxy_outs:
            producer.setdefault(o.name, i)
    # names that may alias each parameter (views of views included, forward-made views too)
    alias_of = view_aliases(bw, view_aliases(fw) if fw is not None else None)
    uses_by_root: dict = {}
    for name, i in last_use.items():
        root = alias_of.get(name, name)
        uses_by_root[root] = max(uses_by_root.get(root, -1), i)
    ready: dict = {}  # bsym index -> [output positions]
    seen_grads: set = set()
    for k, g in enumerate(outs):
        if k >= len(param_names) or param_names[k] is None or not isinstance(g, TensorProxy):
            continue
        if g.name in seen_grads:  # the same proxy returned twice: leave it to the post-backward step
            continue
        seen_grads.add(g.name)
        r = max(producer.get(g.name, -1), uses_by_root.get(param_names[k], -1),
                max((i for n, i in last_use.items() if alias_of.get(n) == g.name), default=-1))
        ready.setdefault(r, []).append(k)
    if not ready:
        return bw

    out = []
    pending: list = []
    pending_bytes = 0

    def flush():
        nonlocal pending, pending_bytes
        if pending:
            ks = tuple(pending)
            out.append(host_call("optim_grad_ready", _grad_ready, args=(ks, *[outs[k] for k in ks])))
        pending, pending_bytes = [], 0

    for k in ready.get(-1, []):
        pending.append(k)
        pending_bytes += _nbytes(outs[k])
    for i, b in enumerate(bsyms):
        if i == ret_i:
            flush()
        out.append(b)
        if i in ready and i != ret_i:
            for k in ready[i]:
                pending.append(k)
                pending_bytes += _nbytes(outs[k])
            if pending_bytes >= bucket_bytes:
                flush()
    new = from_trace(bw)
    new.bound_symbols = out
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance("Optimizer step overlapped with the backward (grad-ready hooks)"))
    return new


def _nbytes(t) -> int:
    n = 1
    for s in t.shape:
        n *= int(s)
    return n * t.dtype.itemsize


def _grad_ready(positions, *grads):
    st = getattr(_tls, "ctx", None)
    if st is None:
        return None
    opt, params_by_pos, handled = st
    ps, gs = [], []
    for k, g in zip(positions, grads):
        p = params_by_pos.get(k)
        if p is None or g is None:
            continue
        ps.append(p)
        gs.append(g)
        handled.add(k)
    if ps:
        opt.overlapped_update(ps, gs)
    return None


@contextmanager
def active(opt, params_by_pos: dict, handled: set):
    """Makes ``opt`` the target of the grad-ready hooks of the backward run inside the block."""
    prev = getattr(_tls, "ctx", None)
    _tls.ctx = (opt, params_by_pos, handled)
    try:
        yield
    finally:
        _tls.ctx = prev


def overlap_with_backward(jitted, optimizer, bucket_mb: int = 128) -> None:
    """Issue ``optimizer``'s update of each parameter inside ``jitted``'s backward (see the module
    docstring).  Call before the first forward (already compiled entries are dropped)."""
    from .. import compile_data, compile_stats

    if not hasattr(optimizer, "overlapped_update"):
        raise TypeError("the optimizer must implement overlapped_update (lightning_thunder_amd.optim.AdamW does)")
    cd = compile_data(jitted)
    cd.overlap_optimizer = optimizer
    cd.overlap_bucket_bytes = int(bucket_mb) << 20
    cs = compile_stats(jitted)
    if cs is not None and getattr(cs, "interpreter_cache", None):
        cs.interpreter_cache.clear()
