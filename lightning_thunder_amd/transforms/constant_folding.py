"""ConstantFolding: evaluate, at compile time, every computation whose inputs are all
compile-time constants (tensor factories with literal arguments and ops on them), and replace
the sub-graph by the precomputed tensor.

Reference parity: ``thunder/transforms/constant_folding.py:105-266``.  Folded tensors are held
by the trace (a zero-argument ``folded_constant_N()`` call per value), so a step no longer
launches the kernels that rebuild e.g. causal masks, position ids or RoPE tables.
"""
from __future__ import annotations

import itertools

import torch

from ..core import prims
from ..core.prims import PrimIDs, OpTags
from ..core.proxies import TensorProxy, Proxy
from ..core.pytree import tree_flatten, tree_map
from ..core.symbol import Symbol, BoundSymbol
from ..core.trace import from_trace, TraceProvenance
from ..core.transform_common import Transform

_SOURCES = {PrimIDs.FULL, PrimIDs.IOTA, PrimIDs.TENSOR_FROM_SEQUENCE}
_SOURCE_NAMES = {"full", "zeros", "ones", "arange", "tensor", "eye", "linspace", "full_like", "zeros_like", "ones_like",
                 "tril", "triu"}
_counter = itertools.count()


def _evaluate(b: BoundSymbol, env: dict):
    from ..executors.torchex import ex as tex

    def get(x):
        return env[x.name] if isinstance(x, Proxy) and x.name in env else x

    args = tree_map(get, b.args)
    kwargs = tree_map(get, b.kwargs)
    impl = tex.implmap.get(b.sym.id)
    if impl is not None and impl.symbol is not None:
        fn = getattr(impl.symbol, "impl_fn", None)
        tfn = getattr(b, "torch_fn", None)
        if getattr(impl.symbol, "replay_torch", False) and tfn is not None:
            fn = tfn
        out = fn(*args, **kwargs)
    elif b.subsymbols:
        for s in b.subsymbols:
            _evaluate(s, env)
        return
    else:
        raise RuntimeError(f"cannot fold {b.sym.name}")
    for o, v in zip(tree_flatten(b.output)[0], tree_flatten(out)[0]):
        if isinstance(o, Proxy):
            env[o.name] = v


def _is_source(b) -> bool:
    return b.sym.id in _SOURCES or b.sym.name in _SOURCE_NAMES


def _foldable(b) -> bool:
    tags = set(b.sym.tags or ())
    if OpTags.RANDOM_OP in tags or OpTags.DONT_DCE in tags or OpTags.IN_PLACE in tags:
        return False
    if b.sym.id in (PrimIDs.RETURN, PrimIDs.DEL) or (isinstance(b.sym.id, str) and b.sym.id.startswith("dist.")):
        return False
    outs = b.flat_proxy_outs
    return bool(outs) and all(isinstance(o, TensorProxy) for o in outs)


class ConstantFolding(Transform):
    def __init__(self, max_bytes: int = 1 << 30):
        self.max_bytes = max_bytes
        self.folded: dict[str, torch.Tensor] = {}

    def transform_traces_pre_prologue(self, prologue_trace, computation_trace, epilogue_trace, **kwargs):
        const: set[str] = set()
        env: dict = {}
        for b in computation_trace.bound_symbols:
            if not _foldable(b):
                continue
            targs = [a for a in b.flat_proxy_args]
            if _is_source(b) and not any(isinstance(a, TensorProxy) and a.name not in const for a in targs) and \
                    not any(isinstance(a, Proxy) and not isinstance(a, TensorProxy) for a in targs):
                pass
            elif not targs or any(a.name not in const for a in targs):
                continue
            try:
                _evaluate(b, env)
            except Exception:
                continue
            const |= {o.name for o in b.flat_proxy_outs}
        if not const:
            return prologue_trace, computation_trace, epilogue_trace
        # values still needed by non-constant computations (or returned) become folded constants
        needed = set()
        for b in computation_trace.bound_symbols:
            if all(o.name in const for o in b.flat_proxy_outs) and b.flat_proxy_outs:
                continue
            needed |= {a.name for a in b.flat_proxy_args if a.name in const}
        new = from_trace(computation_trace)
        new.bound_symbols = []
        new.scopes = [new.bound_symbols]
        emitted = set()
        for b in computation_trace.bound_symbols:
            outs = b.flat_proxy_outs
            if outs and all(o.name in const for o in outs):
                for o in outs:
                    if o.name in needed and o.name not in emitted:
                        t = env[o.name]
                        if t.numel() * t.element_size() > self.max_bytes:
                            raise RuntimeError("constant too large to fold")
                        nm = f"folded_constant_{next(_counter)}"
                        self.folded[o.name] = t
                        from ..executors.pythonex import ex as pyex

                        sym = Symbol(nm, meta=None, is_prim=True, executor=pyex)
                        new.bound_symbols.append(BoundSymbol(sym, args=(), kwargs={}, output=o,
                                                             _call_ctx={nm: (lambda t=t: t)}))
                        emitted.add(o.name)
                continue
            new.bound_symbols.append(b)
        new.set_provenance(TraceProvenance(f"Constant folding ({len(emitted)} tensors)"))
        return prologue_trace, new, epilogue_trace
