"""Per-bound-symbol forward/backward construction (parity: reference ``thunder/core/vjp_utils.py`` —
``make_aug_forward_and_backward`` :29-193, ``get_saved_for_backward_tensors`` :195,
``set_saved_for_backward_tensors`` :235).

``make_aug_forward_and_backward(bsym)`` differentiates a single bound symbol with the framework's
autodiff (executor grad transforms first, then VJP rules, then decomposition) and returns two
callables that re-emit the augmented forward (``-> (output, saved)``) and the backward
(``(*saved, *cotangents) -> grads``) into whatever trace is current.  Results are cached per
symbol and argument metadata, which is what executors that fuse whole fwd/bwd regions use.
"""
from __future__ import annotations

from typing import Callable, Sequence

from .proxies import Proxy, TensorProxy, NumberProxy
from .pytree import tree_flatten, tree_unflatten, tree_map
from .symbol import BoundSymbol
from .trace import TraceCtx, tracectx
from .prims import PrimIDs

_cache: dict = {}


def _meta_key(x):
    if isinstance(x, TensorProxy):
        return ("T", tuple(x.shape), x.dtype, str(x.device), bool(x.requires_grad))
    if isinstance(x, NumberProxy):
        return ("N", type(x.value), x.value)
    if isinstance(x, (list, tuple)):
        return (type(x).__name__,) + tuple(_meta_key(v) for v in x)
    try:
        hash(x)
        return x
    except TypeError:
        return ("id", id(x))


def make_aug_forward_and_backward(bsym: BoundSymbol, *, executors=()) -> tuple[Callable, Callable]:
    from . import prims
    from ..transforms.autodiff import forward_and_backward_from_trace
    from .trace_interpreter import interpret_trace

    key = (bsym.sym.id, _meta_key(bsym.args), _meta_key(tuple(sorted(bsym.kwargs.items()))), tuple(e.name for e in executors))
    hit = _cache.get(key)
    if hit is None:
        t = TraceCtx(None)
        t.fn_name = "vjp_region"
        with tracectx(t):
            flat, spec = tree_flatten((bsym.args, bsym.kwargs))
            fresh = [x.replace() if isinstance(x, TensorProxy) else x for x in flat]
            a, k = tree_unflatten(fresh, spec)
            t.args = [x for x in fresh if isinstance(x, Proxy)]
            out = bsym.sym(*a, **k)
            prims.python_return(out)
        fb = forward_and_backward_from_trace(t, executors=executors)
        hit = (fb, [i for i, x in enumerate(flat) if isinstance(x, Proxy)])
        _cache[key] = hit
    fb, proxy_pos = hit

    def fw_fn(*args, **kwargs):
        flat, _ = tree_flatten((args, kwargs))
        out = interpret_trace(fb.forward_trace, *[flat[i] for i in proxy_pos])
        result, saved_t, saved_o = out
        return result, tuple(saved_t) + tuple(saved_o)

    def bw_fn(*saved_and_cotangents):
        return interpret_trace(fb.backward_trace, *saved_and_cotangents)

    return fw_fn, bw_fn


def get_saved_for_backward_tensors(trace: TraceCtx) -> tuple:
    """The saved-for-backward tensors returned by an augmented forward trace."""
    ret = trace.bound_symbols[-1]
    if ret.sym.id != PrimIDs.RETURN:
        raise ValueError("expected an augmented forward trace ending in a return")
    return tuple(ret.args[0][1])


def set_saved_for_backward_tensors(trace: TraceCtx, saved_tensors: Sequence[TensorProxy]) -> None:
    """Replaces the saved-for-backward tensors of an augmented forward trace (in place)."""
    ret = trace.bound_symbols[-1]
    if ret.sym.id != PrimIDs.RETURN:
        raise ValueError("expected an augmented forward trace ending in a return")
    fw_out, _, other = ret.args[0]
    trace.bound_symbols[-1] = ret.from_bsym(args=((fw_out, tuple(saved_tensors), other),))
    trace.scopes = [trace.bound_symbols]


def clear_cache() -> None:
    _cache.clear()
