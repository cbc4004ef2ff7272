"""``torch.autograd.Function`` subclasses inside compiled programs (parity: reference
``thunder/core/jit_ext.py:797`` ``_general_jit_torch_autograd_function_apply_lookaside`` and
``thunder/torch/__init__.py:6712`` ``autograd_function_apply``).

``MyFn.apply(*args)`` becomes one composite bound symbol per Function class whose decomposition is
the user's ``forward`` (so executors may claim/fuse what it does) and whose VJP is the user's
``backward``, traced into the backward program with the ``ctx`` the forward filled in.  Both the
old style (``forward(ctx, *args)``) and the new style (``forward(*args)`` + ``setup_context``) are
supported; ``ctx.save_for_backward`` / ``saved_tensors``, attributes on ``ctx``,
``needs_input_grad``, ``mark_non_differentiable`` and ``set_materialize_grads`` work as in eager.
"""
from __future__ import annotations

import torch

from ..core.proxies import TensorProxy
from ..core.pytree import tree_flatten
from ..core.symbol import Symbol, register_symbol

_symbols: dict[type, Symbol] = {}
_last_ctx: dict[type, "FunctionCtx"] = {}


class FunctionCtx:
    """Stand-in for the autograd ``ctx`` while tracing."""

    def __init__(self, args):
        self.saved_tensors = ()
        self.needs_input_grad = tuple(isinstance(a, TensorProxy) and a.requires_grad for a in args)
        self.materialize_grads = True
        self.non_differentiable = ()

    def save_for_backward(self, *tensors):
        self.saved_tensors = tuple(tensors)

    def mark_non_differentiable(self, *tensors):
        self.non_differentiable = tuple(tensors)

    def set_materialize_grads(self, value: bool):
        self.materialize_grads = bool(value)

    def mark_dirty(self, *tensors):
        raise NotImplementedError("in-place autograd.Function (ctx.mark_dirty) is not supported inside jit")


def _new_style(cls) -> bool:
    base = getattr(torch.autograd.function, "_SingleLevelFunction", torch.autograd.Function)
    sc = getattr(cls, "setup_context", None)
    return sc is not None and getattr(sc, "__func__", sc) is not getattr(base.setup_context, "__func__", base.setup_context)


def _run_forward(cls, args, kwargs):
    from ..core.jit_ext import user_code_tracing

    ctx = FunctionCtx(args)
    with user_code_tracing():
        if _new_style(cls):
            out = cls.forward(*args, **kwargs)
            cls.setup_context(ctx, args, out)
        else:
            out = cls.forward(ctx, *args, **kwargs)
    _last_ctx[cls] = ctx
    return out


def symbol_for(cls) -> Symbol:
    sym = _symbols.get(cls)
    if sym is not None:
        return sym

    def meta(*args, **kwargs):
        return _run_forward(cls, args, kwargs)

    name = f"autograd_function_{cls.__name__}"
    sym = Symbol(name, meta, id=f"autograd_function.{cls.__module__}.{cls.__qualname__}", is_prim=False)
    register_symbol(sym)
    _symbols[cls] = sym
    _register_vjp(cls, sym)
    return sym


def _register_vjp(cls, sym):
    from ..core.transforms import register_vjp

    def rule(*args, **kwargs):
        out = sym(*args, **kwargs)
        ctx = _last_ctx[cls]

        def bwd(*grads):
            from ..core.jit_ext import ThunderTorchFunctionMode, _state_stack, _AcquisitionState

            nd = {id(t) for t in ctx.non_differentiable}
            outs = tree_flatten(out)[0]
            gs = []
            for o, g in zip(outs, grads):
                if g is None and ctx.materialize_grads and isinstance(o, TensorProxy) and id(o) not in nd:
                    from .. import torch as ltorch

                    g = ltorch.zeros_like(o)
                gs.append(g)
            _state_stack.append(_AcquisitionState())
            try:
                with ThunderTorchFunctionMode():
                    res = cls.backward(ctx, *gs)
            finally:
                _state_stack.pop()
            res = res if isinstance(res, tuple) else (res,)
            return tuple(res[: len(args)]) + (None,) * max(0, len(args) - len(res))

        return out, bwd

    register_vjp(sym)(rule)


def apply(cls, *args, **kwargs):
    """``cls.apply(*args)`` while tracing."""
    return symbol_for(cls)(*args, **kwargs)
