"""``torch.library.custom_op`` operators as Thunder symbols with their registered autograd.

Parity: reference ``thunder/torch/custom_op.py:67-445`` (custom op -> symbol, fake-impl meta,
``setup_context``-driven saved tensors, backward from ``register_autograd``) and the ``custom_op``
executor ``thunder/executors/custom_op_ex.py:15``.

* **Symbol**: ``custom_op_<ns>_<name>``; meta = the op's fake (abstract) implementation run on meta
  tensors; executed by the ``custom_op`` executor through the dispatcher overload.
* **Autograd**: if the op has ``register_autograd(backward, setup_context=...)``, the VJP rule runs
  ``setup_context`` at TRACE time on a recording context: the proxies it passes to
  ``ctx.save_for_backward`` (and any tensor it stores as a ctx attribute) become exactly the
  saved-for-backward values of the compiled forward; its other attributes (dtypes, shapes, flags
  derived from the inputs) are constants of the program.  The backward is one symbol,
  ``custom_op_bwd_<ns>_<name>``, that rebuilds a ctx from those values and calls the registered
  backward — no re-execution of the forward, unlike the generic opaque-op rule.  (The reference
  recovers the saved indices by parsing ``setup_context``'s AST; running it on proxies gives the
  same information and also handles computed attributes.)
* If ``setup_context`` cannot run on proxies, the generic opaque rule (torch.autograd re-run) is
  used instead.
"""
from __future__ import annotations

import inspect

import torch

from ..core.proxies import Proxy, TensorProxy, NumberProxy, pyval
from ..core.pytree import tree_flatten, tree_map
from ..core.symbol import Symbol, register_symbol

try:
    from torch._library import custom_ops as _co
except ImportError:  # pragma: no cover
    _co = None

_symbols: dict = {}


def opdef_of(func):
    """The ``CustomOpDef`` behind ``func`` (the decorated function or its OpOverload), or None."""
    if _co is None:
        return None
    if isinstance(func, _co.CustomOpDef):
        return func
    if isinstance(func, torch._ops.OpOverload):
        return _co.OPDEFS.get(func._schema.name)
    return None


def _meta_tensor(x):
    if isinstance(x, TensorProxy):
        return torch.empty(x.shape, dtype=x.dtype, device="meta")
    if isinstance(x, NumberProxy):
        return pyval(x)
    return x


def _device_of(flat):
    for x in flat:
        if isinstance(x, TensorProxy):
            return x.device
    return torch.device("cpu")


def _proxy_like(o, device):
    if isinstance(o, torch.Tensor):
        return TensorProxy(shape=tuple(o.shape), device=device, dtype=o.dtype)
    return o


def _fwd_meta(op):
    def meta(*args, **kwargs):
        flat, _ = tree_flatten((args, kwargs))
        device = _device_of(flat)
        margs, mkwargs = tree_map(_meta_tensor, (args, kwargs))
        with torch.no_grad():
            out = op(*margs, **mkwargs)
        return tree_map(lambda o: _proxy_like(o, device), out)

    return meta


class _RecordingCtx:
    """Stands in for the autograd ctx while ``setup_context`` runs on proxies."""

    def __init__(self):
        object.__setattr__(self, "_saved", ())
        object.__setattr__(self, "_attrs", {})

    def save_for_backward(self, *ts):
        object.__setattr__(self, "_saved", ts)

    def mark_non_differentiable(self, *args):
        pass

    def set_materialize_grads(self, value):
        pass

    def __setattr__(self, k, v):
        self._attrs[k] = v

    def __getattr__(self, k):
        try:
            return object.__getattribute__(self, "_attrs")[k]
        except KeyError:
            raise AttributeError(k) from None


class _RuntimeCtx:
    """The ctx the registered backward receives: saved tensors plus the recorded attributes."""

    def __init__(self, saved, attrs, needs_input_grad):
        self.saved_tensors = tuple(saved)
        self.needs_input_grad = needs_input_grad
        for k, v in attrs.items():
            setattr(self, k, v)


class _BwdState:
    """What the backward symbol of one traced call needs besides its tensor operands.  It travels as
    the symbol's ``_state`` keyword, so the trace that calls the backward owns it (printed into the
    program's object context) and it is freed with that trace — no process-global registry."""

    __slots__ = ("n_saved", "tnames", "static", "needs", "input_likes")

    def __init__(self, n_saved, tnames, static, needs, input_likes):
        self.n_saved, self.tnames, self.static, self.needs = n_saved, tnames, static, needs
        self.input_likes = input_likes  # (shape, device, dtype) of each differentiable input, else None


def _bwd_impl(opdef):
    def impl(*flat, _state):
        st = _state
        saved = flat[:st.n_saved]
        tvals = flat[st.n_saved:st.n_saved + len(st.tnames)]
        grads = flat[st.n_saved + len(st.tnames):]
        attrs = dict(st.static)
        attrs.update(zip(st.tnames, tvals))
        res = opdef._backward_fn(_RuntimeCtx(saved, attrs, st.needs), *grads)
        return tuple(res) if isinstance(res, (tuple, list)) else (res,)

    return impl


def _bwd_meta(opdef):
    impl = _bwd_impl(opdef)

    def meta(*flat, _state):
        device = _device_of(flat)
        mflat = [_meta_tensor(x) for x in flat]
        try:
            with torch.no_grad():
                out = impl(*mflat, _state=_state)
            return tuple(_proxy_like(o, device) for o in out)
        except Exception:
            # the backward does not run on meta tensors: assume one gradient per tensor input
            return tuple(None if lk is None else TensorProxy(shape=lk[0], device=lk[1], dtype=lk[2])
                         for lk in _state.input_likes)

    return meta


def check_supported(opdef) -> None:
    """Refuse custom ops that mutate their arguments, as the reference does
    (``thunder/torch/custom_op.py:347-350``): a pure symbol would let DCE drop the write (e.g. a
    mutator returning None) and CSE merge two calls, losing the mutation without an error."""
    schema = opdef._opoverload._schema
    if schema.is_mutable:
        mutated = [a.name for a in schema.arguments if a.alias_info is not None and a.alias_info.is_write]
        raise NotImplementedError(
            f"custom op {opdef._namespace}::{opdef._name} mutates one or more of its arguments "
            f"({', '.join(mutated) or 'see its schema'}), which is not supported")


def custom_op_symbol(opdef) -> Symbol:
    """The Thunder symbol of a custom op (created, registered and made differentiable on first use)."""
    op = opdef._opoverload
    sym = _symbols.get(op)
    if sym is not None:
        return sym
    check_supported(opdef)
    qual = f"{opdef._namespace}::{opdef._name}"
    pname = "custom_op_" + "".join(c if c.isalnum() else "_" for c in f"{opdef._namespace}_{opdef._name}")
    from ..core.prims import OpTags

    # AUTO_REGISTERED: if setup_context cannot run on proxies, the generic opaque rule
    # (torch.autograd on the op itself) differentiates it
    sym = Symbol(pname, _fwd_meta(op), id=f"custom_op.{qual}", is_prim=True, tags=(OpTags.AUTO_REGISTERED,))
    sym.torch_fn = op
    register_symbol(sym)
    from ..executors import custom_opex

    custom_opex.register(sym, op)
    if opdef._backward_fn is not None and opdef._setup_context_fn is not None:
        bsym = Symbol(pname.replace("custom_op_", "custom_op_bwd_", 1), _bwd_meta(opdef),
                      id=f"custom_op_bwd.{qual}", is_prim=True)
        register_symbol(bsym)
        custom_opex.register(bsym, _bwd_impl(opdef))
        from ..core.transforms import register_vjp

        register_vjp(sym)(_make_rule(sym, bsym, opdef))
    _symbols[op] = sym
    return sym


def _make_rule(sym, bsym, opdef):
    sig = inspect.signature(opdef._init_fn)

    def rule(*args, **kwargs):
        try:
            bound = sig.bind(*args, **kwargs)
            bound.apply_defaults()
        except TypeError:
            return None
        inputs = tuple(bound.arguments.values())
        out = sym(*args, **kwargs)
        rc = _RecordingCtx()
        try:
            opdef._setup_context_fn(rc, inputs, out)
        except Exception:
            return None  # not traceable on proxies: the generic opaque rule takes over
        saved = tuple(rc._saved)
        tnames, tvals, static = [], [], {}
        for k, v in rc._attrs.items():
            if isinstance(v, TensorProxy):
                tnames.append(k)
                tvals.append(v)
            else:
                static[k] = tree_map(lambda x: pyval(x) if isinstance(x, NumberProxy) else x, v)
        if any(isinstance(x, Proxy) for x in tree_flatten(static)[0]):
            return None
        needs = tuple(isinstance(x, TensorProxy) and x.dtype.is_floating_point for x in inputs)
        outs = tuple(out) if isinstance(out, (tuple, list)) else (out,)
        likes = tuple((tuple(x.shape), x.device, x.dtype) if isinstance(x, TensorProxy) and x.dtype.is_floating_point
                      else None for x in inputs)
        state = _BwdState(len(saved), tuple(tnames), static, needs, likes)

        def bwd(*gs):
            if any(g is None for g in gs):
                from .. import torch as ltorch

                gs = tuple(ltorch.zeros_like(o) if g is None else g for g, o in zip(gs, outs))
            grads = bsym(*saved, *tvals, *gs, _state=state)
            grads = tuple(grads) if isinstance(grads, (tuple, list)) else (grads,)
            # one entry per positional argument of the call
            return tuple(grads[i] if i < len(grads) else None for i in range(len(args)))

        return out, bwd

    return rule
