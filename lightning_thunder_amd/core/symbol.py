"""Symbols and bound symbols (parity: reference ``thunder/core/symbol.py:120-355``, ``BoundSymbol`` :371,
``from_bsym_swap_proxies`` :444, ``BoundSymbolRHS`` :749).

Calling a ``Symbol`` while a trace is active runs its meta function and records a
``BoundSymbol``.  For composite (non-prim) symbols the meta is a decomposition
written in terms of other symbols; the bound symbols it records become the
``subsymbols`` of the new bound symbol, so executors can either claim the
composite op whole or fall through to its decomposition.
"""
from __future__ import annotations

import torch
from enum import Enum, auto
from types import ModuleType
from typing import Any, Callable, Sequence

from .codeutils import has_proxy_output, prettyprint, print_output_target, type_comment
from .proxies import Proxy, TensorProxy, NumberProxy
from .pytree import tree_flatten, tree_map, tree_unflatten
from .trace import get_tracectx
from . import dtypes


META_DEPTH = [0]
# The exact torch callable the user invoked (set by the acquisition frontend) so the torch
# executor can replay a top-level ltorch bound symbol with the user's own call signature.
CALLED_TORCH_FN = [None]


class BoundSymbolTag(Enum):
    RECOMPUTE_IN_BACKWARD = auto()
    BACKWARD = auto()
    DONT_AUTO_RECOMPUTE_IN_BACKWARD = auto()
    NO_GRAD = auto()  # recorded while grad mode was off (torch.no_grad / set_grad_enabled(False) in user code)


class Symbol:
    __slots__ = (
        "name",
        "meta",
        "id",
        "is_prim",
        "tags",
        "module",
        "executor",
        "python_printer",
        "python_impl",
        "_bind_postprocess",
        "is_fusion",
        "method_name",
        "_print_as",
        "__dict__",
    )

    def __init__(
        self,
        name: str,
        meta: Callable | None,
        *,
        id: Any = None,
        is_prim: bool = False,
        tags: Sequence = (),
        module: ModuleType | str | None = None,
        executor: Any = None,
        python_printer: Callable | None = None,
        python_impl: Callable | None = None,
        _bind_postprocess: Callable | None = None,
        is_fusion: bool = False,
        print_as: str | None = None,
    ):
        self.name = name
        self.meta = meta
        self.id = id if id is not None else name
        self.is_prim = is_prim
        self.tags = tuple(tags)
        self.module = module
        self.executor = executor
        self.python_printer = python_printer
        self.python_impl = python_impl
        self._bind_postprocess = _bind_postprocess
        self.is_fusion = is_fusion
        self.method_name = None
        self._print_as = print_as

    def __repr__(self):
        return f"[Symbol name={self.name}]"

    def __hash__(self):
        return hash(self.id)

    def __eq__(self, other):
        return isinstance(other, Symbol) and self.id == other.id and self.executor is other.executor

    def __reduce__(self):
        return (_lookup_symbol, (self.id,))

    @property
    def print_name(self) -> str:
        if self._print_as is not None:
            return self._print_as
        mod = self.module
        if isinstance(mod, ModuleType):
            short = {
                "lightning_thunder_amd.core.prims": "prims",
                "lightning_thunder_amd.torch": "ltorch",
                "lightning_thunder_amd.clang": "clang",
            }.get(mod.__name__, None)
            if short is not None:
                return f"{short}.{self.name}"
        elif isinstance(mod, str):
            return f"{mod}.{self.name}"
        return self.name

    def bind(self, *args, output, subsymbols=(), _call_ctx=None, **kwargs) -> "BoundSymbol":
        b = BoundSymbol(self, args=tuple(args), kwargs=kwargs, output=output, subsymbols=list(subsymbols), _call_ctx=_call_ctx)
        if self._bind_postprocess is not None:
            self._bind_postprocess(b)
        return b

    def __call__(self, *args, **kwargs):
        trace = get_tracectx()
        if trace is None:
            raise RuntimeError(
                f"Symbol {self.name} was called outside of a trace; wrap the function with lightning_thunder_amd.jit"
            )
        # Autocast hook (reference: symbol.py:294-298)
        if trace.autocast_dtype is not None and not self.is_prim:
            from ..transforms.autocast import maybe_autocast

            rule = maybe_autocast(self)
            if rule is not None:
                return rule(*args, **kwargs, dtype=trace.autocast_dtype)

        called_fn = CALLED_TORCH_FN[0]
        CALLED_TORCH_FN[0] = None
        tracker = trace.alias_tracker if len(trace.scopes) == 1 else None
        if tracker is not None:
            tracker.before_call(args, kwargs)
        # While a meta runs, torch calls made by the compiler itself (e.g. meta-tensor shape
        # inference) must execute eagerly instead of being traced by the acquisition mode.
        META_DEPTH[0] += 1
        try:
            if self.is_prim:
                result = self.meta(*args, **kwargs)
                subsymbols = []
                _propagate_requires_grad(self, args, kwargs, result)
            else:
                scope: list = []
                trace.push_scope(scope)
                try:
                    result = self.meta(*args, **kwargs)
                finally:
                    trace.pop_scope()
                subsymbols = scope
        finally:
            META_DEPTH[0] -= 1
        call_ctx = None
        if self.executor is not None and self.python_impl is None:
            impl = getattr(self, "_exec_fn", None)
            if impl is not None:
                call_ctx = {self.name: impl}
        bsym = self.bind(*args, output=result, subsymbols=subsymbols, _call_ctx=call_ctx, **kwargs)
        if called_fn is not None:
            bsym.torch_fn = called_fn
        if len(trace.scopes) == 1 and not torch.is_grad_enabled():
            # user code switched autograd off around this op (the interpreter runs torch.no_grad /
            # set_grad_enabled for real): its outputs are constants for the backward (reference:
            # grad-mode tracking in jit_ext / ltorch._set_grad_enabled_with_warning)
            bsym.tags.add(BoundSymbolTag.NO_GRAD)
            for o in bsym.flat_proxy_outs:
                if isinstance(o, TensorProxy):
                    o.requires_grad = False
        if self.is_prim or subsymbols or self.name in _LAYOUT_IDENTITIES or not _is_identity(bsym):
            # an op that decomposed to nothing and returns its own input (dropout in eval, a
            # same-dtype .to, cat of one tensor) is not recorded: a line "t1 = op(t1)" would
            # re-bind a name that dead-code elimination treats as produced twice
            trace.add_bound_symbol(bsym)
        if tracker is not None:
            result = tracker.after_call(bsym, result)
        return result


# identity at the proxy level but not at run time (memory layout)
_LAYOUT_IDENTITIES = {"contiguous"}


def _is_identity(bsym) -> bool:
    outs = bsym.flat_proxy_outs
    if not outs:
        return False
    ins = {id(a) for a in bsym.flat_proxy_args}
    return all(id(o) in ins for o in outs)


_symbol_registry: dict[Any, Symbol] = {}


def register_symbol(sym: Symbol) -> Symbol:
    _symbol_registry.setdefault(sym.id, sym)
    return sym


def _lookup_symbol(id):
    return _symbol_registry[id]


NON_DIFFERENTIABLE_TAG = "non_differentiable"


def _propagate_requires_grad(sym: Symbol, args, kwargs, result) -> None:
    if NON_DIFFERENTIABLE_TAG in sym.tags:
        return
    flat_in, _ = tree_flatten((args, kwargs))
    rg = any(isinstance(a, TensorProxy) and a.requires_grad for a in flat_in)
    if not rg:
        return
    flat_out, _ = tree_flatten(result)
    for o in flat_out:
        if isinstance(o, TensorProxy) and dtypes.is_inexact_dtype(o.dtype):
            o.requires_grad = True


class BoundSymbol:
    __slots__ = ("sym", "args", "kwargs", "output", "subsymbols", "header", "_call_ctx", "tags", "_flat_args", "_flat_outs", "torch_fn")

    def __init__(self, sym: Symbol, args=(), kwargs=None, output=None, subsymbols=(), header="", _call_ctx=None, tags=None):
        self.sym = sym
        self.args = tuple(args)
        self.kwargs = dict(kwargs) if kwargs else {}
        self.output = output
        self.subsymbols = list(subsymbols)
        self.header = header
        self._call_ctx = _call_ctx
        self.tags = set(tags) if tags else set()
        self._flat_args = None
        self._flat_outs = None
        self.torch_fn = None

    def from_bsym(self, **changes) -> "BoundSymbol":
        kw = dict(
            sym=self.sym,
            args=self.args,
            kwargs=self.kwargs,
            output=self.output,
            subsymbols=self.subsymbols,
            header=self.header,
            _call_ctx=self._call_ctx,
            tags=set(self.tags),
        )
        kw.update(changes)
        b = BoundSymbol(**kw)
        b.torch_fn = self.torch_fn
        return b

    # --- flattening -----------------------------------------------------------------
    @property
    def flat_args(self) -> list:
        if self._flat_args is None:
            self._flat_args, _ = tree_flatten((self.args, self.kwargs))
        return self._flat_args

    @property
    def flat_outs(self) -> list:
        if self._flat_outs is None:
            self._flat_outs, _ = tree_flatten(self.output)
        return self._flat_outs

    @property
    def flat_proxy_args(self) -> list:
        return [a for a in self.flat_args if isinstance(a, Proxy)]

    @property
    def flat_proxy_outs(self) -> list:
        return [o for o in self.flat_outs if isinstance(o, Proxy)]

    @property
    def flat_tensor_args(self) -> list:
        return [a for a in self.flat_args if isinstance(a, TensorProxy)]

    @property
    def flat_tensor_outs(self) -> list:
        return [o for o in self.flat_outs if isinstance(o, TensorProxy)]

    def swap_proxies(self, swap_map: dict[str, Proxy], *, skip_inputs=False, skip_output=False, skip_subsymbols=False):
        return from_bsym_swap_proxies(self, swap_map, skip_inputs=skip_inputs, skip_output=skip_output, skip_subsymbols=skip_subsymbols)

    # --- keys ------------------------------------------------------------------------
    def rhs(self):
        """Hashable right-hand side used by CSE (reference ``BoundSymbolRHS`` :749)."""

        def key(x):
            if isinstance(x, Proxy):
                return ("__proxy__", x.name)
            if isinstance(x, (list, tuple)):
                return (type(x).__name__,) + tuple(key(v) for v in x)
            if isinstance(x, dict):
                return ("dict",) + tuple((k, key(v)) for k, v in x.items())
            if isinstance(x, slice):
                return ("slice", key(x.start), key(x.stop), key(x.step))
            try:
                hash(x)
                return x
            except TypeError:
                return ("__id__", id(x))

        return (self.sym.id, id(self.sym.executor), key(self.args), key(self.kwargs))

    # --- printing ---------------------------------------------------------------------
    def call_name(self) -> str:
        if self._call_ctx:
            return next(iter(self._call_ctx.keys()))
        return self.sym.print_name

    def python(self, indent: int = 0, print_depth: int = 1, obj_ctx: dict | None = None) -> list[str]:
        pad = "  " * indent
        if self.sym.python_printer is not None:
            s = self.sym.python_printer(self, obj_ctx)
            lines = s if isinstance(s, list) else [s]
            return [pad + ln for ln in lines]
        arg_strs = [prettyprint(a, obj_ctx) for a in self.args]
        kwarg_strs = [f"{k}={prettyprint(v, obj_ctx)}" for k, v in self.kwargs.items()]
        call = f"{self.call_name()}({', '.join(arg_strs + kwarg_strs)})"
        if has_proxy_output(self.output):
            line = f"{print_output_target(self.output)} = {call}"
            tc = type_comment(self.output)
            if tc:
                line += f"  # {tc}"
        else:
            line = call
        lines = []
        if self.header:
            for h in self.header.splitlines():
                lines.append(pad + "# " + h)
        lines.append(pad + line)
        if print_depth > 0 and self.subsymbols and not self._call_ctx and not self.sym.is_fusion:
            for sub in self.subsymbols:
                for ln in sub.python(0, print_depth - 1, obj_ctx):
                    lines.append(pad + "  # " + ln.strip())
        elif self.sym.is_fusion and print_depth > 0:
            for sub in self.subsymbols:
                for ln in sub.python(0, 0, obj_ctx):
                    lines.append(pad + "  # " + ln.strip())
        return lines

    def __repr__(self):
        return "\n".join(self.python(0, 1))


def from_bsym_swap_proxies(
    bsym: BoundSymbol,
    swap_map: dict[str, Proxy],
    *,
    skip_inputs: bool = False,
    skip_output: bool = False,
    skip_subsymbols: bool = False,
) -> BoundSymbol:
    if not swap_map:
        return bsym

    def swap(x):
        if isinstance(x, Proxy):
            seen = set()
            while x.name in swap_map and x.name not in seen:
                seen.add(x.name)
                nx = swap_map[x.name]
                if nx is x:
                    break
                x = nx
        return x

    args = bsym.args if skip_inputs else tree_map(swap, bsym.args)
    kwargs = bsym.kwargs if skip_inputs else tree_map(swap, bsym.kwargs)
    output = bsym.output if skip_output else tree_map(swap, bsym.output)
    subsymbols = (
        bsym.subsymbols
        if skip_subsymbols
        else [from_bsym_swap_proxies(s, swap_map, skip_inputs=skip_inputs, skip_output=skip_output) for s in bsym.subsymbols]
    )
    return bsym.from_bsym(args=args, kwargs=kwargs, output=output, subsymbols=subsymbols)


def has_tags(bsym: BoundSymbol, tags) -> bool:
    return bool(set(tags) & set(bsym.sym.tags)) or bool(set(tags) & bsym.tags)
