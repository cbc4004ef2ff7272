"""Executor framework (parity: reference ``thunder/extend/__init__.py:35-664``).

An ``Executor`` maps symbol ids to ``ImplInfo`` (its own operator symbol, a
checker, an optional execution transform and an optional grad transform).
``FusionExecutor`` s additionally group claimed bound symbols into fused
regions in their ``fusion_pass``.  Executors are looked up by name through a
registry; the default priority order for MI355X is
``hipex (hand-written HIP kernels) → hipfuse (HIP fusion codegen) → torch → python``.
"""
from __future__ import annotations

import os
from typing import Any, Callable, Sequence

import torch

from ..core.symbol import Symbol, BoundSymbol, register_symbol
from ..core.proxies import TensorProxy
from ..core import dtypes


class ImplInfo:
    __slots__ = ("symbol", "checker", "execution_transform", "grad_transform")

    def __init__(self, symbol=None, checker=None, execution_transform=None, grad_transform=None):
        self.symbol = symbol
        self.checker = checker
        self.execution_transform = execution_transform
        self.grad_transform = grad_transform


def _always_true(*args, **kwargs):
    return True


def _resolve_printable_path(fn: Callable) -> str | None:
    """If ``fn`` is reachable as ``torch.<...>`` return that dotted path (so traces call torch directly)."""
    mod = getattr(fn, "__module__", None)
    name = getattr(fn, "__name__", None)
    if name is None:
        return None
    candidates = []
    if isinstance(fn, type(torch.Tensor.add)) or getattr(fn, "__objclass__", None) is torch._C.TensorBase:
        candidates.append(f"torch.Tensor.{name}")
    if mod:
        m = mod.replace("torch._C._nn", "torch.nn.functional").replace("torch._C._VariableFunctions", "torch")
        candidates.append(f"{m}.{name}")
    candidates.append(f"torch.{name}")
    candidates.append(f"torch.nn.functional.{name}")
    for c in candidates:
        if not c.startswith("torch"):
            continue
        try:
            obj = eval(c, {"torch": torch})
        except Exception:
            continue
        if obj is fn:
            return c
    return None


class Executor:
    def __init__(self, name: str, *, version: Any = None):
        self.name = name
        self.version = version
        self.implmap: dict[Any, ImplInfo] = {}
        self.opmap: dict[str, Symbol] = {}
        self._lookasides: dict[Callable, Callable] = {}

    def __repr__(self):
        return f"{type(self).__name__}('{self.name}')"

    def __hash__(self):
        return hash(self.name)

    def __eq__(self, other):
        return isinstance(other, Executor) and other.name == self.name

    # --- capability checks --------------------------------------------------------
    def can_execute_directly(self, bsym: BoundSymbol) -> bool:
        impl = self.implmap.get(bsym.sym.id)
        if impl is None:
            return False
        checker = impl.checker or _always_true
        try:
            return bool(checker(*bsym.args, **bsym.kwargs))
        except Exception:
            return False

    def can_execute(self, bsym: BoundSymbol) -> bool:
        return self.can_execute_directly(bsym)

    def can_fuse(self, bsym: BoundSymbol) -> bool:
        return False

    def get_impl(self, sym_id):
        return self.implmap.get(sym_id)

    def get_execution_transform(self, sym: Symbol):
        impl = self.implmap.get(sym.id)
        return None if impl is None else impl.execution_transform

    def get_grad_transform(self, sym: Symbol):
        impl = self.implmap.get(sym.id)
        return None if impl is None else impl.grad_transform

    # --- registration --------------------------------------------------------------
    def register_operator(
        self,
        name: str,
        *,
        meta: Callable | None = None,
        like: Symbol | None = None,
        fn: Callable,
        tags: Sequence = (),
        replaces: Callable | None = None,
        print_as: str | None = None,
        module=None,
    ) -> Symbol:
        """Creates an executor operator symbol implemented by ``fn``."""
        if meta is None:
            assert like is not None, "register_operator needs meta= or like="
            meta = like.meta
        if not tags and like is not None:
            tags = like.tags
        printable = print_as if print_as is not None else _resolve_printable_path(fn)
        op_name = name
        sym = Symbol(op_name, meta, id=f"{self.name}.{name}", is_prim=True, tags=tags, executor=self, print_as=printable)
        if printable is None:
            sym._exec_fn = fn
        else:
            sym._exec_fn = None
        sym.impl_fn = fn
        if like is not None and getattr(like, "written_args", None) is not None:
            sym.written_args = like.written_args
        self.opmap[name] = sym
        self.implmap[sym.id] = ImplInfo(symbol=sym)
        register_symbol(sym)
        if replaces is not None:
            self._lookasides[replaces] = sym
        return sym

    def register_implementation(
        self,
        id_or_symbol,
        op: Symbol | None = None,
        *,
        checker: Callable | None = None,
        execution_transform: Callable | None = None,
        grad_transform: Callable | None = None,
    ) -> None:
        sid = id_or_symbol.id if isinstance(id_or_symbol, Symbol) else id_or_symbol
        self.implmap[sid] = ImplInfo(symbol=op, checker=checker, execution_transform=execution_transform, grad_transform=grad_transform)

    def register_lookaside(self, fn: Callable, replacement: Callable) -> None:
        self._lookasides[fn] = replacement

    def register_python_lookaside(self, owner: Any, attr: str, replacement: Callable) -> None:
        """While a program is acquired, ``owner.attr`` (a python function, e.g. a model helper) is
        replaced by ``replacement``; the replacement may emit this executor's fused operators."""
        if not hasattr(self, "_python_lookasides"):
            self._python_lookasides = []
        self._python_lookasides.append((owner, attr, replacement))

    def bind_call_ctx(self, bsym: BoundSymbol, original: BoundSymbol | None = None) -> BoundSymbol:
        # Replay the exact torch callable the user invoked (keeps the user's call signature valid)
        if original is not None and getattr(bsym.sym, "replay_torch", False):
            tfn = getattr(original, "torch_fn", None)
            if tfn is not None:
                path = _resolve_printable_path(tfn)
                key = path if path is not None else f"_torchfn_{getattr(tfn, '__name__', 'op')}_{id(tfn) & 0xFFFF}"
                kwargs = bsym.kwargs
                if original.sym.id in _FACTORY_IDS and isinstance(bsym.output, TensorProxy):
                    # factory calls resolve dtype / device from torch's global defaults at trace
                    # time; pin them so the replay does not depend on the defaults at run time
                    kwargs = dict(kwargs)
                    if kwargs.get("dtype") is None:
                        kwargs["dtype"] = dtypes.to_torch_dtype(bsym.output.dtype)
                    if kwargs.get("device") is None:
                        kwargs["device"] = bsym.output.device
                    return bsym.from_bsym(kwargs=kwargs, _call_ctx={key: tfn})
                return bsym.from_bsym(_call_ctx={key: tfn})
        fn = getattr(bsym.sym, "_exec_fn", None)
        if fn is not None:
            return bsym.from_bsym(_call_ctx={bsym.sym.name: fn})
        return bsym


_FACTORY_IDS = frozenset(f"torch.{n}" for n in ("ones", "zeros", "empty", "full", "rand", "randn", "arange", "linspace",
                                                  "logspace", "eye", "randint", "randperm"))


class OperatorExecutor(Executor):
    pass


class FusionExecutor(Executor):
    """Executors that group bound symbols into fused regions (reference :201-257).

    ``optimization fuel`` (env ``THUNDER_HIPFUSE_FUEL``) bounds the number of
    fusions created, to bisect a miscompiling fusion.
    """

    def __init__(self, name: str, *, version: Any = None):
        super().__init__(name, version=version)
        self._fuel = None
        fuel = os.environ.get(f"THUNDER_{name.upper()}_FUEL")
        if fuel is not None:
            self._fuel = int(fuel)

    def get_fuel(self, amount: int = 1) -> bool:
        if self._fuel is None:
            return True
        if self._fuel < amount:
            return False
        self._fuel -= amount
        return True

    def set_fuel(self, value: int | None) -> None:
        self._fuel = value

    def register_supported(self, id_or_symbol, checker: Callable | None = None) -> None:
        sid = id_or_symbol.id if isinstance(id_or_symbol, Symbol) else id_or_symbol
        self.implmap[sid] = ImplInfo(checker=checker)

    def can_fuse(self, bsym: BoundSymbol) -> bool:
        """A bsym is fusible if directly supported, or all its subsymbols are (recursively)."""
        if self.can_execute_directly(bsym):
            return True
        if not bsym.subsymbols:
            return False
        return all(self.can_fuse(s) for s in bsym.subsymbols)

    def can_execute(self, bsym: BoundSymbol) -> bool:
        return self.can_fuse(bsym)

    def fusion_pass(self, trace):
        return trace


class StatefulExecutor(OperatorExecutor):
    """Executor whose operators carry per-bound-symbol state objects (reference :284-353; used by FP8)."""

    def __init__(self, name: str, *, version: Any = None):
        super().__init__(name, version=version)
        self._states: dict[str, Any] = {}

    def get_state(self, key: str, factory: Callable[[], Any]):
        s = self._states.get(key)
        if s is None:
            s = factory()
            self._states[key] = s
        return s


class TemporaryExecutor(OperatorExecutor):
    """Ad-hoc executor for opaque user functions discovered while tracing (reference :356-455)."""

    _counter = 0

    def __init__(self):
        TemporaryExecutor._counter += 1
        super().__init__(f"__ad_hoc_executor_{TemporaryExecutor._counter}")


# -----------------------------------------------------------------------------------------
# Registry
# -----------------------------------------------------------------------------------------
_executor_map: dict[str, Executor] = {}
_default_executors: list[Executor] = []
_always_executors: list[Executor] = []


def register_executor(ex: Executor) -> Executor:
    _executor_map[ex.name] = ex
    return ex


def deregister_executor(ex: Executor | str) -> None:
    name = ex if isinstance(ex, str) else ex.name
    _executor_map.pop(name, None)
    remove_default_executor(name)


def get_all_executors() -> tuple[Executor, ...]:
    _ensure_builtin_executors()
    return tuple(_executor_map.values())


def get_executor(name: str) -> Executor | None:
    _ensure_builtin_executors()
    return _executor_map.get(name)


def get_default_executors() -> tuple[Executor, ...]:
    _ensure_builtin_executors()
    return tuple(_default_executors)


def get_always_executors() -> tuple[Executor, ...]:
    _ensure_builtin_executors()
    return tuple(_always_executors)


def add_default_executor(ex: Executor, *, last: bool = False) -> None:
    """Highest priority by default; ``last=True`` appends (below every registered default)."""
    remove_default_executor(ex.name)
    if last:
        _default_executors.append(ex)
    else:
        _default_executors.insert(0, ex)


def add_always_executor(ex: Executor) -> None:
    if ex not in _always_executors:
        _always_executors.append(ex)


def remove_default_executor(name: str) -> None:
    for i, e in enumerate(list(_default_executors)):
        if e.name == name:
            _default_executors.pop(i)
            break


def set_default_executors(exs: Sequence[Executor]) -> None:
    _default_executors.clear()
    _default_executors.extend(exs)


def resolve_executors(executors) -> tuple[Executor, ...]:
    if executors is None:
        return get_default_executors()
    out = []
    for e in executors:
        if isinstance(e, str):
            ex = get_executor(e)
            if ex is None:
                raise ValueError(f"Unknown executor {e}; known: {list(_executor_map)}")
            out.append(ex)
        elif isinstance(e, Executor):
            out.append(e)
        else:
            raise ValueError(f"Expected an executor or its name, got {e}")
    return tuple(out)


def add_executor_lists(a, b) -> tuple[Executor, ...]:
    out = list(a)
    for e in b:
        if e not in out:
            out.append(e)
    return tuple(out)


_builtin_loaded = False


def _ensure_builtin_executors():
    global _builtin_loaded
    if _builtin_loaded:
        return
    _builtin_loaded = True
    from ..executors import pythonex, torchex  # noqa: F401  (register themselves)
    from ..executors import hipex, hipfuse  # noqa: F401
    from ..executors import custom_opex  # noqa: F401
