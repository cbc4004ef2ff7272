"""Proxies: the values a trace computes on (parity: reference ``thunder/core/proxies.py``
``Proxy`` :94, ``TensorProxy`` :1442, ``FutureTensorProxy`` :1318, ``DistParallelType`` :1218-1224).

A proxy is a named placeholder with metadata.  ``TensorProxy`` carries shape,
device, dtype, ``requires_grad`` and the distributed annotations consumed by the
DDP/FSDP/TP transforms.  Operator overloads and tensor methods dispatch to the
active language context (``ltorch`` by default), which records bound symbols
into the active trace.
"""
from __future__ import annotations

import itertools
import math
from enum import Enum, auto
from numbers import Number
from typing import Any, Sequence

import torch

from . import dtypes
from .devices import to_device, device_str


from .symbolic import SymInt, make_shape

class DistParallelType(Enum):
    NONE = auto()
    REPLICATED = auto()
    FULLY_SHARDED = auto()
    COLUMN_WISE = auto()
    ROW_WISE = auto()


class ProxyTag(Enum):
    STATIC_MEMORY_LOCATION = auto()  # parameters/buffers: stable addresses across calls (hipGraph static inputs)
    RECOMPUTE_IN_BACKWARD = auto()
    DETACHED_AUTOGRAD_GRAPH = auto()


_fallback_counter = itertools.count()


def _get_tracectx():
    from .trace import get_tracectx

    return get_tracectx()


def make_proxy_name(prefix: str) -> str:
    trc = _get_tracectx()
    if trc is not None:
        return trc.make_name(prefix)
    return f"_{prefix}{next(_fallback_counter)}"


class Proxy:
    prefix = "p"

    def __init__(self, name: str | None = None, *, prefix: str | None = None, tags=None):
        if name is None:
            name = make_proxy_name(prefix or self.prefix)
        else:
            trc = _get_tracectx()
            if trc is not None:
                trc.add_name(name)
        self._name = name
        self.tags = set(tags) if tags else set()

    @property
    def name(self) -> str:
        return self._name

    def replace_name(self, name: str | None = None):
        """Returns a copy of this proxy with a new (or fresh) name."""
        return self.replace(name=name)

    def replace(self, **changes):
        raise NotImplementedError

    def type_string(self) -> str:
        return "Any"

    def __repr__(self):
        return f'<{type(self).__name__}(name="{self.name}")>'

    __hash__ = object.__hash__


class AnyProxy(Proxy):
    prefix = "obj"

    def __init__(self, value=None, name=None, *, prefix=None, tags=None):
        super().__init__(name, prefix=prefix, tags=tags)
        self.value = value

    def replace(self, **changes):
        return AnyProxy(changes.get("value", self.value), name=changes.get("name"), tags=self.tags)


class StringProxy(AnyProxy):
    prefix = "s"


class NumberProxy(Proxy):
    """A number whose value is known at trace time.

    With the default ``"constant values"`` cache option numbers are specialized,
    so NumberProxy mostly appears for values produced inside traces (e.g. by
    ``item``) and for symbolic-values caching.
    """

    prefix = "n"

    def __init__(self, value=None, python_type=None, name=None, *, prefix=None, tags=None):
        super().__init__(name, prefix=prefix, tags=tags)
        self.value = value
        self.python_type = python_type if python_type is not None else type(value)

    def replace(self, **changes):
        return type(self)(changes.get("value", self.value), self.python_type, name=changes.get("name"), tags=self.tags)

    def type_string(self):
        return self.python_type.__name__

    # A symbolic number (``cache="symbolic values"`` input) stays a trace input only while the
    # program passes it along to operations; anything that reads its value (Python arithmetic,
    # comparisons, branching, shapes, ``pyval``) specializes the program on that value: the hook
    # turns the input's prologue check back into a value check.
    _on_value = None

    def concrete(self):
        hook = self._on_value
        if hook is not None:
            hook()
        if self.value is None:
            raise NotImplementedError(
                f"the value of {self.name} ({self.python_type.__name__}) depends on tensor data (e.g. Tensor.item()) "
                "and is unknown while the program is traced: data-dependent Python control flow or arithmetic "
                "is not supported; express it with tensor operations (torch.where, masking) or move it out of "
                "the compiled function")
        return self.value

    def __index__(self):
        return int(self.concrete())

    def __int__(self):
        return int(self.concrete())

    def __float__(self):
        return float(self.concrete())

    def __bool__(self):
        return bool(self.concrete())

    def __eq__(self, other):
        if isinstance(other, Proxy):
            return self is other
        return self.concrete() == other

    def __ne__(self, other):
        return not self.__eq__(other)

    __hash__ = Proxy.__hash__

    def __round__(self, ndigits=None):
        return round(self.concrete(), ndigits)

    def __neg__(self):
        return -self.concrete()

    def __pos__(self):
        return +self.concrete()

    def __abs__(self):
        return abs(self.concrete())


def _number_binop(name):
    import operator

    op = getattr(operator, name)

    def fwd(self, other):
        if isinstance(other, Proxy) and not isinstance(other, NumberProxy):
            return NotImplemented  # e.g. a tensor: its reflected operator records the op
        return op(self.concrete(), other.concrete() if isinstance(other, NumberProxy) else other)

    def rev(self, other):
        if isinstance(other, Proxy) and not isinstance(other, NumberProxy):
            return NotImplemented
        return op(other.concrete() if isinstance(other, NumberProxy) else other, self.concrete())

    return fwd, rev


for _n in ("add", "sub", "mul", "truediv", "floordiv", "mod", "pow", "and_", "or_", "xor", "lshift", "rshift"):
    _f, _r = _number_binop(_n)
    _dn = _n.rstrip("_")
    setattr(NumberProxy, f"__{_dn}__", _f)
    setattr(NumberProxy, f"__r{_dn}__", _r)
for _n in ("lt", "le", "gt", "ge"):
    setattr(NumberProxy, f"__{_n}__", _number_binop(_n)[0])


class IntegerProxy(NumberProxy):
    prefix = "i"

    def __init__(self, value=None, python_type=int, name=None, *, prefix=None, tags=None):
        super().__init__(value, python_type, name, prefix=prefix, tags=tags)


class FloatProxy(NumberProxy):
    prefix = "f"

    def __init__(self, value=None, python_type=float, name=None, *, prefix=None, tags=None):
        super().__init__(value, python_type, name, prefix=prefix, tags=tags)


class ComplexProxy(NumberProxy):
    prefix = "c"

    def __init__(self, value=None, python_type=complex, name=None, *, prefix=None, tags=None):
        super().__init__(value, python_type, name, prefix=prefix, tags=tags)


# Collection proxies exist for API parity; traces here take flat arguments so
# these only wrap python containers that flow through prologues.
class TupleProxy(AnyProxy):
    prefix = "tup"


class ListProxy(AnyProxy):
    prefix = "lst"


class DictProxy(AnyProxy):
    prefix = "d"


def _ltorch():
    from .. import torch as ltorch

    return ltorch


def _capture_real(x):
    """A real tensor meeting a proxy in an operator (e.g. a constant built by an opaque call while
    tracing) becomes a constant input of the program."""
    if isinstance(x, torch.Tensor) and not isinstance(x, Proxy):
        from .jit_ext import _current_state

        st = _current_state()
        if st is not None:
            return st.proxify_constant(x)
    return x


def _method(name):
    def fn(self, *args, **kwargs):
        if args:
            args = tuple(_capture_real(a) for a in args)
        return getattr(_ltorch(), name)(self, *args, **kwargs)

    fn.__name__ = name
    return fn


def _rmethod(name):
    def fn(self, other):
        return getattr(_ltorch(), name)(_capture_real(other), self)

    fn.__name__ = "r" + name
    return fn


class TensorProxy(Proxy):
    prefix = "t"

    def __init__(
        self,
        name: str | None = None,
        *,
        like: "TensorProxy | torch.Tensor | None" = None,
        shape: Sequence[int] | None = None,
        device=None,
        dtype=None,
        requires_grad: bool | None = None,
        grad=None,
        distparallel_type: DistParallelType | None = None,
        thunder_fsdp_padding_size: int | None = None,
        prefix: str | None = None,
        tags=None,
    ):
        super().__init__(name, prefix=prefix, tags=tags)
        if like is not None:
            shape = tuple(like.shape) if shape is None else shape
            device = like.device if device is None else device
            dtype = like.dtype if dtype is None else dtype
            requires_grad = like.requires_grad if requires_grad is None else requires_grad
            if distparallel_type is None:
                distparallel_type = getattr(like, "distparallel_type", None)
            if thunder_fsdp_padding_size is None:
                thunder_fsdp_padding_size = getattr(like, "thunder_fsdp_padding_size", None)
        # symbolic dims (cache="symbolic values", core/symbolic.py) stay SymInts; everything else is a plain int
        self._shape = tuple(s if isinstance(s, SymInt) else int(s) for s in shape)
        self._device = to_device(device)
        self._dtype = dtypes.to_torch_dtype(dtype)
        self.requires_grad = bool(requires_grad) if requires_grad is not None else False
        self.distparallel_type = distparallel_type if distparallel_type is not None else DistParallelType.NONE
        self.thunder_fsdp_padding_size = thunder_fsdp_padding_size
        self.grad = grad

    # --- metadata -----------------------------------------------------------------
    @property
    def shape(self):
        return make_shape(self._shape)

    @property
    def device(self) -> torch.device:
        return self._device

    @property
    def dtype(self) -> torch.dtype:
        return self._dtype

    @property
    def ndim(self) -> int:
        return len(self._shape)

    def dim(self) -> int:
        return len(self._shape)

    ndimension = dim

    @property
    def numel(self):  # reference exposes numel as a property; calls go through _NumelInt
        n = math.prod(self._shape)
        return n if isinstance(n, SymInt) else _CallableInt(n)

    def nelement(self):
        return math.prod(self._shape)

    def size(self, dim: int | None = None):
        if dim is None:
            return make_shape(self._shape)
        return self._shape[dim]

    def stride(self, dim: int | None = None):
        strides = contiguous_strides(self._shape)
        return strides if dim is None else strides[dim]

    def element_size(self) -> int:
        return dtypes.itemsize(self._dtype)

    @property
    def itemsize(self):
        return dtypes.itemsize(self._dtype)

    @property
    def nbytes(self) -> int:
        return math.prod(self._shape) * dtypes.itemsize(self._dtype)

    @property
    def is_symbolic(self) -> bool:
        return any(isinstance(s, SymInt) for s in self._shape)

    @property
    def is_cuda(self) -> bool:
        return self._device.type == "cuda"

    @property
    def is_cpu(self) -> bool:
        return self._device.type == "cpu"

    @property
    def is_meta(self) -> bool:
        return self._device.type == "meta"

    @property
    def is_sparse(self):
        return False

    @property
    def is_quantized(self):
        return False

    @property
    def is_nested(self):
        return False

    @property
    def layout(self):
        return torch.strided

    def is_floating_point(self) -> bool:
        return dtypes.is_float_dtype(self._dtype)

    def is_complex(self) -> bool:
        return dtypes.is_complex_dtype(self._dtype)

    def is_contiguous(self, memory_format=None) -> bool:
        return True

    def get_device(self) -> int:
        return -1 if self._device.index is None else self._device.index

    def __len__(self):
        if not self._shape:
            raise TypeError("len() of a 0-d tensor")
        return self._shape[0]

    def __iter__(self):
        return iter(self.unbind(0))

    def __bool__(self):
        raise RuntimeError(
            f"Data-dependent control flow on tensor {self.name} is not supported while tracing "
            "(the value is not known at trace time)."
        )

    def __index__(self):
        raise RuntimeError(f"Cannot use tensor {self.name} as a python index while tracing")

    def replace(self, **changes):
        kw = dict(
            like=self,
            shape=changes.get("shape", self._shape),
            device=changes.get("device", self._device),
            dtype=changes.get("dtype", self._dtype),
            requires_grad=changes.get("requires_grad", self.requires_grad),
            distparallel_type=changes.get("distparallel_type", self.distparallel_type),
            thunder_fsdp_padding_size=changes.get("thunder_fsdp_padding_size", self.thunder_fsdp_padding_size),
            tags=changes.get("tags", self.tags),
        )
        return TensorProxy(changes.get("name"), **kw)

    def _shape_str(self) -> str:
        return "[" + ", ".join(s.expr if isinstance(s, SymInt) else repr(s) for s in self._shape) + "]"

    def type_string(self) -> str:
        return f"{device_str(self._device)} {dtypes.short_name(self._dtype)}{self._shape_str()}"

    def __repr__(self):
        return f'<TensorProxy(name="{self.name}", dtype={self._dtype}, shape={self._shape_str()}, device={self._device})>'

    # --- torch interop ---------------------------------------------------------------
    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        from .jit_ext import dispatch_torch_function

        return dispatch_torch_function(func, args, kwargs or {})

    # --- python operators ----------------------------------------------------------------
    __add__ = _method("add")
    __radd__ = _rmethod("add")
    __sub__ = _method("sub")
    __rsub__ = _rmethod("sub")
    __mul__ = _method("mul")
    __rmul__ = _rmethod("mul")
    __truediv__ = _method("true_divide")
    __rtruediv__ = _rmethod("true_divide")
    __floordiv__ = _method("floor_divide")
    __rfloordiv__ = _rmethod("floor_divide")
    __mod__ = _method("remainder")
    __rmod__ = _rmethod("remainder")
    __pow__ = _method("pow")
    __rpow__ = _rmethod("pow")
    __matmul__ = _method("matmul")
    __rmatmul__ = _rmethod("matmul")
    __and__ = _method("bitwise_and")
    __rand__ = _rmethod("bitwise_and")
    __or__ = _method("bitwise_or")
    __ror__ = _rmethod("bitwise_or")
    __xor__ = _method("bitwise_xor")
    __rxor__ = _rmethod("bitwise_xor")
    __lshift__ = _method("bitwise_left_shift")
    __rshift__ = _method("bitwise_right_shift")
    __eq__ = _method("eq")
    __ne__ = _method("ne")
    __lt__ = _method("lt")
    __le__ = _method("le")
    __gt__ = _method("gt")
    __ge__ = _method("ge")
    __neg__ = _method("neg")
    __pos__ = lambda self: self  # noqa: E731
    __abs__ = _method("abs")
    __invert__ = _method("bitwise_not")
    __getitem__ = _method("getitem")
    __hash__ = object.__hash__

    def __setitem__(self, key, value):
        _ltorch().setitem_(self, key, value)

    # in-place python operators
    def __iadd__(self, other):
        return _ltorch().add_(self, other)

    def __isub__(self, other):
        return _ltorch().sub_(self, other)

    def __imul__(self, other):
        return _ltorch().mul_(self, other)

    def __itruediv__(self, other):
        return _ltorch().div_(self, other)

    # --- tensor attributes --------------------------------------------------------------
    @property
    def T(self):
        return _ltorch().permute(self, tuple(reversed(range(self.ndim))))

    @property
    def mT(self):
        return _ltorch().transpose(self, -2, -1)

    @property
    def data(self):
        return _ltorch().detach(self)

    @property
    def real(self):
        return _ltorch().real(self)

    @property
    def imag(self):
        return _ltorch().imag(self)

    def __getattr__(self, attr: str):
        # Only called when normal lookup fails: resolve tensor methods in the language context.
        if attr.startswith("__") or attr.startswith("_"):
            raise AttributeError(attr)
        ltorch = _ltorch()
        method = ltorch.get_method(attr)
        if method is None:
            method = ltorch.resolve_fallback_method(attr)
        if method is None:
            raise AttributeError(f"TensorProxy has no attribute or method '{attr}' in the torch language context")

        tmethod = getattr(torch.Tensor, attr, None)

        def bound(*args, **kwargs):
            from .symbol import CALLED_TORCH_FN

            CALLED_TORCH_FN[0] = tmethod  # exact replay of the tensor method by the torch executor
            return method(self, *args, **kwargs)

        bound.__name__ = attr
        return bound


class _CallableInt(int):
    """``t.numel`` works both as a property (reference style) and as ``t.numel()`` (torch style)."""

    def __call__(self):
        return int(self)


class FutureTensorProxy(Proxy):
    """Result of an async collective; ``wait()`` materializes a TensorProxy (reference :1318)."""

    prefix = "fut"

    def __init__(self, name=None, *, like=None, shape=None, device=None, dtype=None, tags=None):
        super().__init__(name, tags=tags)
        if like is not None:
            shape = like.shape if shape is None else shape
            device = like.device if device is None else device
            dtype = like.dtype if dtype is None else dtype
        # symbolic dims (cache="symbolic values", core/symbolic.py) stay SymInts; everything else is a plain int
        self._shape = tuple(s if isinstance(s, SymInt) else int(s) for s in shape)
        self._device = to_device(device)
        self._dtype = dtype
        self.requires_grad = False

    @property
    def shape(self):
        return make_shape(self._shape)

    @property
    def dtype(self):
        return self._dtype

    @property
    def device(self):
        return self._device

    @property
    def ndim(self):
        return len(self._shape)

    def replace(self, **changes):
        return FutureTensorProxy(
            changes.get("name"),
            shape=changes.get("shape", self._shape),
            device=changes.get("device", self._device),
            dtype=changes.get("dtype", self._dtype),
            tags=self.tags,
        )

    def type_string(self):
        return f"FUTURE {device_str(self._device)} {dtypes.short_name(self._dtype)}{TensorProxy._shape_str(self)}"

    def wait(self):
        from ..distributed import prims as dist_prims

        return dist_prims.wait(self)


def contiguous_strides(shape) -> tuple[int, ...]:
    strides = []
    acc = 1
    for s in reversed(tuple(shape)):
        strides.append(acc)
        acc = acc * (s if isinstance(s, SymInt) else max(int(s), 1))  # symbolic dims are >= 2
    return tuple(reversed(strides))


def is_proxyable(x) -> bool:
    return isinstance(x, (torch.Tensor, Number)) and not isinstance(x, Proxy)


class DTensorProxy(TensorProxy):
    """Proxy of a ``torch.distributed.tensor.DTensor`` (parity: reference
    ``thunder/torch/experimental/dtensor_proxy.py``).  ``shape`` is the global shape; the device
    mesh, placements and local shape ride along.  Every torch operation on it is routed to a
    DTensor-aware opaque symbol (``distributed/dtensor.py``) whose meta runs DTensor's own sharding
    propagation on meta-device local tensors and whose execution is the torch op on the real
    DTensors (which issues the RCCL/gloo collectives a redistribution needs)."""

    prefix = "dt"

    def __init__(self, name=None, *, mesh=None, placements=None, local_shape=None, stride=None, like=None, **kw):
        super().__init__(name, like=like, **kw)
        if like is not None and isinstance(like, DTensorProxy):
            mesh = like.mesh if mesh is None else mesh
            placements = like.placements if placements is None else placements
            local_shape = like.local_shape if local_shape is None else local_shape
            stride = like.stride_ if stride is None else stride
        self.mesh = mesh
        self.placements = tuple(placements) if placements is not None else ()
        self.local_shape = tuple(local_shape) if local_shape is not None else tuple(self._shape)
        self.stride_ = tuple(stride) if stride is not None else None

    def replace(self, **changes):
        kw = dict(
            like=self,
            shape=changes.get("shape", self._shape),
            device=changes.get("device", self._device),
            dtype=changes.get("dtype", self._dtype),
            requires_grad=changes.get("requires_grad", self.requires_grad),
            tags=changes.get("tags", self.tags),
        )
        return DTensorProxy(changes.get("name"), **kw)

    def type_string(self) -> str:
        pl = ",".join(str(p) for p in self.placements)
        return f"{super().type_string()} DTensor[{pl}] local{list(self.local_shape)}"

    def _dispatch(self, name, *args, **kwargs):
        from .jit_ext import dispatch_torch_function

        return dispatch_torch_function(getattr(torch.Tensor, name), (self,) + args, kwargs)

    def __getattr__(self, attr: str):
        if attr.startswith("_"):
            raise AttributeError(attr)
        tm = getattr(torch.Tensor, attr, None)
        if tm is None:
            from torch.distributed.tensor import DTensor

            tm = getattr(DTensor, attr, None)
            if tm is None or not callable(tm):
                raise AttributeError(f"DTensorProxy has no attribute '{attr}'")

            def dt_bound(*args, **kwargs):
                from ..distributed.dtensor import dtensor_symbol

                return dtensor_symbol(tm, f"DTensor.{attr}")(self, *args, **kwargs)

            return dt_bound
        if not callable(tm):
            raise AttributeError(f"DTensorProxy has no attribute '{attr}'")

        def bound(*args, **kwargs):
            return self._dispatch(attr, *args, **kwargs)

        return bound


def _dt_op(name):
    def fn(self, *args):
        return self._dispatch(name, *args)

    fn.__name__ = name
    return fn


for _n in ("__add__", "__radd__", "__sub__", "__rsub__", "__mul__", "__rmul__", "__truediv__", "__rtruediv__",
           "__matmul__", "__rmatmul__", "__pow__", "__neg__", "__getitem__", "__eq__", "__ne__", "__lt__", "__le__",
           "__gt__", "__ge__"):
    setattr(DTensorProxy, _n, _dt_op(_n))
DTensorProxy.__hash__ = object.__hash__
DTensorProxy.T = property(lambda self: self._dispatch("permute", *reversed(range(self.ndim))))
DTensorProxy.mT = property(lambda self: self._dispatch("transpose", -2, -1))


def tensorproxy(t: torch.Tensor, name: str | None = None, **kw) -> TensorProxy:
    if _is_dtensor(t):
        return DTensorProxy(
            name,
            shape=tuple(t.shape),
            device=t.device,
            dtype=t.dtype,
            requires_grad=t.requires_grad,
            mesh=t.device_mesh,
            placements=t.placements,
            local_shape=tuple(t.to_local().shape),
            stride=tuple(t.stride()),
            **kw,
        )
    return TensorProxy(
        name,
        shape=tuple(t.shape),
        device=t.device,
        dtype=t.dtype,
        requires_grad=t.requires_grad,
        distparallel_type=getattr(t, "distparallel_type", None),
        thunder_fsdp_padding_size=getattr(t, "thunder_fsdp_padding_size", None),
        **kw,
    )


def _is_dtensor(t) -> bool:
    cls = type(t)
    return cls.__name__ == "DTensor" and cls.__module__.startswith("torch.distributed")


def proxy(x: Any, *, name: str | None = None):
    if isinstance(x, torch.Tensor):
        return tensorproxy(x, name=name)
    if isinstance(x, bool):
        return NumberProxy(x, bool, name=name, prefix="b")
    if isinstance(x, int):
        return IntegerProxy(x, name=name)
    if isinstance(x, float):
        return FloatProxy(x, name=name)
    if isinstance(x, complex):
        return ComplexProxy(x, name=name)
    if isinstance(x, str):
        return StringProxy(x, name=name)
    return AnyProxy(x, name=name)


def pyval(x):
    """Value of a number proxy (or the value itself); reading a symbolic number's value specializes it."""
    if isinstance(x, NumberProxy):
        return x.concrete()
    return x


def is_tensor_like(x) -> bool:
    return isinstance(x, (TensorProxy, torch.Tensor))
