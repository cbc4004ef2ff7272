"""ltorch: PyTorch-semantics operator language (parity: reference ``thunder/torch/__init__.py``;
``torchsymbol`` :153-255, ``_torch_to_thunder_function_map`` :102, ``rms_norm`` :4450-4477,
``cross_entropy`` :5226, SDPA decomposition :6190-6230, ``softmax`` :6239-6272).

Each ``@torchsymbol`` op is a Symbol whose meta is a decomposition into clang /
prims.  Executors can claim the op whole (the torch executor maps it straight to
ATen, the HIP executor to a hand-written kernel) or fall back to the
decomposition (the HIP fusion executor fuses its prims).  Torch callables that
have no ``@torchsymbol`` are auto-registered as opaque ops (see
``default_torch_ops``).
"""
from __future__ import annotations

import builtins
import math
import sys
from numbers import Number
from typing import Any, Callable, Sequence

import torch

from ..core import dtypes, prims
from ..core.baseutils import check
from ..core.symbolic import SymInt
from ..core.devices import to_device
from ..core.proxies import TensorProxy, NumberProxy, Proxy, pyval, FutureTensorProxy
from ..core.symbol import Symbol, register_symbol, NON_DIFFERENTIABLE_TAG
from .. import clang
from ..clang import ELEMENTWISE_TYPE_PROMOTION_KIND as K, canonicalize_dim, canonicalize_dims

_this = sys.modules[__name__]

_torch_to_thunder_function_map: dict[Callable, Symbol] = {}
_methods: dict[str, Callable] = {}
_inplace_to_out_of_place: dict[Callable, tuple[Callable, int]] = {}

Tensor = TensorProxy


def torchsymbol(*torchfns, is_method: bool = False, method_name: str | None = None, id: str | None = None, tags=(), is_prim=False):
    def decorator(fn):
        name = fn.__name__
        sym = Symbol(name, fn, id=id or f"torch.{name}", module=_this, tags=tags, is_prim=is_prim)
        tfns = [t for t in torchfns if t is not None]
        sym.torch_fn = tfns[0] if tfns else None
        register_symbol(sym)
        for tfn in torchfns:
            if tfn is not None:
                _torch_to_thunder_function_map[tfn] = sym
        if is_method:
            _methods[method_name or name] = sym
        sym.__doc__ = fn.__doc__
        return sym

    return decorator


def register_method(name: str, fn: Callable) -> None:
    _methods[name] = fn


def get_method(name: str):
    return _methods.get(name)


def resolve_fallback_method(name: str):
    """Tensor methods without a hand-written symbol: ``foo_`` becomes the out-of-place ``foo``
    plus ``copy_`` (functionalized by the frontend), anything else an auto-registered opaque op."""
    tm = getattr(torch.Tensor, name, None)
    if tm is None or not callable(tm):
        return None
    if name.endswith("_") and not name.endswith("__"):
        base = _methods.get(name[:-1])
        if base is None and callable(getattr(torch.Tensor, name[:-1], None)):
            from .default_torch_ops import opaque_symbol

            base = opaque_symbol(getattr(torch.Tensor, name[:-1]))
        if base is None:
            return None
        sym = _inplace(name, base)
    else:
        from .default_torch_ops import opaque_symbol

        sym = opaque_symbol(tm)
    _methods[name] = sym
    return sym


def _tfn(*names):
    """Resolves torch callables by dotted name, skipping ones missing in this torch build."""
    out = []
    for n in names:
        obj = torch
        ok = True
        for part in n.split("."):
            if not hasattr(obj, part):
                ok = False
                break
            obj = getattr(obj, part)
        if ok:
            out.append(obj)
    return out


def _dim_list(dim, ndim):
    if dim is None:
        return tuple(range(ndim))
    if isinstance(dim, (builtins.int, NumberProxy)):
        return (canonicalize_dim(ndim, pyval(dim)),)
    if len(dim) == 0:
        return tuple(range(ndim))
    return tuple(canonicalize_dim(ndim, pyval(d)) for d in dim)


def _shape_args(shape):
    if len(shape) == 1 and isinstance(shape[0], (tuple, list, torch.Size)):
        shape = tuple(shape[0])
    return tuple(pyval(s) for s in shape)


def _default_device(device):
    if device is None:
        return torch.device("cpu") if torch.get_default_device is None else to_device(torch.get_default_device())
    return to_device(device)


def _default_dtype(dtype, fallback=None):
    if dtype is None:
        return fallback if fallback is not None else torch.get_default_dtype()
    return dtype


# =========================================================================================
# Elementwise unary
# =========================================================================================
def _unary(name, clang_fn, *, method=True, extra_torch=()):
    torchfns = _tfn(f"{name}", f"Tensor.{name}", f"special.{name}") + list(extra_torch)

    def fn(a):
        return clang_fn(a)

    fn.__name__ = name
    return torchsymbol(*torchfns, is_method=method)(fn)


abs = _unary("abs", clang.abs)
acos = _unary("acos", clang.acos)
acosh = _unary("acosh", clang.acosh)
asin = _unary("asin", clang.asin)
asinh = _unary("asinh", clang.asinh)
atan = _unary("atan", clang.atan)
atanh = _unary("atanh", clang.atanh)
bitwise_not = _unary("bitwise_not", clang.bitwise_not)
ceil = _unary("ceil", clang.ceil)
cos = _unary("cos", clang.cos)
cosh = _unary("cosh", clang.cosh)
digamma = _unary("digamma", clang.digamma)
erf = _unary("erf", clang.erf)
erfc = _unary("erfc", clang.erfc)
erfinv = _unary("erfinv", clang.erfinv)
exp = _unary("exp", clang.exp)
exp2 = _unary("exp2", clang.exp2)
expm1 = _unary("expm1", clang.expm1)
floor = _unary("floor", clang.floor)
isfinite = _unary("isfinite", clang.isfinite)
lgamma = _unary("lgamma", clang.lgamma)
log = _unary("log", clang.log)
log10 = _unary("log10", clang.log10)
log1p = _unary("log1p", clang.log1p)
log2 = _unary("log2", clang.log2)
neg = _unary("neg", clang.neg, extra_torch=_tfn("negative", "Tensor.negative"))
reciprocal = _unary("reciprocal", clang.reciprocal)
round = _unary("round", clang.round)
rsqrt = _unary("rsqrt", clang.rsqrt)
sign = _unary("sign", clang.sign)
signbit = _unary("signbit", clang.signbit)
sin = _unary("sin", clang.sin)
sinh = _unary("sinh", clang.sinh)
sqrt = _unary("sqrt", clang.sqrt)
tan = _unary("tan", clang.tan)
tanh = _unary("tanh", clang.tanh, extra_torch=_tfn("nn.functional.tanh"))
trunc = _unary("trunc", clang.trunc, extra_torch=_tfn("fix", "Tensor.fix"))


@torchsymbol(torch.real, is_method=False)
def real(a):
    if not dtypes.is_complex_dtype(a.dtype):
        return a
    return prims.real(a)


@torchsymbol(torch.imag)
def imag(a):
    return prims.imag(a)


@torchsymbol(*_tfn("isnan", "Tensor.isnan"), is_method=True)
def isnan(a):
    return clang.ne(a, a)


@torchsymbol(*_tfn("isinf", "Tensor.isinf"), is_method=True)
def isinf(a):
    return logical_and(logical_not(isfinite(a)), logical_not(isnan(a)))


@torchsymbol(*_tfn("square", "Tensor.square"), is_method=True)
def square(a):
    return mul(a, a)


@torchsymbol(*_tfn("sigmoid", "Tensor.sigmoid", "nn.functional.sigmoid", "special.expit"), is_method=True)
def sigmoid(a):
    # 1 / (1 + exp(-a)) computed in fp32 for low precision inputs
    compute, result = clang.elementwise_type_promotion(a, type_promotion_kind=K.INT_TO_FLOAT)
    x = clang.maybe_convert_to_dtype(a, compute)
    y = prims.reciprocal(prims.add(prims.exp(prims.neg(x)), 1.0))
    return clang.maybe_convert_to_dtype(y, result)


@torchsymbol(*_tfn("relu", "Tensor.relu", "nn.functional.relu"), is_method=True)
def relu(a, inplace: bool = False):
    out = clang.where(clang.le(a, 0), _zero_like_scalar(a), a)  # NaN-propagating like torch.relu
    if inplace:
        return prims.copy_(out, a)
    return out


def _zero_like_scalar(a):
    return 0 if dtypes.is_integer_dtype(a.dtype) else 0.0


@torchsymbol(*_tfn("nn.functional.relu6"))
def relu6(a, inplace: bool = False):
    return clamp(a, 0, 6)


@torchsymbol(*_tfn("nn.functional.leaky_relu"))
def leaky_relu(a, negative_slope: float = 0.01, inplace: bool = False):
    return clang.where(clang.gt(a, 0), a, mul(a, negative_slope))


@torchsymbol(*_tfn("nn.functional.elu"))
def elu(a, alpha: float = 1.0, inplace: bool = False):
    return clang.where(clang.gt(a, 0), a, mul(expm1(a), alpha))


@torchsymbol(*_tfn("nn.functional.silu"))
def silu(a, inplace: bool = False):
    compute, result = clang.elementwise_type_promotion(a, type_promotion_kind=K.INT_TO_FLOAT)
    x = clang.maybe_convert_to_dtype(a, compute)
    y = prims.div(x, prims.add(prims.exp(prims.neg(x)), 1.0))
    return clang.maybe_convert_to_dtype(y, result)


@torchsymbol(*_tfn("nn.functional.gelu"))
def gelu(a, approximate: str = "none"):
    compute, result = clang.elementwise_type_promotion(a, type_promotion_kind=K.INT_TO_FLOAT)
    x = clang.maybe_convert_to_dtype(a, compute)
    if approximate == "none":
        y = prims.mul(prims.mul(x, 0.5), prims.add(prims.erf(prims.mul(x, 1.0 / math.sqrt(2.0))), 1.0))
    elif approximate == "tanh":
        inner = prims.mul(prims.add(x, prims.mul(prims.mul(prims.mul(x, x), x), 0.044715)), math.sqrt(2.0 / math.pi))
        y = prims.mul(prims.mul(x, 0.5), prims.add(prims.tanh(inner), 1.0))
    else:
        raise ValueError(f"gelu: unknown approximation {approximate}")
    return clang.maybe_convert_to_dtype(y, result)


@torchsymbol(*_tfn("nn.functional.softplus"))
def softplus(a, beta: float = 1.0, threshold: float = 20.0):
    scaled = mul(a, beta)
    return where(gt(scaled, threshold), a, true_divide(log1p(exp(scaled)), beta))


@torchsymbol(*_tfn("nn.functional.mish"))
def mish(a, inplace: bool = False):
    return mul(a, tanh(softplus(a)))


@torchsymbol(*_tfn("nn.functional.hardswish"))
def hardswish(a, inplace: bool = False):
    return true_divide(mul(a, clamp(add(a, 3), 0, 6)), 6)


@torchsymbol(*_tfn("nn.functional.hardtanh"))
def hardtanh(a, min_val: float = -1.0, max_val: float = 1.0, inplace: bool = False):
    return clamp(a, min_val, max_val)


@torchsymbol(*_tfn("nn.functional.logsigmoid"))
def logsigmoid(a):
    return neg(softplus(neg(a)))


# =========================================================================================
# Elementwise binary
# =========================================================================================
@torchsymbol(torch.add, torch.Tensor.add, *_tfn("Tensor.__add__"), is_method=True)
def add(a, b, *, alpha=None):
    if alpha is not None and pyval(alpha) != 1:
        b = clang.mul(b, pyval(alpha))
    return clang.add(a, b)


@torchsymbol(torch.sub, torch.Tensor.sub, *_tfn("subtract", "Tensor.subtract"), is_method=True)
def sub(a, b, *, alpha=None):
    if alpha is not None and pyval(alpha) != 1:
        b = clang.mul(b, pyval(alpha))
    return clang.sub(a, b)


@torchsymbol(*_tfn("rsub", "Tensor.rsub"))
def rsub(a, b, *, alpha=None):
    return sub(b, a, alpha=alpha)


@torchsymbol(torch.mul, torch.Tensor.mul, *_tfn("multiply", "Tensor.multiply"), is_method=True)
def mul(a, b):
    return clang.mul(a, b)


@torchsymbol(torch.true_divide, torch.Tensor.true_divide, is_method=True)
def true_divide(a, b):
    return clang.true_divide(a, b)


@torchsymbol(torch.div, torch.Tensor.div, *_tfn("divide", "Tensor.divide"), is_method=True)
def div(a, b, *, rounding_mode=None):
    if rounding_mode is None:
        return clang.true_divide(a, b)
    if rounding_mode == "trunc":
        return trunc(clang.true_divide(a, b)) if not _is_int(a, b) else _int_trunc_div(a, b)
    if rounding_mode == "floor":
        return floor_divide(a, b)
    raise ValueError(f"div: rounding_mode {rounding_mode}")


def _is_int(a, b):
    _, r = clang.elementwise_type_promotion(a, b, type_promotion_kind=K.DEFAULT)
    return dtypes.is_integer_dtype(r)


def _int_trunc_div(a, b):
    q = floor_divide(a, b)
    r = remainder(a, b)
    adj = logical_and(ne(r, 0), ne(lt(a, 0), lt(b, 0)))
    return where(adj, add(q, 1), q)


@torchsymbol(torch.floor_divide, torch.Tensor.floor_divide, is_method=True)
def floor_divide(a, b):
    return clang.floor_divide(a, b)


@torchsymbol(torch.remainder, torch.Tensor.remainder, is_method=True)
def remainder(a, b):
    return clang.remainder(a, b)


@torchsymbol(torch.fmod, torch.Tensor.fmod, is_method=True)
def fmod(a, b):
    return clang.fmod(a, b)


@torchsymbol(torch.pow, torch.Tensor.pow, is_method=True)
def pow(a, b):
    if isinstance(b, (builtins.int, builtins.float)) and not isinstance(b, builtins.bool) and isinstance(a, TensorProxy):
        if b == 2:
            return mul(a, a)
        if b == 1:
            return a
        if b == 0.5:
            return sqrt(a)
    return clang.pow(a, b)


@torchsymbol(torch.maximum, torch.Tensor.maximum, is_method=True)
def maximum(a, b):
    return clang.maximum(a, b)


@torchsymbol(torch.minimum, torch.Tensor.minimum, is_method=True)
def minimum(a, b):
    return clang.minimum(a, b)


@torchsymbol(torch.atan2, torch.Tensor.atan2, is_method=True)
def atan2(a, b):
    return clang.atan2(a, b)


@torchsymbol(torch.copysign, torch.Tensor.copysign, is_method=True)
def copysign(a, b):
    return clang.copysign(a, b)


@torchsymbol(torch.nextafter, torch.Tensor.nextafter, is_method=True)
def nextafter(a, b):
    return clang.nextafter(a, b)


def _cmp(name, clang_fn):
    def fn(a, b):
        return clang_fn(a, b)

    fn.__name__ = name
    return torchsymbol(*_tfn(name, f"Tensor.{name}"), is_method=True)(fn)


eq = _cmp("eq", clang.eq)
ne = _cmp("ne", clang.ne)
lt = _cmp("lt", clang.lt)
le = _cmp("le", clang.le)
gt = _cmp("gt", clang.gt)
ge = _cmp("ge", clang.ge)
_torch_to_thunder_function_map.update({torch.greater: gt, torch.less: lt, torch.greater_equal: ge, torch.less_equal: le, torch.not_equal: ne})

bitwise_and = _cmp("bitwise_and", clang.bitwise_and)
bitwise_or = _cmp("bitwise_or", clang.bitwise_or)
bitwise_xor = _cmp("bitwise_xor", clang.bitwise_xor)
bitwise_left_shift = _cmp("bitwise_left_shift", clang.bitwise_left_shift)
bitwise_right_shift = _cmp("bitwise_right_shift", clang.bitwise_right_shift)


def _to_bool(a):
    if isinstance(a, TensorProxy):
        return a if a.dtype == torch.bool else clang.ne(a, 0)
    return builtins.bool(pyval(a))


@torchsymbol(torch.logical_and, torch.Tensor.logical_and, is_method=True)
def logical_and(a, b):
    return clang.bitwise_and(_to_bool(a), _to_bool(b))


@torchsymbol(torch.logical_or, torch.Tensor.logical_or, is_method=True)
def logical_or(a, b):
    return clang.bitwise_or(_to_bool(a), _to_bool(b))


@torchsymbol(torch.logical_xor, torch.Tensor.logical_xor, is_method=True)
def logical_xor(a, b):
    return clang.bitwise_xor(_to_bool(a), _to_bool(b))


@torchsymbol(torch.logical_not, torch.Tensor.logical_not, is_method=True)
def logical_not(a):
    if isinstance(a, TensorProxy):
        return clang.eq(a, 0) if a.dtype != torch.bool else clang.bitwise_xor(a, True)
    return not pyval(a)


@torchsymbol(torch.where, torch.Tensor.where, is_method=True)
def where(pred, a=None, b=None):
    check(a is not None and b is not None, "where with a single argument (nonzero) is data-dependent and unsupported")
    return clang.where(pred, a, b)


@torchsymbol(torch.clamp, torch.Tensor.clamp, *_tfn("clip", "Tensor.clip"), is_method=True)
def clamp(a, min=None, max=None):
    if min is not None:
        a = clang.where(clang.lt(a, min), min, a)
    if max is not None:
        a = clang.where(clang.gt(a, max), max, a)
    return a


@torchsymbol(*_tfn("clamp_min", "Tensor.clamp_min"), is_method=True)
def clamp_min(a, min):
    return clamp(a, min=min)


@torchsymbol(*_tfn("clamp_max", "Tensor.clamp_max"), is_method=True)
def clamp_max(a, max):
    return clamp(a, max=max)


@torchsymbol(torch.lerp, torch.Tensor.lerp, is_method=True)
def lerp(start, end, weight):
    return add(start, mul(weight, sub(end, start)))


@torchsymbol(torch.masked_fill, torch.Tensor.masked_fill, is_method=True)
def masked_fill(a, mask, value):
    if isinstance(value, TensorProxy):
        value = clang.maybe_convert_to_dtype(value, a.dtype)
    else:
        value = pyval(value)
        if dtypes.is_integer_dtype(a.dtype) and isinstance(value, builtins.float) and not math.isinf(value):
            value = builtins.int(value)
    return clang.where(mask, value, a)


@torchsymbol(*_tfn("addcmul", "Tensor.addcmul"), is_method=True)
def addcmul(a, t1, t2, *, value=1):
    return add(a, mul(mul(t1, t2), value))


@torchsymbol(*_tfn("addcdiv", "Tensor.addcdiv"), is_method=True)
def addcdiv(a, t1, t2, *, value=1):
    return add(a, mul(true_divide(t1, t2), value))


@torchsymbol(*_tfn("nan_to_num", "Tensor.nan_to_num"), is_method=True)
def nan_to_num(a, nan=0.0, posinf=None, neginf=None):
    finfo = torch.finfo(a.dtype)
    posinf = finfo.max if posinf is None else posinf
    neginf = finfo.min if neginf is None else neginf
    a = where(isnan(a), nan, a)
    a = where(logical_and(isinf(a), gt(a, 0)), posinf, a)
    return where(logical_and(isinf(a), lt(a, 0)), neginf, a)


# =========================================================================================
# Conversions
# =========================================================================================
@torchsymbol(torch.Tensor.to, is_method=True)
def to(a, *args, **kwargs):
    device = kwargs.pop("device", None)
    dtype = kwargs.pop("dtype", None)
    kwargs.pop("non_blocking", None)
    kwargs.pop("copy", None)
    memory_format = kwargs.pop("memory_format", None)
    for x in args:
        if isinstance(x, torch.dtype):
            dtype = x
        elif isinstance(x, (torch.device, str)):
            device = x
        elif isinstance(x, TensorProxy):
            dtype, device = x.dtype, x.device
    out = a
    if device is not None:
        out = clang.device_put(out, device)
    if dtype is not None:
        out = clang.maybe_convert_to_dtype(out, dtype)
    if memory_format is not None and memory_format is not torch.preserve_format:
        # a layout change: recorded (so the call is replayed with its memory_format) even when
        # dtype and device already match
        out = contiguous(out, memory_format=memory_format)
    return out


@torchsymbol(torch.Tensor.type_as, is_method=True)
def type_as(a, b):
    return clang.maybe_convert_to_dtype(a, b.dtype)


def _cast_method(name, dtype):
    def fn(a, memory_format=None):
        return clang.maybe_convert_to_dtype(a, dtype)

    fn.__name__ = name
    return torchsymbol(getattr(torch.Tensor, name), is_method=True)(fn)


tensor_float = _cast_method("float", torch.float32)
double = _cast_method("double", torch.float64)
half = _cast_method("half", torch.float16)
bfloat16 = _cast_method("bfloat16", torch.bfloat16)
long = _cast_method("long", torch.int64)
tensor_int = _cast_method("int", torch.int32)
tensor_bool = _cast_method("bool", torch.bool)
short = _cast_method("short", torch.int16)
byte = _cast_method("byte", torch.uint8)
char = _cast_method("char", torch.int8)


@torchsymbol(torch.Tensor.type, is_method=True)
def tensor_type(a, dtype=None, non_blocking=False):
    check(dtype is not None, "Tensor.type() without a dtype returns a string and is not traceable")
    if isinstance(dtype, str):
        dtype = {"torch.FloatTensor": torch.float32, "torch.cuda.FloatTensor": torch.float32}.get(dtype)
    return clang.maybe_convert_to_dtype(a, dtype)


@torchsymbol(torch.Tensor.cuda, is_method=True)
def cuda(a, device=None, non_blocking=False, memory_format=None):
    return clang.device_put(a, "cuda" if device is None else device)


@torchsymbol(torch.Tensor.cpu, is_method=True)
def cpu(a, memory_format=None):
    return clang.device_put(a, "cpu")


# =========================================================================================
# Creation
# =========================================================================================
def _infer_device(device):
    if device is None:
        try:
            d = torch.get_default_device()
        except AttributeError:
            d = torch.device("cpu")
        return to_device(d)
    return to_device(device)


@torchsymbol(torch.full)
def full(shape, fill_value, *, dtype=None, device=None, layout=None, requires_grad=False, pin_memory=False, out=None):
    if dtype is None:
        fv = pyval(fill_value)
        dtype = torch.bool if isinstance(fv, builtins.bool) else (torch.int64 if isinstance(fv, builtins.int) else torch.get_default_dtype())
    return clang.full(tuple(pyval(s) for s in shape), pyval(fill_value), device=_infer_device(device), dtype=dtype)


@torchsymbol(torch.full_like)
def full_like(a, fill_value, *, dtype=None, device=None, layout=None, requires_grad=False, memory_format=None, pin_memory=False):
    return clang.full(a.shape, pyval(fill_value), device=to_device(device) if device is not None else a.device, dtype=dtype or a.dtype)


@torchsymbol(torch.zeros)
def zeros(*shape, dtype=None, device=None, layout=None, requires_grad=False, pin_memory=False, out=None):
    return clang.full(_shape_args(shape), 0, device=_infer_device(device), dtype=_default_dtype(dtype))


@torchsymbol(torch.ones)
def ones(*shape, dtype=None, device=None, layout=None, requires_grad=False, pin_memory=False, out=None):
    return clang.full(_shape_args(shape), 1, device=_infer_device(device), dtype=_default_dtype(dtype))


@torchsymbol(torch.empty)
def empty(*shape, dtype=None, device=None, layout=None, requires_grad=False, pin_memory=False, memory_format=None, out=None):
    return prims.empty(_shape_args(shape), device=_infer_device(device), dtype=_default_dtype(dtype))


@torchsymbol(torch.zeros_like)
def zeros_like(a, *, dtype=None, device=None, layout=None, requires_grad=False, memory_format=None, pin_memory=False):
    return full_like(a, 0, dtype=dtype, device=device)


@torchsymbol(torch.ones_like)
def ones_like(a, *, dtype=None, device=None, layout=None, requires_grad=False, memory_format=None, pin_memory=False):
    return full_like(a, 1, dtype=dtype, device=device)


@torchsymbol(torch.empty_like)
def empty_like(a, *, dtype=None, device=None, layout=None, requires_grad=False, memory_format=None, pin_memory=False):
    return prims.empty(a.shape, device=to_device(device) if device else a.device, dtype=dtype or a.dtype)


@torchsymbol(torch.Tensor.new_zeros, is_method=True)
def new_zeros(a, *shape, dtype=None, device=None, requires_grad=False, layout=None, pin_memory=False):
    return clang.full(_shape_args(shape), 0, device=to_device(device) if device else a.device, dtype=dtype or a.dtype)


@torchsymbol(torch.Tensor.new_ones, is_method=True)
def new_ones(a, *shape, dtype=None, device=None, requires_grad=False, layout=None, pin_memory=False):
    return clang.full(_shape_args(shape), 1, device=to_device(device) if device else a.device, dtype=dtype or a.dtype)


@torchsymbol(torch.Tensor.new_full, is_method=True)
def new_full(a, shape, fill_value, *, dtype=None, device=None, requires_grad=False, layout=None, pin_memory=False):
    return clang.full(tuple(shape), pyval(fill_value), device=to_device(device) if device else a.device, dtype=dtype or a.dtype)


@torchsymbol(torch.Tensor.new_empty, is_method=True)
def new_empty(a, *shape, dtype=None, device=None, requires_grad=False, layout=None, pin_memory=False):
    return prims.empty(_shape_args(shape), device=to_device(device) if device else a.device, dtype=dtype or a.dtype)


@torchsymbol(torch.arange)
def arange(start, end=None, step=1, *, dtype=None, device=None, layout=None, requires_grad=False, pin_memory=False, out=None):
    start, end, step = pyval(start), pyval(end), pyval(step)
    if end is None:
        start, end = 0, start
    if dtype is None:
        dtype = torch.int64 if builtins.all(isinstance(x, builtins.int) for x in (start, end, step)) else torch.get_default_dtype()
    length = builtins.max(0, math.ceil((end - start) / step))
    return prims.iota(length, start=start, step=step, device=_infer_device(device), dtype=dtype)


@torchsymbol(torch.linspace)
def linspace(start, end, steps, *, dtype=None, device=None, layout=None, requires_grad=False, pin_memory=False, out=None):
    dtype = dtype or torch.get_default_dtype()
    device = _infer_device(device)
    if steps == 1:
        return clang.full((1,), start, device=device, dtype=dtype)
    idx = prims.iota(steps, start=0, step=1, device=device, dtype=torch.float32)
    step = (end - start) / (steps - 1)
    return clang.maybe_convert_to_dtype(add(mul(idx, step), start), dtype)


@torchsymbol(torch.tensor)
def tensor(data, *, dtype=None, device=None, requires_grad=False, pin_memory=False):
    return prims.tensor_from_sequence(data, dtype=dtype, device=_infer_device(device))


@torchsymbol(torch.rand)
def rand(*shape, generator=None, dtype=None, device=None, layout=None, requires_grad=False, pin_memory=False, out=None):
    return prims.uniform(_shape_args(shape), 0.0, 1.0, device=_infer_device(device), dtype=_default_dtype(dtype))


@torchsymbol(torch.rand_like)
def rand_like(a, *, dtype=None, device=None, layout=None, requires_grad=False, memory_format=None):
    return prims.uniform(a.shape, 0.0, 1.0, device=to_device(device) if device else a.device, dtype=dtype or a.dtype)


@torchsymbol(torch.randn)
def randn(*shape, generator=None, dtype=None, device=None, layout=None, requires_grad=False, pin_memory=False, out=None):
    return prims.randn(_shape_args(shape), device=_infer_device(device), dtype=_default_dtype(dtype))


@torchsymbol(torch.randn_like)
def randn_like(a, *, dtype=None, device=None, layout=None, requires_grad=False, memory_format=None):
    return prims.randn(a.shape, device=to_device(device) if device else a.device, dtype=dtype or a.dtype)


@torchsymbol(torch.Tensor.uniform_, is_method=True)
def uniform_(a, from_=0.0, to=1.0, *, generator=None):
    return prims.copy_(prims.uniform(a.shape, from_, to, device=a.device, dtype=a.dtype), a)


def uniform_philox(shape, minval=0.0, maxval=1.0, *, device, dtype, seed, offset):
    return prims.uniform_philox(tuple(shape), minval, maxval, device=to_device(device), dtype=dtype, seed=seed, offset=offset)


# =========================================================================================
# Shape ops
# =========================================================================================
@torchsymbol(torch.reshape, torch.Tensor.reshape, is_method=True)
def reshape(a, *shape):
    return clang.reshape(a, _shape_args(shape))


@torchsymbol(torch.Tensor.view, is_method=True)
def view(a, *shape):
    if len(shape) == 1 and isinstance(shape[0], torch.dtype):
        check(dtypes.itemsize(shape[0]) == dtypes.itemsize(a.dtype), "view(dtype) with different item sizes is unsupported")
        return prims.bitcast(a, shape[0])
    return clang.reshape(a, _shape_args(shape))


@torchsymbol(torch.Tensor.view_as, torch.Tensor.reshape_as, is_method=True)
def view_as(a, b):
    return clang.reshape(a, b.shape)


register_method("reshape_as", view_as)


@torchsymbol(torch.flatten, torch.Tensor.flatten, is_method=True)
def flatten(a, start_dim: int = 0, end_dim: int = -1):
    if a.ndim == 0:
        return clang.reshape(a, (1,))
    s = canonicalize_dim(a.ndim, start_dim)
    e = canonicalize_dim(a.ndim, end_dim)
    if s >= e:
        return a
    shape = tuple(a.shape[:s]) + (math.prod(a.shape[s:e + 1]),) + tuple(a.shape[e + 1:])
    return clang.reshape(a, shape)


@torchsymbol(torch.unflatten, torch.Tensor.unflatten, is_method=True)
def unflatten(a, dim, sizes):
    dim = canonicalize_dim(a.ndim, dim)
    sizes = list(sizes)
    if -1 in sizes:
        i = sizes.index(-1)
        sizes[i] = a.shape[dim] // math.prod(s for s in sizes if s != -1)
    return clang.reshape(a, tuple(a.shape[:dim]) + tuple(sizes) + tuple(a.shape[dim + 1:]))


@torchsymbol(torch.permute, torch.Tensor.permute, is_method=True)
def permute(a, *dims):
    dims = _shape_args(dims)
    return clang.transpose(a, canonicalize_dims(a.ndim, dims))


@torchsymbol(torch.transpose, torch.Tensor.transpose, *_tfn("swapaxes", "Tensor.swapaxes", "swapdims", "Tensor.swapdims"), is_method=True)
def transpose(a, dim0, dim1):
    if a.ndim == 0:
        return a
    d0 = canonicalize_dim(a.ndim, dim0)
    d1 = canonicalize_dim(a.ndim, dim1)
    perm = list(range(a.ndim))
    perm[d0], perm[d1] = perm[d1], perm[d0]
    return clang.transpose(a, perm)


@torchsymbol(torch.t, torch.Tensor.t, is_method=True)
def t(a):
    if a.ndim < 2:
        return a
    return transpose(a, 0, 1)


@torchsymbol(torch.movedim, torch.Tensor.movedim, *_tfn("moveaxis", "Tensor.moveaxis"), is_method=True)
def movedim(a, source, destination):
    src = _dim_list(source, a.ndim)
    dst = _dim_list(destination, a.ndim)
    perm = [-1] * a.ndim
    for s, d in zip(src, dst):
        perm[d] = s
    rest = iter(i for i in range(a.ndim) if i not in src)
    perm = [p if p != -1 else next(rest) for p in perm]
    return clang.transpose(a, perm)


@torchsymbol(torch.unsqueeze, torch.Tensor.unsqueeze, is_method=True)
def unsqueeze(a, dim):
    return clang.unsqueeze(a, pyval(dim))


@torchsymbol(torch.squeeze, torch.Tensor.squeeze, is_method=True)
def squeeze(a, dim=None):
    if dim is None:
        return clang.squeeze(a)
    return clang.squeeze(a, _dim_list(dim, a.ndim) if a.ndim else ())


@torchsymbol(torch.Tensor.expand, is_method=True)
def expand(a, *shape):
    return clang.expand(a, _shape_args(shape))


@torchsymbol(torch.Tensor.expand_as, is_method=True)
def expand_as(a, b):
    return clang.expand(a, tuple(b.shape))


@torchsymbol(torch.broadcast_to)
def broadcast_to(a, shape):
    return clang.expand(a, tuple(shape))


@torchsymbol(torch.Tensor.repeat, is_method=True)
def repeat(a, *repeats):
    repeats = _shape_args(repeats)
    check(len(repeats) >= a.ndim, "repeat: number of repeats must be >= ndim")
    a = clang.reshape(a, (1,) * (len(repeats) - a.ndim) + tuple(a.shape))
    # expand each dim with a new leading axis then merge
    shape_interleaved = []
    bdims = []
    for i, (r, s) in enumerate(zip(repeats, a.shape)):
        shape_interleaved += [r, s]
        bdims.append(2 * i + 1)
    x = prims.broadcast_in_dim(a, tuple(shape_interleaved), tuple(bdims))
    return clang.reshape(x, tuple(r * s for r, s in zip(repeats, a.shape)))


@torchsymbol(torch.repeat_interleave, torch.Tensor.repeat_interleave, is_method=True)
def repeat_interleave(a, repeats, dim=None, *, output_size=None):
    check(isinstance(repeats, (builtins.int, NumberProxy)), "repeat_interleave with tensor repeats is data-dependent")
    repeats = pyval(repeats)
    if dim is None:
        a = flatten(a)
        dim = 0
    dim = canonicalize_dim(a.ndim, dim)
    shape = list(a.shape)
    x = clang.unsqueeze(a, dim + 1)
    tgt = list(x.shape)
    tgt[dim + 1] = repeats
    x = clang.expand(x, tgt)
    shape[dim] = shape[dim] * repeats
    return clang.reshape(x, tuple(shape))


@torchsymbol(torch.split, torch.Tensor.split, is_method=True)
def split(a, split_size_or_sections, dim: int = 0):
    dim = canonicalize_dim(a.ndim, dim)
    n = a.shape[dim]
    if isinstance(split_size_or_sections, (builtins.int, NumberProxy)):
        s = pyval(split_size_or_sections)
        sizes = [s] * (n // s) + ([n % s] if n % s else [])
    else:
        sizes = [pyval(x) for x in split_size_or_sections]
    outs = []
    start = 0
    for s in sizes:
        outs.append(clang.slice_in_dim(a, start, start + s, 1, dim))
        start += s
    return tuple(outs)


@torchsymbol(*_tfn("Tensor.split_with_sizes"), is_method=True)
def split_with_sizes(a, split_sizes, dim: int = 0):
    return split(a, list(split_sizes), dim)


@torchsymbol(torch.chunk, torch.Tensor.chunk, is_method=True)
def chunk(a, chunks: int, dim: int = 0):
    dim = canonicalize_dim(a.ndim, dim)
    n = a.shape[dim]
    size = math.ceil(n / chunks)
    return split(a, size, dim)


@torchsymbol(torch.tensor_split, torch.Tensor.tensor_split, is_method=True)
def tensor_split(a, indices_or_sections, dim: int = 0):
    dim = canonicalize_dim(a.ndim, dim)
    n = a.shape[dim]
    if isinstance(indices_or_sections, builtins.int):
        k = indices_or_sections
        q, r = divmod(n, k)
        sizes = [q + 1] * r + [q] * (k - r)
    else:
        idx = [0] + list(indices_or_sections) + [n]
        sizes = [idx[i + 1] - idx[i] for i in range(len(idx) - 1)]
    return split(a, sizes, dim)


@torchsymbol(torch.unbind, torch.Tensor.unbind, is_method=True)
def unbind(a, dim: int = 0):
    dim = canonicalize_dim(a.ndim, dim)
    return tuple(clang.squeeze(clang.slice_in_dim(a, i, i + 1, 1, dim), (dim,)) for i in range(a.shape[dim]))


@torchsymbol(torch.cat, *_tfn("concat", "concatenate"))
def cat(tensors, dim: int = 0):
    tensors = [t for t in tensors if not (t.ndim == 1 and t.shape[0] == 0)] or list(tensors)[:1]
    return clang.cat(list(tensors), dim)


@torchsymbol(torch.stack)
def stack(tensors, dim: int = 0):
    rank = tensors[0].ndim + 1
    dim = canonicalize_dim(rank, dim)
    return clang.cat([clang.unsqueeze(t, dim) for t in tensors], dim)


@torchsymbol(torch.hstack)
def hstack(tensors):
    return cat(tensors, 0 if tensors[0].ndim == 1 else 1)


@torchsymbol(torch.vstack)
def vstack(tensors):
    return cat([t if t.ndim > 1 else clang.unsqueeze(t, 0) for t in tensors], 0)


@torchsymbol(torch.narrow, torch.Tensor.narrow, is_method=True)
def narrow(a, dim, start, length):
    dim = canonicalize_dim(a.ndim, dim)
    start = pyval(start)
    if start < 0:
        start += a.shape[dim]
    return clang.slice_in_dim(a, start, start + pyval(length), 1, dim)


@torchsymbol(torch.select, torch.Tensor.select, is_method=True)
def select(a, dim, index):
    dim = canonicalize_dim(a.ndim, dim)
    index = pyval(index)
    if index < 0:
        index += a.shape[dim]
    return clang.squeeze(clang.slice_in_dim(a, index, index + 1, 1, dim), (dim,))


@torchsymbol(torch.flip, torch.Tensor.flip, is_method=True)
def flip(a, *dims):
    dims = _shape_args(dims)
    return clang.flip(a, dims)


@torchsymbol(torch.roll, torch.Tensor.roll, is_method=True)
def roll(a, shifts, dims=None):
    if dims is None:
        return reshape(roll(flatten(a), shifts, 0), a.shape)
    shifts = (shifts,) if isinstance(shifts, builtins.int) else tuple(shifts)
    dims = (dims,) if isinstance(dims, builtins.int) else tuple(dims)
    for s, d in zip(shifts, dims):
        d = canonicalize_dim(a.ndim, d)
        n = a.shape[d]
        s = s % n if n else 0
        if s:
            a = clang.cat([clang.slice_in_dim(a, n - s, n, 1, d), clang.slice_in_dim(a, 0, n - s, 1, d)], d)
    return a


@torchsymbol(torch.Tensor.contiguous, is_method=True)
def contiguous(a, memory_format=torch.contiguous_format):
    return a


@torchsymbol(torch.clone, torch.Tensor.clone, is_method=True)
def clone(a, *, memory_format=None):
    return prims.shallow_copy(a)


@torchsymbol(torch.detach, torch.Tensor.detach, is_method=True, tags=(NON_DIFFERENTIABLE_TAG,))
def detach(a):
    # Recorded as an opaque op so autodiff can stop gradients here.
    return TensorProxy(like=a, requires_grad=False)


register_method("detach_", detach)


@torchsymbol(torch.tril, torch.Tensor.tril, is_method=True)
def tril(a, diagonal: int = 0):
    rows, cols = a.shape[-2], a.shape[-1]
    r = prims.iota(rows, start=0, step=1, device=a.device, dtype=torch.int64)
    c = prims.iota(cols, start=0, step=1, device=a.device, dtype=torch.int64)
    mask = clang.le(clang.sub(clang.unsqueeze(c, 0), clang.unsqueeze(r, 1)), diagonal)
    zero = False if a.dtype == torch.bool else 0
    return clang.where(mask, a, zero)


@torchsymbol(torch.triu, torch.Tensor.triu, is_method=True)
def triu(a, diagonal: int = 0):
    rows, cols = a.shape[-2], a.shape[-1]
    r = prims.iota(rows, start=0, step=1, device=a.device, dtype=torch.int64)
    c = prims.iota(cols, start=0, step=1, device=a.device, dtype=torch.int64)
    mask = clang.ge(clang.sub(clang.unsqueeze(c, 0), clang.unsqueeze(r, 1)), diagonal)
    zero = False if a.dtype == torch.bool else 0
    return clang.where(mask, a, zero)


@torchsymbol(*_tfn("nn.functional.pad"))
def pad(a, pad, mode: str = "constant", value=None):
    if mode != "constant":
        # reflect / replicate / circular: ATen's kernels (and their autograd) as an opaque op
        from .default_torch_ops import opaque_symbol

        return opaque_symbol(torch.nn.functional.pad, "nn.functional.pad")(a, tuple(pyval(p) for p in pad), mode=mode)
    value = 0 if value is None else pyval(value)
    cfg = [(0, 0, 0)] * a.ndim
    for i in range(len(pad) // 2):
        d = a.ndim - 1 - i
        cfg[d] = (pad[2 * i], pad[2 * i + 1], 0)
    if builtins.all(lo >= 0 and hi >= 0 for lo, hi, _ in cfg):
        return prims.pad(a, value, cfg)
    # negative padding = slicing
    out = a
    for d, (lo, hi, _) in enumerate(cfg):
        if lo < 0 or hi < 0:
            out = clang.slice_in_dim(out, builtins.max(-lo, 0), out.shape[d] - builtins.max(-hi, 0), 1, d)
    cfg2 = [(builtins.max(lo, 0), builtins.max(hi, 0), 0) for lo, hi, _ in cfg]
    return prims.pad(out, value, cfg2)


@torchsymbol(torch.index_select, torch.Tensor.index_select, is_method=True)
def index_select(a, dim, index):
    return clang.take(a, index, dim)


@torchsymbol(torch.gather, torch.Tensor.gather, is_method=True)
def gather(a, dim, index, *, sparse_grad=False):
    return clang.take_along_axis(a, index, dim)


@torchsymbol(torch.take_along_dim, is_method=False)
def take_along_dim(a, indices, dim=None):
    if dim is None:
        return clang.take_along_axis(flatten(a), flatten(indices), 0)
    return clang.take_along_axis(a, indices, dim)


@torchsymbol(torch.scatter_add, torch.Tensor.scatter_add, is_method=True)
def scatter_add(a, dim, index, src):
    return prims.scatter_add(a, index, src, canonicalize_dim(a.ndim, dim))


@torchsymbol(torch.scatter, torch.Tensor.scatter, is_method=True)
def scatter(a, dim, index, src=None, *, value=None, reduce=None):
    check(reduce is None, "scatter with reduce is not supported")
    if src is None:
        src = clang.full(index.shape, value, device=a.device, dtype=a.dtype)
    return prims.scatter(a, index, src, canonicalize_dim(a.ndim, dim))


@torchsymbol(torch.index_add, torch.Tensor.index_add, is_method=True)
def index_add(a, dim, index, source, *, alpha=1):
    if alpha != 1:
        source = mul(source, alpha)
    return prims.index_add(a, index, source, canonicalize_dim(a.ndim, dim))


@torchsymbol(torch.index_put, torch.Tensor.index_put, is_method=True)
def index_put(a, indices, values, accumulate=False):
    return prims.index_put(a, tuple(indices), values, accumulate)


@torchsymbol(torch.outer, torch.Tensor.outer, *_tfn("ger"), is_method=True)
def outer(a, b):
    return mul(clang.unsqueeze(a, 1), clang.unsqueeze(b, 0))


# getitem --------------------------------------------------------------------------------
def getitem(a, key):
    return _getitem_sym(a, key)


def _normalize_key(key):
    if not isinstance(key, tuple):
        key = (key,)
    return key


@torchsymbol(torch.Tensor.__getitem__, id="torch.Tensor.__getitem__")
def _getitem_sym(a, key):
    key = _normalize_key(key)
    # Advanced indexing with tensors
    tensor_keys = [k for k in key if isinstance(k, TensorProxy)]
    if tensor_keys:
        return _advanced_getitem(a, key)
    if builtins.any(isinstance(k, builtins.list) for k in key):
        # a list of indices (``x[[-2]]``, ``x[:, [0, 2]]``): advanced indexing with constant indices
        return _opaque_index(a, tuple(pyval(k) if isinstance(k, NumberProxy) else k for k in key))
    # expand ellipsis
    n_specified = builtins.sum(1 for k in key if k is not None and k is not Ellipsis)
    if builtins.any(k is Ellipsis for k in key):
        i = next(j for j, k in enumerate(key) if k is Ellipsis)
        key = key[:i] + (slice(None),) * (a.ndim - n_specified) + key[i + 1:]
    else:
        key = key + (slice(None),) * (a.ndim - n_specified)
    starts, ends, strides = [], [], []
    squeeze_dims = []
    unsqueeze_positions = []
    dim = 0
    out_dim = 0
    for k in key:
        if k is None:
            unsqueeze_positions.append(out_dim)
            out_dim += 1
            continue
        size = a.shape[dim]
        if isinstance(k, (builtins.int, NumberProxy)) and not isinstance(k, builtins.bool):
            idx = pyval(k)
            if idx < 0:
                idx += size
            check(0 <= idx < size, lambda: f"index {pyval(k)} is out of bounds for dimension {dim} with size {size}", IndexError)
            starts.append(idx)
            ends.append(idx + 1)
            strides.append(1)
            squeeze_dims.append(dim)
        elif isinstance(k, slice):
            s, e, st = _slice_indices(k, size)
            st = pyval(st)
            check(st > 0, "step must be greater than zero")
            if e < s:
                e = s
            starts.append(s)
            ends.append(e)
            strides.append(st)
            out_dim += 1
        else:
            raise TypeError(f"Unsupported index {k!r}")
        dim += 1
    out = a
    if builtins.any(s != 0 for s in starts) or builtins.any(e != sz for e, sz in zip(ends, a.shape)) or builtins.any(st != 1 for st in strides):
        out = prims.slice_prim(a, starts, ends, strides)
    if squeeze_dims:
        out = prims.squeeze(out, tuple(squeeze_dims))
    if unsqueeze_positions:
        out = clang.unsqueeze(out, unsqueeze_positions)
    return out


def _slice_indices(k: slice, size):
    """``slice.indices`` that keeps symbolic dims / bounds symbolic (``slice.indices`` itself turns them
    into plain ints through ``__index__``); the clamping comparisons record shape guards."""
    from ..core.symbolic import SymInt

    if not builtins.any(isinstance(v, SymInt) for v in (k.start, k.stop, k.step, size)):
        return k.indices(pyval(size))
    step = 1 if k.step is None else pyval(k.step)
    check(step > 0, "step must be greater than zero")

    def norm(v, default):
        if v is None:
            return default
        v = pyval(v)
        if v < 0:
            v = v + size
            if v < 0:
                return 0
        elif v > size:
            return size
        return v

    return norm(k.start, 0), norm(k.stop, size), step


def _advanced_getitem(a, key):
    # Supports a single tensor index in one position (possibly with basic slices elsewhere).
    positions = [i for i, k in enumerate(key) if isinstance(k, TensorProxy)]
    if len(positions) == 1 and not builtins.any(k is Ellipsis or k is None for k in key):
        p = positions[0]
        idx = key[p]
        if idx.dtype == torch.bool:
            raise RuntimeError("boolean mask indexing is data-dependent and unsupported while tracing")
        pre = tuple(key[:p])
        base = _getitem_sym(a, pre + (slice(None),) * (a.ndim - len(pre))) if builtins.any(not (isinstance(k, slice) and k == slice(None)) for k in pre) else a
        out = clang.take(base, _wrap_negative_indices(idx, base.shape[p]), p)
        rest = key[p + 1:]
        if rest:
            out = _getitem_sym(out, (slice(None),) * (p + idx.ndim) + tuple(rest))
        return out
    return _opaque_index(a, key)


def _wrap_negative_indices(idx, size):
    return idx  # torch executors handle negative indices in index_select/take


_opaque_index = None  # set by default_torch_ops


register_method("__getitem__", getitem)


@torchsymbol(id="torch.setitem_")
def setitem_(a, key, value):
    from .default_torch_ops import functional_setitem

    out = functional_setitem(a, key, value)
    return prims.copy_(out, a)


# =========================================================================================
# Reductions
# =========================================================================================
def _reduction_dtype(a, dtype):
    if dtype is not None:
        return dtype
    if dtypes.is_integer_dtype(a.dtype):
        return torch.int64
    return a.dtype


def _restore_keepdim(out, a, dims, keepdim):
    if not keepdim:
        return out
    shape = [1 if i in dims else s for i, s in enumerate(a.shape)]
    return clang.reshape(out, tuple(shape))


@torchsymbol(torch.sum, torch.Tensor.sum, is_method=True)
def sum(a, dim=None, keepdim: bool = False, *, dtype=None):
    dims = _dim_list(dim, a.ndim)
    result_dtype = _reduction_dtype(a, dtype)
    compute = clang.compute_dtype(result_dtype)
    x = clang.maybe_convert_to_dtype(a, compute)
    out = prims.sum(x, dims) if a.ndim else x
    out = clang.maybe_convert_to_dtype(out, result_dtype)
    return _restore_keepdim(out, a, dims, keepdim)


@torchsymbol(torch.prod, torch.Tensor.prod, is_method=True)
def prod(a, dim=None, keepdim: bool = False, *, dtype=None):
    dims = _dim_list(dim, a.ndim)
    result_dtype = _reduction_dtype(a, dtype)
    x = clang.maybe_convert_to_dtype(a, clang.compute_dtype(result_dtype))
    out = prims.prod(x, dims) if a.ndim else x
    return _restore_keepdim(clang.maybe_convert_to_dtype(out, result_dtype), a, dims, keepdim)


@torchsymbol(torch.mean, torch.Tensor.mean, is_method=True)
def mean(a, dim=None, keepdim: bool = False, *, dtype=None):
    dims = _dim_list(dim, a.ndim)
    result_dtype = dtype or a.dtype
    check(dtypes.is_inexact_dtype(result_dtype), "mean requires a floating point dtype")
    compute = clang.compute_dtype(result_dtype)
    x = clang.maybe_convert_to_dtype(a, compute)
    n = math.prod(a.shape[d] for d in dims) if a.ndim else 1
    out = prims.sum(x, dims) if a.ndim else x
    # a symbolic element count stays symbolic (the division happens at run time on the bound dims)
    out = prims.div(out, n if isinstance(n, SymInt) else builtins.float(n))
    return _restore_keepdim(clang.maybe_convert_to_dtype(out, result_dtype), a, dims, keepdim)


def _correction(unbiased, correction):
    if correction is not None:
        return pyval(correction)
    if unbiased is None:
        return 1
    return 1 if unbiased else 0


@torchsymbol(torch.var, torch.Tensor.var, is_method=True)
def var(a, dim=None, unbiased=None, keepdim: bool = False, *, correction=None):
    if isinstance(dim, builtins.bool):
        unbiased, dim = dim, None
    dims = _dim_list(dim, a.ndim)
    c = _correction(unbiased, correction)
    x = clang.maybe_convert_to_dtype(a, clang.compute_dtype(a.dtype))
    out = prims.var(x, dims, correction=c)
    out = clang.maybe_convert_to_dtype(out, dtypes.corresponding_real_dtype(a.dtype))
    return _restore_keepdim(out, a, dims, keepdim)


@torchsymbol(torch.var_mean)
def var_mean(a, dim=None, unbiased=None, keepdim: bool = False, *, correction=None):
    if isinstance(dim, builtins.bool):
        unbiased, dim = dim, None
    dims = _dim_list(dim, a.ndim)
    c = _correction(unbiased, correction)
    x = clang.maybe_convert_to_dtype(a, clang.compute_dtype(a.dtype))
    v, m = prims.var_mean(x, dims, correction=c)
    v = clang.maybe_convert_to_dtype(v, dtypes.corresponding_real_dtype(a.dtype))
    m = clang.maybe_convert_to_dtype(m, a.dtype)
    return _restore_keepdim(v, a, dims, keepdim), _restore_keepdim(m, a, dims, keepdim)


@torchsymbol(torch.std, torch.Tensor.std, is_method=True)
def std(a, dim=None, unbiased=None, keepdim: bool = False, *, correction=None):
    return sqrt(var(a, dim, unbiased, keepdim, correction=correction))


@torchsymbol(torch.std_mean)
def std_mean(a, dim=None, unbiased=None, keepdim: bool = False, *, correction=None):
    v, m = var_mean(a, dim, unbiased, keepdim, correction=correction)
    return sqrt(v), m


@torchsymbol(torch.amax, torch.Tensor.amax, is_method=True)
def amax(a, dim=(), keepdim: bool = False):
    dims = _dim_list(dim, a.ndim)
    out = prims.amax(a, dims) if a.ndim else a
    return _restore_keepdim(out, a, dims, keepdim)


@torchsymbol(torch.amin, torch.Tensor.amin, is_method=True)
def amin(a, dim=(), keepdim: bool = False):
    dims = _dim_list(dim, a.ndim)
    out = prims.amin(a, dims) if a.ndim else a
    return _restore_keepdim(out, a, dims, keepdim)


@torchsymbol(torch.argmax, torch.Tensor.argmax, is_method=True, tags=(NON_DIFFERENTIABLE_TAG,))
def argmax(a, dim=None, keepdim: bool = False):
    if dim is None:
        out = prims.argmax(flatten(a), 0)
        return clang.reshape(out, (1,) * a.ndim) if keepdim else out
    d = canonicalize_dim(a.ndim, dim)
    return _restore_keepdim(prims.argmax(a, d), a, (d,), keepdim)


@torchsymbol(torch.argmin, torch.Tensor.argmin, is_method=True, tags=(NON_DIFFERENTIABLE_TAG,))
def argmin(a, dim=None, keepdim: bool = False):
    if dim is None:
        out = prims.argmin(flatten(a), 0)
        return clang.reshape(out, (1,) * a.ndim) if keepdim else out
    d = canonicalize_dim(a.ndim, dim)
    return _restore_keepdim(prims.argmin(a, d), a, (d,), keepdim)


@torchsymbol(torch.max, torch.Tensor.max, is_method=True)
def max(a, dim=None, keepdim: bool = False):
    if isinstance(dim, TensorProxy):
        return maximum(a, dim)
    if dim is None:
        return amax(a)
    d = canonicalize_dim(a.ndim, dim)
    values = amax(a, d, keepdim)
    indices = argmax(a, d, keepdim)
    return torch.return_types.max((values, indices))


@torchsymbol(torch.min, torch.Tensor.min, is_method=True)
def min(a, dim=None, keepdim: bool = False):
    if isinstance(dim, TensorProxy):
        return minimum(a, dim)
    if dim is None:
        return amin(a)
    d = canonicalize_dim(a.ndim, dim)
    values = amin(a, d, keepdim)
    indices = argmin(a, d, keepdim)
    return torch.return_types.min((values, indices))


@torchsymbol(torch.all, torch.Tensor.all, is_method=True, tags=(NON_DIFFERENTIABLE_TAG,))
def all(a, dim=None, keepdim: bool = False):
    return logical_not(any(logical_not(_to_bool(a)), dim, keepdim))


@torchsymbol(torch.any, torch.Tensor.any, is_method=True, tags=(NON_DIFFERENTIABLE_TAG,))
def any(a, dim=None, keepdim: bool = False):
    x = clang.maybe_convert_to_dtype(_to_bool(a), torch.int32)
    return clang.ne(amax(x, () if dim is None else dim, keepdim), 0)


@torchsymbol(torch.topk, torch.Tensor.topk, is_method=True)
def topk(a, k, dim=-1, largest=True, sorted=True):
    d = canonicalize_dim(a.ndim, dim)
    v, i = prims.topk(a, pyval(k), d, largest, sorted)
    return torch.return_types.topk((v, i))


@torchsymbol(torch.sort, torch.Tensor.sort, is_method=True)
def sort(a, dim=-1, descending=False, stable=False):
    d = canonicalize_dim(a.ndim, dim)
    v, i = prims.sort(a, d, descending, stable)
    return torch.return_types.sort((v, i))


@torchsymbol(torch.argsort, torch.Tensor.argsort, is_method=True, tags=(NON_DIFFERENTIABLE_TAG,))
def argsort(a, dim=-1, descending=False, stable=False):
    return sort(a, dim, descending, stable)[1]


@torchsymbol(torch.cumsum, torch.Tensor.cumsum, is_method=True)
def cumsum(a, dim, *, dtype=None):
    d = canonicalize_dim(a.ndim, dim)
    rd = _reduction_dtype(a, dtype)
    return prims.cumsum(clang.maybe_convert_to_dtype(a, rd), d)


@torchsymbol(torch.logsumexp, torch.Tensor.logsumexp, is_method=True)
def logsumexp(a, dim, keepdim: bool = False):
    dims = _dim_list(dim, a.ndim)
    x = clang.maybe_convert_to_dtype(a, clang.compute_dtype(a.dtype))
    m = prims.amax(x, dims)
    m_safe = clang.where(clang.isfinite(m), m, 0.0)
    mb = _restore_keepdim(m_safe, a, dims, True)
    s = prims.sum(prims.exp(prims.sub(x, clang.expand(mb, x.shape))), dims)
    out = clang.add(clang.log(s), m_safe)
    return _restore_keepdim(clang.maybe_convert_to_dtype(out, a.dtype), a, dims, keepdim)


@torchsymbol(torch.softmax, torch.Tensor.softmax, *_tfn("nn.functional.softmax", "_softmax"), is_method=True)
def softmax(a, dim, dtype=None, *, _stacklevel=3):
    dim = canonicalize_dim(a.ndim, dim)
    result_dtype = dtype or a.dtype
    x = clang.maybe_convert_to_dtype(a, clang.compute_dtype(result_dtype))
    m = clang.unsqueeze(prims.amax(x, (dim,)), dim)
    e = prims.exp(prims.sub(x, clang.expand(m, x.shape)))
    s = clang.unsqueeze(prims.sum(e, (dim,)), dim)
    out = prims.div(e, clang.expand(s, e.shape))
    return clang.maybe_convert_to_dtype(out, result_dtype)


@torchsymbol(torch.log_softmax, torch.Tensor.log_softmax, *_tfn("nn.functional.log_softmax"), is_method=True)
def log_softmax(a, dim, dtype=None, *, _stacklevel=3):
    dim = canonicalize_dim(a.ndim, dim)
    result_dtype = dtype or a.dtype
    x = clang.maybe_convert_to_dtype(a, clang.compute_dtype(result_dtype))
    m = clang.unsqueeze(prims.amax(x, (dim,)), dim)
    sh = prims.sub(x, clang.expand(m, x.shape))
    lse = clang.unsqueeze(prims.log(prims.sum(prims.exp(sh), (dim,))), dim)
    out = prims.sub(sh, clang.expand(lse, sh.shape))
    return clang.maybe_convert_to_dtype(out, result_dtype)


# =========================================================================================
# Linear algebra
# =========================================================================================
@torchsymbol(torch.matmul, torch.Tensor.matmul, is_method=True)
def matmul(a, b):
    return prims.matmul(a, b)


@torchsymbol(torch.mm, torch.Tensor.mm, is_method=True)
def mm(a, b):
    return prims.matmul(a, b)


@torchsymbol(torch.bmm, torch.Tensor.bmm, is_method=True)
def bmm(a, b):
    return prims.matmul(a, b)


@torchsymbol(torch.baddbmm, torch.Tensor.baddbmm, is_method=True)
def baddbmm(a, b1, b2, *, beta=1, alpha=1):
    out = prims.matmul(b1, b2)
    if alpha != 1:
        out = mul(out, alpha)
    return add(mul(a, beta) if beta != 1 else a, out)


@torchsymbol(torch.addmm, torch.Tensor.addmm, is_method=True)
def addmm(a, m1, m2, *, beta=1, alpha=1):
    out = prims.matmul(m1, m2)
    if alpha != 1:
        out = mul(out, alpha)
    return add(mul(a, beta) if beta != 1 else a, out)


@torchsymbol(torch.nn.functional.linear)
def linear(a, w, bias=None):
    return prims.linear(a, w, bias)


@torchsymbol(*_tfn("_grouped_mm"))
def _grouped_mm(a, b, offs=None, bias=None, out_dtype=None):
    return prims._grouped_mm(a, b, offs)


@torchsymbol(torch.einsum)
def einsum(equation, *operands):
    from .default_torch_ops import opaque_einsum

    if len(operands) == 1 and isinstance(operands[0], (list, tuple)):
        operands = tuple(operands[0])
    return opaque_einsum(equation, *operands)


# =========================================================================================
# NN
# =========================================================================================
@torchsymbol(torch.nn.functional.embedding)
def embedding(a, weight, padding_idx=None, max_norm=None, norm_type=2.0, scale_grad_by_freq=False, sparse=False):
    check(max_norm is None, "embedding: max_norm is not supported")
    padding_idx = -1 if padding_idx is None else padding_idx
    return prims.embedding(a, weight, padding_idx=padding_idx, max_norm=max_norm, norm_type=norm_type,
                           scale_grad_by_freq=scale_grad_by_freq, sparse=sparse)


@torchsymbol(torch.nn.functional.layer_norm)
def layer_norm(a, normalized_shape, weight=None, bias=None, eps: float = 1e-5):
    nd = len(normalized_shape)
    dims = tuple(range(a.ndim - nd, a.ndim))
    x = clang.maybe_convert_to_dtype(a, clang.compute_dtype(a.dtype))
    v, m = prims.var_mean(x, dims, correction=0)
    rstd = prims.rsqrt(prims.add(v, eps))
    shape = tuple(a.shape[: a.ndim - nd]) + (1,) * nd
    y = prims.mul(prims.sub(x, clang.expand(clang.reshape(m, shape), x.shape)), clang.expand(clang.reshape(rstd, shape), x.shape))
    if weight is not None:
        y = clang.mul(y, clang.maybe_convert_to_dtype(weight, y.dtype))
    if bias is not None:
        y = clang.add(y, clang.maybe_convert_to_dtype(bias, y.dtype))
    return clang.maybe_convert_to_dtype(y, a.dtype)


def _rms_norm_torchfns():
    return _tfn("nn.functional.rms_norm", "rms_norm")


@torchsymbol(*_rms_norm_torchfns())
def rms_norm(a, normalized_shape, weight=None, eps: float | None = None):
    """y = a * rsqrt(mean(a^2) + eps) * weight, computed in fp32 (reference :4450-4477)."""
    if eps is None:
        eps = torch.finfo(a.dtype).eps
    nd = len(normalized_shape)
    dims = tuple(range(a.ndim - nd, a.ndim))
    x = clang.maybe_convert_to_dtype(a, clang.compute_dtype(a.dtype))
    n = math.prod(normalized_shape)
    ms = prims.div(prims.sum(prims.mul(x, x), dims), builtins.float(n))
    rstd = prims.rsqrt(prims.add(ms, eps))
    shape = tuple(a.shape[: a.ndim - nd]) + (1,) * nd
    y = prims.mul(x, clang.expand(clang.reshape(rstd, shape), x.shape))
    if weight is not None:
        y = clang.mul(y, clang.maybe_convert_to_dtype(weight, y.dtype))
    return clang.maybe_convert_to_dtype(y, a.dtype)


@torchsymbol(*_tfn("nn.functional.group_norm"))
def group_norm(a, num_groups, weight=None, bias=None, eps=1e-5):
    N, C = a.shape[0], a.shape[1]
    x = reshape(a, (N, num_groups, -1))
    x = clang.maybe_convert_to_dtype(x, clang.compute_dtype(a.dtype))
    v, m = prims.var_mean(x, (2,), correction=0)
    rstd = prims.rsqrt(prims.add(v, eps))
    y = prims.mul(prims.sub(x, clang.expand(clang.unsqueeze(m, 2), x.shape)), clang.expand(clang.unsqueeze(rstd, 2), x.shape))
    y = clang.reshape(y, a.shape)
    wshape = (1, C) + (1,) * (a.ndim - 2)
    if weight is not None:
        y = clang.mul(y, clang.reshape(clang.maybe_convert_to_dtype(weight, y.dtype), wshape))
    if bias is not None:
        y = clang.add(y, clang.reshape(clang.maybe_convert_to_dtype(bias, y.dtype), wshape))
    return clang.maybe_convert_to_dtype(y, a.dtype)


@torchsymbol(torch.nn.functional.dropout)
def dropout(a, p: float = 0.5, training: bool = True, inplace: bool = False):
    p = pyval(p)
    if not training or p == 0.0:
        return a
    if p == 1.0:
        return clang.full_like(a, 0)
    scale = 1.0 / (1.0 - p)
    keep = philox_keep_mask(a, p, *prims.get_rng_seed_offset(_numel(a)))
    compute = clang.compute_dtype(a.dtype)
    x = clang.maybe_convert_to_dtype(a, compute)
    y = prims.mul(prims.mul(x, clang.maybe_convert_to_dtype(keep, compute)), scale)
    return clang.maybe_convert_to_dtype(y, a.dtype)


def _numel(a):
    n = 1
    for d in a.shape:
        n *= d
    return n


def philox_keep_mask(a, p, seed, offset):
    """Dropout keep-mask from the counter-based RNG: a pure function of (seed, offset), so the
    backward recomputes it (fused into its kernel) instead of saving it."""
    r = prims.uniform_philox(tuple(a.shape), 0.0, 1.0, device=a.device, dtype=torch.float32, seed=seed, offset=offset)
    return clang.lt(r, 1.0 - p)


@torchsymbol(*_tfn("nn.functional.scaled_dot_product_attention"))
def scaled_dot_product_attention(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False, *, scale=None, enable_gqa=False):
    """Reference decomposition (reference :6190-6230); the HIP executor claims this op whole."""
    L, S = query.shape[-2], key.shape[-2]
    E = query.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(E)
    if enable_gqa or key.shape[-3] != query.shape[-3]:
        rep = query.shape[-3] // key.shape[-3]
        if rep > 1:
            key = repeat_interleave(key, rep, -3)
            value = repeat_interleave(value, rep, -3)
    logits = mul(matmul(query, transpose(key, -2, -1)), scale)
    if is_causal:
        mask = tril(ones(L, S, dtype=torch.bool, device=query.device))
        logits = masked_fill(logits, logical_not(mask), -math.inf)
    if attn_mask is not None:
        if attn_mask.dtype == torch.bool:
            logits = masked_fill(logits, logical_not(attn_mask), -math.inf)
        else:
            logits = add(logits, attn_mask)
    attn = softmax(logits, -1, dtype=torch.float32)
    attn = clang.maybe_convert_to_dtype(attn, query.dtype)
    if dropout_p > 0.0:
        attn = dropout(attn, dropout_p, True)
    return matmul(attn, value)


def _reduce_loss(loss, reduction, weight_sum=None):
    if reduction == "none":
        return loss
    if reduction == "sum":
        return sum(loss)
    if reduction == "mean":
        if weight_sum is not None:
            return true_divide(sum(loss), weight_sum)
        return mean(loss)
    raise ValueError(f"Unknown reduction {reduction}")


@torchsymbol(torch.nn.functional.nll_loss)
def nll_loss(a, target, weight=None, size_average=None, ignore_index: int = -100, reduce=None, reduction: str = "mean"):
    # a: [N, C] or [N, C, d...] log-probabilities
    if a.ndim == 1:
        a = clang.unsqueeze(a, 0)
        target = clang.unsqueeze(target, 0)
    if a.ndim > 2:
        C = a.shape[1]
        a = reshape(movedim(a, 1, -1), (-1, C))
        target = flatten(target)
    valid = ne(target, ignore_index)
    safe_t = where(valid, target, 0)
    picked = clang.squeeze(clang.take_along_axis(a, clang.unsqueeze(safe_t, 1), 1), (1,))
    w = None
    if weight is not None:
        w = clang.take(weight, safe_t, 0)
        picked = mul(picked, w)
    loss = where(valid, neg(picked), 0.0)
    if reduction == "mean":
        denom = sum(where(valid, w, 0.0)) if w is not None else sum(clang.maybe_convert_to_dtype(valid, a.dtype))
        return true_divide(sum(loss), denom)
    return _reduce_loss(loss, reduction)


@torchsymbol(torch.nn.functional.cross_entropy)
def cross_entropy(a, target, weight=None, size_average=None, ignore_index: int = -100, reduce=None, reduction: str = "mean", label_smoothing: float = 0.0):
    """Softmax cross entropy with class indices (reference :5226); the HIP executor claims it whole."""
    check(dtypes.is_integer_dtype(target.dtype), "cross_entropy: only class-index targets are supported")
    lsm = log_softmax(a, 1 if a.ndim > 1 else 0)
    if label_smoothing == 0.0:
        return nll_loss(lsm, target, weight, ignore_index=ignore_index, reduction=reduction)
    C = a.shape[1] if a.ndim > 1 else a.shape[0]
    nll = nll_loss(lsm, target, weight, ignore_index=ignore_index, reduction="none")
    x = lsm if a.ndim > 1 else clang.unsqueeze(lsm, 0)
    if x.ndim > 2:
        x = reshape(movedim(x, 1, -1), (-1, C))
    valid = flatten(ne(target, ignore_index))
    smooth = neg(sum(x, 1))
    smooth = where(valid, smooth, 0.0)
    loss = add(mul(flatten(nll), 1.0 - label_smoothing), mul(smooth, label_smoothing / C))
    if reduction == "mean":
        return true_divide(sum(loss), sum(clang.maybe_convert_to_dtype(valid, loss.dtype)))
    if reduction == "sum":
        return sum(loss)
    return reshape(loss, target.shape)


@torchsymbol(torch.nn.functional.mse_loss)
def mse_loss(a, target, size_average=None, reduce=None, reduction: str = "mean", weight=None):
    d = sub(a, target)
    sq = mul(d, d)
    if weight is not None:
        sq = mul(sq, weight)
    return _reduce_loss(sq, reduction)


@torchsymbol(torch.nn.functional.l1_loss)
def l1_loss(a, target, size_average=None, reduce=None, reduction: str = "mean"):
    return _reduce_loss(abs(sub(a, target)), reduction)


@torchsymbol(*_tfn("nn.functional.binary_cross_entropy_with_logits"))
def binary_cross_entropy_with_logits(a, target, weight=None, size_average=None, reduce=None, reduction="mean", pos_weight=None):
    log_sig = logsigmoid(a)
    log_1m = logsigmoid(neg(a))
    if pos_weight is not None:
        loss = neg(add(mul(mul(target, pos_weight), log_sig), mul(sub(1, target), log_1m)))
    else:
        loss = neg(add(mul(target, log_sig), mul(sub(1, target), log_1m)))
    if weight is not None:
        loss = mul(loss, weight)
    return _reduce_loss(loss, reduction)


@torchsymbol(*_tfn("nn.functional.normalize"))
def normalize(a, p=2.0, dim=1, eps=1e-12, out=None):
    norm = pow(sum(pow(abs(a), p), dim, True), 1.0 / p)
    return true_divide(a, clamp(norm, min=eps))


@torchsymbol(*_tfn("nn.functional.one_hot"), tags=(NON_DIFFERENTIABLE_TAG,))
def one_hot(a, num_classes=-1):
    check(num_classes > 0, "one_hot requires an explicit num_classes while tracing")
    c = prims.iota(num_classes, start=0, step=1, device=a.device, dtype=torch.int64)
    return clang.maybe_convert_to_dtype(clang.eq(clang.unsqueeze(a, -1), c), torch.int64)


# =========================================================================================
# In-place ops: functionalized into out-of-place + copy_
# =========================================================================================
@torchsymbol(torch.Tensor.copy_, is_method=True)
def copy_(a, b, non_blocking: bool = False):
    if isinstance(b, TensorProxy):
        b = clang.maybe_convert_to_dtype(clang.expand(clang.device_put(b, a.device), a.shape), a.dtype)
    else:
        b = clang.full(a.shape, b, device=a.device, dtype=a.dtype)
    return prims.copy_(b, a)


def _inplace(name, fn, nargs=1):
    def inplace(a, *args, **kwargs):
        out = fn(a, *args, **kwargs)
        if isinstance(out, TensorProxy) and out.dtype != a.dtype:
            out = clang.maybe_convert_to_dtype(out, a.dtype)
        return prims.copy_(out, a)

    inplace.__name__ = name
    tf = getattr(torch.Tensor, name, None)
    sym = torchsymbol(*([tf] if tf is not None else []), is_method=True, id=f"torch.Tensor.{name}")(inplace)
    return sym


add_ = _inplace("add_", add)
sub_ = _inplace("sub_", sub)
mul_ = _inplace("mul_", mul)
div_ = _inplace("div_", div)
pow_ = _inplace("pow_", pow)
clamp_ = _inplace("clamp_", clamp)
masked_fill_ = _inplace("masked_fill_", masked_fill)
exp_ = _inplace("exp_", exp)
neg_ = _inplace("neg_", neg)
sqrt_ = _inplace("sqrt_", sqrt)
tanh_ = _inplace("tanh_", tanh)
sigmoid_ = _inplace("sigmoid_", sigmoid)
relu_ = _inplace("relu_", relu)
addcmul_ = _inplace("addcmul_", addcmul)
addcdiv_ = _inplace("addcdiv_", addcdiv)
lerp_ = _inplace("lerp_", lerp)
index_add_ = _inplace("index_add_", index_add)
scatter_add_ = _inplace("scatter_add_", scatter_add)
index_put_ = _inplace("index_put_", index_put)
tril_ = _inplace("tril_", tril)
triu_ = _inplace("triu_", triu)


@torchsymbol(torch.Tensor.fill_, is_method=True)
def fill_(a, value):
    return prims.copy_(clang.full(a.shape, pyval(value), device=a.device, dtype=a.dtype), a)


@torchsymbol(torch.Tensor.zero_, is_method=True)
def zero_(a):
    return prims.copy_(clang.full(a.shape, 0, device=a.device, dtype=a.dtype), a)


@torchsymbol(torch.Tensor.requires_grad_, is_method=True)
def requires_grad_(a, requires_grad=True):
    return a


# =========================================================================================
# Misc
# =========================================================================================
@torchsymbol(torch.Tensor.item, is_method=True, tags=(NON_DIFFERENTIABLE_TAG,))
def item(a):
    return prims.item(a)


@torchsymbol(*_tfn("polar"))
def polar(abs_, angle):
    from .default_torch_ops import opaque_polar

    return opaque_polar(abs_, angle)


import torch.utils.checkpoint as _tuc  # noqa: E402


@torchsymbol(_tuc.checkpoint, id="torch.checkpoint")
def checkpoint(function, *args, **kwargs):
    """Activation checkpointing: the region's intermediates are recomputed in backward (reference :6348)."""
    from ..core.trace import get_tracectx

    trc = get_tracectx()
    kwargs.pop("use_reentrant", None)
    kwargs.pop("preserve_rng_state", None)
    kwargs.pop("determinism_check", None)
    kwargs.pop("debug", None)
    kwargs.pop("context_fn", None)
    from ..core.jit_ext import user_code_tracing

    with user_code_tracing():
        return function(*args, **kwargs)


# Distributed torch ops are defined in ..distributed.prims and registered there.

from . import default_torch_ops  # noqa: E402,F401  (auto-registration of the long tail)
from . import nn_ops  # noqa: E402,F401  (conv / pooling / normalization / activation decompositions)
from . import more_ops  # noqa: E402,F401  (losses, special functions, products, scans, shape utilities)
