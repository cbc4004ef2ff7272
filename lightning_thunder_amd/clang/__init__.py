"""The core language between prims and user-facing languages (parity: reference ``thunder/clang/__init__.py``
``maybe_convert_to_dtype`` :66-150, ``expand`` :238, ``slice_in_dim`` :279, elementwise wrappers).

Handles broadcasting, torch-style type promotion and the "compute in fp32, store
in the low-precision dtype" convention for elementwise math, so the prims seen by
the HIP fusion code generator are explicit about every cast.
"""
from __future__ import annotations

import math
from enum import Enum, auto
from numbers import Number
from typing import Sequence

import torch

from ..core import dtypes, prims
from ..core.baseutils import check
from ..core.symbolic import SymInt, unify
from ..core.devices import to_device
from ..core.proxies import TensorProxy, NumberProxy, pyval


def clangop(fn):
    fn.__clangop__ = True
    return fn


class ELEMENTWISE_TYPE_PROMOTION_KIND(Enum):
    DEFAULT = auto()
    PRESERVE = auto()
    INT_TO_FLOAT = auto()
    ALWAYS_BOOL = auto()
    COMPLEX_TO_FLOAT = auto()
    BOOL_TO_LONG = auto()
    NO_OPMATH = auto()


def is_tensor(x) -> bool:
    return isinstance(x, TensorProxy)


def canonicalize_dim(rank: int, dim: int, wrap_scalar: bool = True) -> int:
    if rank == 0 and wrap_scalar:
        rank = 1
    check(-rank <= dim < rank, lambda: f"Dimension {dim} out of range for rank {rank}", IndexError)
    return dim + rank if dim < 0 else dim


def canonicalize_dims(rank: int, dims) -> tuple[int, ...]:
    if isinstance(dims, int):
        return (canonicalize_dim(rank, dims),)
    return tuple(canonicalize_dim(rank, d) for d in dims)


def _opmath_dtype(d):
    if d in (torch.bfloat16, torch.float16) or dtypes.is_float8_dtype(d):
        return torch.float32
    if d is torch.complex32:
        return torch.complex64
    return d


_TORCH_KIND = None


def _torch_kind(k):
    from torch._prims_common import ELEMENTWISE_TYPE_PROMOTION_KIND as TK

    return {
        ELEMENTWISE_TYPE_PROMOTION_KIND.DEFAULT: TK.DEFAULT,
        ELEMENTWISE_TYPE_PROMOTION_KIND.PRESERVE: TK.NO_OPMATH,
        ELEMENTWISE_TYPE_PROMOTION_KIND.NO_OPMATH: TK.NO_OPMATH,
        ELEMENTWISE_TYPE_PROMOTION_KIND.INT_TO_FLOAT: TK.INT_TO_FLOAT,
        ELEMENTWISE_TYPE_PROMOTION_KIND.ALWAYS_BOOL: TK.ALWAYS_BOOL,
        ELEMENTWISE_TYPE_PROMOTION_KIND.COMPLEX_TO_FLOAT: TK.COMPLEX_TO_FLOAT,
        ELEMENTWISE_TYPE_PROMOTION_KIND.BOOL_TO_LONG: TK.BOOL_TO_LONG,
    }[k]


_meta_cache: dict = {}


def _meta_stub(a):
    key = (a.dtype, a.ndim == 0)
    t = _meta_cache.get(key)
    if t is None:
        t = torch.empty(() if a.ndim == 0 else (1,), dtype=a.dtype, device="meta")
        _meta_cache[key] = t
    return t


def elementwise_type_promotion(*args, type_promotion_kind: ELEMENTWISE_TYPE_PROMOTION_KIND):
    """Returns (computation_dtype, result_dtype) with exactly torch's semantics.

    Delegates to torch's own promotion table on meta stubs so traced programs
    promote identically to eager PyTorch.
    """
    from torch._prims_common import elementwise_dtypes

    stubs = []
    for a in args:
        if a is None:
            continue
        if isinstance(a, TensorProxy):
            stubs.append(_meta_stub(a))
        elif isinstance(a, NumberProxy):
            stubs.append(a.value if a.value is not None else a.python_type(0))
        elif isinstance(a, SymInt):
            stubs.append(0)  # only the Python type takes part in promotion (an int)
        elif isinstance(a, (Number, torch.Tensor)):
            stubs.append(a)
    return elementwise_dtypes(*stubs, type_promotion_kind=_torch_kind(type_promotion_kind))


@clangop
def maybe_convert_to_dtype(a, dtype, *, enforce_safe_casting: bool = False):
    if a is None:
        return None
    if isinstance(a, TensorProxy):
        if a.dtype == dtype:
            return a
        return prims.convert_element_type(a, dtype)
    if isinstance(a, (Number, NumberProxy)):
        if isinstance(dtype, torch.dtype):
            pt = dtypes.dtype_to_numbertype(dtype)
        else:
            pt = dtype
        if isinstance(a, NumberProxy) and (pt is a.python_type or (pt is float and a.python_type is int)
                                           or (pt is complex and a.python_type in (int, float))):
            return a  # a widening conversion the operation performs itself: the number stays symbolic
        if isinstance(a, SymInt) and pt in (int, float, complex):
            return a  # likewise for a symbolic int (a size argument used as a value)
        v = pyval(a)
        if pt is int and isinstance(v, float):
            return int(v)
        if pt is bool:
            return bool(v)
        if pt is float and isinstance(v, complex):
            return v
        return pt(v) if not (pt is float and isinstance(v, bool)) else float(v)
    if isinstance(a, (list, tuple)):
        return type(a)(maybe_convert_to_dtype(x, dtype) for x in a)
    raise ValueError(f"Cannot convert {a} to {dtype}")


def compute_broadcast_shape(*shapes):
    shapes = [tuple(s) for s in shapes if s is not None]
    if not shapes:
        return None
    ndim = max(len(s) for s in shapes)
    out = [1] * ndim
    for s in shapes:
        off = ndim - len(s)
        for i, d in enumerate(s):
            cur = out[off + i]
            if cur == 1:
                out[off + i] = d
            elif d == 1:
                continue
            elif d == cur:
                out[off + i] = unify(cur, d)
            else:
                raise RuntimeError(f"Shapes {shapes} are not broadcastable")
    return tuple(out)


@clangop
def expand(a, *shape):
    if len(shape) == 1 and isinstance(shape[0], (tuple, list, torch.Size)):
        shape = tuple(shape[0])
    shape = tuple(pyval(s) for s in shape)
    check(len(shape) >= a.ndim, lambda: f"expand: target rank {len(shape)} < {a.ndim}")
    off = len(shape) - a.ndim
    final = []
    for i, s in enumerate(shape):
        if i < off:
            check(s >= 0, "expand: -1 not allowed for new leading dims")
            final.append(s)
        else:
            cur = a.shape[i - off]
            if s == -1:
                final.append(cur)
            else:
                check(cur == 1 or cur == s, lambda: f"expand: cannot expand {a.shape} to {shape}")
                final.append(s if cur == 1 else unify(s, cur))
    final = tuple(final)
    if final == tuple(a.shape):
        return a
    return prims.broadcast_in_dim(a, final, tuple(range(off, len(final))))


@clangop
def maybe_broadcast(*args):
    shapes = [tuple(a.shape) for a in args if isinstance(a, TensorProxy)]
    common = compute_broadcast_shape(*shapes)
    if common is None:
        return args
    out = []
    for a in args:
        if isinstance(a, TensorProxy) and tuple(a.shape) != common:
            out.append(expand(a, common))
        else:
            out.append(a)
    return tuple(out)


def _elementwise_unary(a, prim, kind=ELEMENTWISE_TYPE_PROMOTION_KIND.DEFAULT):
    if not isinstance(a, TensorProxy):
        return prim(pyval(a))
    compute, result = elementwise_type_promotion(a, type_promotion_kind=kind)
    x = maybe_convert_to_dtype(a, compute)
    y = prim(x)
    if isinstance(y, TensorProxy) and y.dtype != result:
        y = maybe_convert_to_dtype(y, result)
    return y


def _elementwise_binary(a, b, prim, kind=ELEMENTWISE_TYPE_PROMOTION_KIND.DEFAULT):
    if not isinstance(a, TensorProxy) and not isinstance(b, TensorProxy):
        return prim(pyval(a), pyval(b))
    compute, result = elementwise_type_promotion(a, b, type_promotion_kind=kind)
    a, b = maybe_broadcast(a, b)
    a = maybe_convert_to_dtype(a, compute)
    b = maybe_convert_to_dtype(b, compute)
    # Numbers stay python numbers of the compute category
    y = prim(a, b)
    if isinstance(y, TensorProxy) and y.dtype != result:
        y = maybe_convert_to_dtype(y, result)
    return y


K = ELEMENTWISE_TYPE_PROMOTION_KIND


def _u(prim, kind=K.DEFAULT):
    @clangop
    def fn(a):
        return _elementwise_unary(a, prim, kind)

    fn.__name__ = prim.name
    return fn


def _b(prim, kind=K.DEFAULT):
    @clangop
    def fn(a, b):
        return _elementwise_binary(a, b, prim, kind)

    fn.__name__ = prim.name
    return fn


abs = _u(prims.abs)
acos = _u(prims.acos, K.INT_TO_FLOAT)
acosh = _u(prims.acosh, K.INT_TO_FLOAT)
asin = _u(prims.asin, K.INT_TO_FLOAT)
asinh = _u(prims.asinh, K.INT_TO_FLOAT)
atan = _u(prims.atan, K.INT_TO_FLOAT)
atanh = _u(prims.atanh, K.INT_TO_FLOAT)
bitwise_not = _u(prims.bitwise_not)
ceil = _u(prims.ceil)
cos = _u(prims.cos, K.INT_TO_FLOAT)
cosh = _u(prims.cosh, K.INT_TO_FLOAT)
digamma = _u(prims.digamma, K.INT_TO_FLOAT)
erf = _u(prims.erf, K.INT_TO_FLOAT)
erfc = _u(prims.erfc, K.INT_TO_FLOAT)
erfinv = _u(prims.erfinv, K.INT_TO_FLOAT)
erfcinv = _u(prims.erfcinv, K.INT_TO_FLOAT)
ndtri = _u(prims.ndtri, K.INT_TO_FLOAT)
exp = _u(prims.exp, K.INT_TO_FLOAT)
exp2 = _u(prims.exp2, K.INT_TO_FLOAT)
expm1 = _u(prims.expm1, K.INT_TO_FLOAT)
floor = _u(prims.floor)
isfinite = _u(prims.isfinite, K.ALWAYS_BOOL)
lgamma = _u(prims.lgamma, K.INT_TO_FLOAT)
log = _u(prims.log, K.INT_TO_FLOAT)
log10 = _u(prims.log10, K.INT_TO_FLOAT)
log1p = _u(prims.log1p, K.INT_TO_FLOAT)
log2 = _u(prims.log2, K.INT_TO_FLOAT)
neg = _u(prims.neg)
reciprocal = _u(prims.reciprocal, K.INT_TO_FLOAT)
round = _u(prims.round)
rsqrt = _u(prims.rsqrt, K.INT_TO_FLOAT)
sign = _u(prims.sign)
signbit = _u(prims.signbit, K.ALWAYS_BOOL)
sin = _u(prims.sin, K.INT_TO_FLOAT)
sinh = _u(prims.sinh, K.INT_TO_FLOAT)
sqrt = _u(prims.sqrt, K.INT_TO_FLOAT)
tan = _u(prims.tan, K.INT_TO_FLOAT)
tanh = _u(prims.tanh, K.INT_TO_FLOAT)
trunc = _u(prims.trunc)

add = _b(prims.add)
atan2 = _b(prims.atan2, K.INT_TO_FLOAT)
bitwise_and = _b(prims.bitwise_and)
bitwise_or = _b(prims.bitwise_or)
bitwise_xor = _b(prims.bitwise_xor)
bitwise_left_shift = _b(prims.bitwise_left_shift)
bitwise_right_shift = _b(prims.bitwise_right_shift)
copysign = _b(prims.copysign, K.INT_TO_FLOAT)
eq = _b(prims.eq, K.ALWAYS_BOOL)
fmod = _b(prims.fmod)
ge = _b(prims.ge, K.ALWAYS_BOOL)
gt = _b(prims.gt, K.ALWAYS_BOOL)
le = _b(prims.le, K.ALWAYS_BOOL)
lt = _b(prims.lt, K.ALWAYS_BOOL)
maximum = _b(prims.maximum)
minimum = _b(prims.minimum)
mul = _b(prims.mul)
ne = _b(prims.ne, K.ALWAYS_BOOL)
nextafter = _b(prims.nextafter)
pow = _b(prims.pow)
remainder = _b(prims.remainder)
sub = _b(prims.sub)
true_divide = _b(prims.div, K.INT_TO_FLOAT)


@clangop
def floor_divide(a, b):
    compute, result = elementwise_type_promotion(a, b, type_promotion_kind=K.DEFAULT)
    if dtypes.is_integer_dtype(result) and not isinstance(a, TensorProxy) and not isinstance(b, TensorProxy):
        return pyval(a) // pyval(b)
    q = _elementwise_binary(a, b, prims.div, K.NO_OPMATH if dtypes.is_integer_dtype(result) else K.DEFAULT)
    if dtypes.is_integer_dtype(result):
        return q  # integer prims.div truncates; torch floors — executors implement integer div as floor division
    return floor(q)


@clangop
def where(pred, a, b):
    compute, result = elementwise_type_promotion(a, b, type_promotion_kind=K.NO_OPMATH)
    pred, a, b = maybe_broadcast(pred, a, b)
    if isinstance(pred, TensorProxy) and pred.dtype != torch.bool:
        pred = prims.ne(pred, 0)
    a = maybe_convert_to_dtype(a, result)
    b = maybe_convert_to_dtype(b, result)
    return prims.where(pred, a, b)


@clangop
def full(shape, fill_value, *, device, dtype):
    return prims.full(tuple(shape), fill_value, device=to_device(device), dtype=dtype)


@clangop
def full_like(a, fill_value, *, device=None, dtype=None):
    return full(a.shape, fill_value, device=device or a.device, dtype=dtype or a.dtype)


@clangop
def reshape(a, shape):
    shape = list(pyval(s) for s in shape)
    numel = math.prod(a.shape)
    if -1 in shape:
        idx = shape.index(-1)
        known = math.prod(s for s in shape if s != -1)
        shape[idx] = numel // known if known != 0 else 0
    shape = tuple(shape)
    if shape == tuple(a.shape):
        return a
    return prims.reshape(a, shape)


@clangop
def squeeze(a, dims=None):
    if dims is None:
        dims = tuple(i for i, s in enumerate(a.shape) if s == 1)
    dims = canonicalize_dims(a.ndim, dims) if a.ndim else ()
    dims = tuple(d for d in dims if a.shape[d] == 1)
    if not dims:
        return a
    return prims.squeeze(a, dims)


@clangop
def unsqueeze(a, dims):
    if isinstance(dims, int):
        dims = (dims,)
    rank = a.ndim + len(dims)
    dims = sorted(canonicalize_dim(rank, d, wrap_scalar=False) for d in dims)
    shape = list(a.shape)
    for d in dims:
        shape.insert(d, 1)
    bdims = [i for i in range(rank) if i not in dims]
    return prims.broadcast_in_dim(a, tuple(shape), tuple(bdims))


@clangop
def transpose(a, permutation):
    permutation = canonicalize_dims(a.ndim, permutation) if a.ndim else ()
    if tuple(permutation) == tuple(range(a.ndim)):
        return a
    return prims.transpose(a, tuple(permutation))


@clangop
def slice_in_dim(a, start, stop, stride=1, dim=0):
    dim = canonicalize_dim(a.ndim, dim)
    starts = [0] * a.ndim
    ends = list(a.shape)
    strides = [1] * a.ndim
    starts[dim] = start
    ends[dim] = stop
    strides[dim] = stride
    if start == 0 and stop == a.shape[dim] and stride == 1:
        return a
    return prims.slice_prim(a, starts, ends, strides)


@clangop
def cat(tensors, dim):
    dim = canonicalize_dim(tensors[0].ndim, dim)
    compute, result = elementwise_type_promotion(*tensors, type_promotion_kind=K.NO_OPMATH)
    tensors = [maybe_convert_to_dtype(t, result) for t in tensors]
    if len(tensors) == 1:
        return tensors[0]
    return prims.cat(list(tensors), dim)


@clangop
def flip(a, dims):
    dims = canonicalize_dims(a.ndim, dims)
    return prims.flip(a, dims)


@clangop
def sum(a, dims, *, output_dtype=None):
    return prims.sum(a, dims, output_dtype=output_dtype) if output_dtype else prims.sum(a, dims)


@clangop
def convert_element_type(a, dtype):
    return maybe_convert_to_dtype(a, dtype)


@clangop
def device_put(a, device):
    device = to_device(device)
    if a.device == device:
        return a
    return prims.device_put(a, device)


@clangop
def iota(length, *, start=0, step=1, device, dtype):
    return prims.iota(length, start=start, step=step, device=to_device(device), dtype=dtype)


@clangop
def uniform(shape, minval=0.0, maxval=1.0, *, device, dtype):
    return prims.uniform(tuple(shape), minval, maxval, device=to_device(device), dtype=dtype)


@clangop
def matmul(a, b):
    return prims.matmul(a, b)


@clangop
def take(a, indices, dim):
    dim = canonicalize_dim(a.ndim, dim)
    return prims.take(a, indices, dim)


@clangop
def take_along_axis(a, indices, dim):
    dim = canonicalize_dim(a.ndim, dim)
    return prims.take_along_axis(a, indices, dim)


@clangop
def compute_dtype(d):
    return _opmath_dtype(d)
