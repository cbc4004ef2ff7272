"""The primitive operation set (parity: reference ``thunder/core/prims.py`` ``PrimIDs`` :94-284,
``OpTags`` :287-308, ``make_prim`` :313).

Prims are the leaves of every decomposition.  Their metas validate inputs and
produce output proxies; executors (torch, the HIP fusion executor, the HIP
kernel executor, python) implement them.  Elementwise prims take same-shape
tensor inputs (broadcasting is explicit via ``broadcast_in_dim``) so the HIP
fusion code generator only has to deal with explicit index maps.
"""
from __future__ import annotations

import math
import operator
from enum import Enum, auto
from numbers import Number
from typing import Sequence

import torch

from . import dtypes
from .baseutils import check
from .codeutils import prettyprint
from .devices import to_device
from .symbolic import SymInt, unify_shapes
from .proxies import Proxy, TensorProxy, NumberProxy, AnyProxy, FutureTensorProxy, pyval, contiguous_strides
from .symbol import Symbol, register_symbol, NON_DIFFERENTIABLE_TAG
from . import proxies as _proxies


class PrimIDs(Enum):
    # utility / prologue
    RETURN = auto()
    DEL = auto()
    COMMENT = auto()
    UNPACK_TRIVIAL = auto()
    UNPACK_SEQUENCE = auto()
    UNPACK_KEY = auto()
    UNPACK_ATTR = auto()
    UNPACK_PARAMETER = auto()
    UNPACK_BUFFER = auto()
    CHECK_TENSOR_SHAPE_AND_METADATA = auto()
    CHECK_NUMBER_TYPE_AND_VALUE = auto()
    CHECK_NUMBER_TYPE = auto()
    CHECK_LEN = auto()
    CHECK_NONE = auto()
    CHECK_STRING_VALUE = auto()
    CHECK_LITERAL_LIKE = auto()
    # data movement
    CONVERT_ELEMENT_TYPE = auto()
    DEVICE_PUT = auto()
    NUMPY_ARRAY_TO_TORCH_TENSOR = auto()
    # creation
    FULL = auto()
    IOTA = auto()
    UNIFORM = auto()
    UNIFORM_PHILOX = auto()
    GET_RNG_SEED_OFFSET = auto()
    RANDN = auto()
    EMPTY = auto()
    TENSOR_FROM_SEQUENCE = auto()
    # shape
    BROADCAST_IN_DIM = auto()
    CAT = auto()
    FLIP = auto()
    PAD = auto()
    RESHAPE = auto()
    SLICE = auto()
    SQUEEZE = auto()
    TRANSPOSE = auto()
    TAKE = auto()
    TAKE_ALONG_AXIS = auto()
    INDEX_ADD = auto()
    INDEX_PUT = auto()
    SCATTER_ADD = auto()
    SCATTER = auto()
    # elementwise unary
    ABS = auto()
    ACOS = auto()
    ACOSH = auto()
    ASIN = auto()
    ASINH = auto()
    ATAN = auto()
    ATANH = auto()
    BITWISE_NOT = auto()
    CEIL = auto()
    COS = auto()
    COSH = auto()
    DIGAMMA = auto()
    ERF = auto()
    ERFC = auto()
    ERFINV = auto()
    ERFCINV = auto()
    NDTRI = auto()
    EXP = auto()
    EXP2 = auto()
    EXPM1 = auto()
    FLOOR = auto()
    ISFINITE = auto()
    LGAMMA = auto()
    LOG = auto()
    LOG10 = auto()
    LOG1P = auto()
    LOG2 = auto()
    NEG = auto()
    RECIPROCAL = auto()
    ROUND = auto()
    RSQRT = auto()
    SIGN = auto()
    SIGNBIT = auto()
    SIN = auto()
    SINH = auto()
    SQRT = auto()
    TAN = auto()
    TANH = auto()
    TRUNC = auto()
    REAL = auto()
    IMAG = auto()
    # elementwise binary
    ADD = auto()
    ATAN2 = auto()
    BITWISE_AND = auto()
    BITWISE_OR = auto()
    BITWISE_XOR = auto()
    BITWISE_LEFT_SHIFT = auto()
    BITWISE_RIGHT_SHIFT = auto()
    COPYSIGN = auto()
    DIV = auto()
    EQ = auto()
    FMOD = auto()
    GE = auto()
    GT = auto()
    LE = auto()
    LT = auto()
    MAXIMUM = auto()
    MINIMUM = auto()
    MUL = auto()
    NE = auto()
    NEXTAFTER = auto()
    POW = auto()
    REMAINDER = auto()
    SUB = auto()
    ZETA = auto()
    # ternary
    WHERE = auto()
    # reductions
    AMAX = auto()
    AMIN = auto()
    PROD = auto()
    SUM = auto()
    VAR = auto()
    VAR_MEAN = auto()
    ARGMAX = auto()
    ARGMIN = auto()
    TOPK = auto()
    SORT = auto()
    CUMSUM = auto()
    # linear algebra / nn
    MATMUL = auto()
    LINEAR = auto()
    GROUPED_MM = auto()
    EMBEDDING = auto()
    EMBEDDING_BACKWARD = auto()
    CONVOLUTION = auto()
    # memory
    COPY_ = auto()
    ITEM = auto()
    BITCAST = auto()
    SHALLOW_COPY = auto()


class OpTags(Enum):
    REDUCTION_OP = auto()
    RANDOM_OP = auto()
    SHAPE_OP = auto()
    MATMUL_OP = auto()
    DONT_DCE = auto()
    IN_PLACE = auto()
    DEVICE_SYNC_OP = auto()
    AUTO_REGISTERED = auto()
    DONT_AUTO_RECOMPUTE_IN_BACKWARD = auto()
    CTX_MANAGER_ENTER_EXIT_OP = auto()
    ELEMENTWISE = auto()


import sys as _sys

_this_module = _sys.modules[__name__]


def make_prim(id, name, *, meta, tags=(), python_printer=None, python_impl=None, print_as=None):
    sym = Symbol(
        name,
        meta,
        id=id,
        is_prim=True,
        tags=tags,
        module=_this_module,
        python_printer=python_printer,
        python_impl=python_impl,
        print_as=print_as,
    )
    register_symbol(sym)
    return sym


# -----------------------------------------------------------------------------------------
# Utility prims
# -----------------------------------------------------------------------------------------
def _return_meta(*args):
    return None


def _return_printer(bsym, obj_ctx):
    if len(bsym.args) == 1:
        return f"return {prettyprint(bsym.args[0], obj_ctx)}"
    return "return " + prettyprint(tuple(bsym.args), obj_ctx)


python_return = make_prim(PrimIDs.RETURN, "python_return", meta=_return_meta, python_printer=_return_printer, tags=(OpTags.DONT_DCE,))


def _del_printer(bsym, obj_ctx):
    names = [a.name for a in bsym.args if isinstance(a, Proxy)]
    return f"del {', '.join(names)}" if names else "pass"


python_del = make_prim(PrimIDs.DEL, "python_del", meta=_return_meta, python_printer=_del_printer, tags=(OpTags.DONT_DCE,))


def _comment_printer(bsym, obj_ctx):
    return "# " + str(bsym.args[0])


comment = make_prim(PrimIDs.COMMENT, "comment", meta=_return_meta, python_printer=_comment_printer, tags=(OpTags.DONT_DCE,))


def _unpack_trivial_meta(x, *, name=None):
    return x


def _unpack_trivial_printer(bsym, obj_ctx):
    return f"# {bsym.output.name} (unpacked trivially)" if isinstance(bsym.output, Proxy) else "pass"


unpack_trivial = make_prim(PrimIDs.UNPACK_TRIVIAL, "unpack_trivial", meta=_unpack_trivial_meta, python_printer=_unpack_trivial_printer)


def _check_tensor_meta(t, shape, device, dtype, requires_grad):
    return None


check_tensor_shape_and_metadata = make_prim(
    PrimIDs.CHECK_TENSOR_SHAPE_AND_METADATA,
    "check_tensor_shape_and_metadata",
    meta=_check_tensor_meta,
    tags=(OpTags.DONT_DCE,),
)
check_number_type_and_value = make_prim(
    PrimIDs.CHECK_NUMBER_TYPE_AND_VALUE, "check_number_type_and_value", meta=lambda n, v: None, tags=(OpTags.DONT_DCE,)
)
check_number_type = make_prim(
    PrimIDs.CHECK_NUMBER_TYPE, "check_number_type", meta=lambda n, typ: None, tags=(OpTags.DONT_DCE,)
)  # symbolic-values inputs: only the Python type is part of the cache key
check_len = make_prim(PrimIDs.CHECK_LEN, "check_len", meta=lambda x, n: None, tags=(OpTags.DONT_DCE,))
check_none = make_prim(PrimIDs.CHECK_NONE, "check_none", meta=lambda x: None, tags=(OpTags.DONT_DCE,))
check_string_value = make_prim(PrimIDs.CHECK_STRING_VALUE, "check_string_value", meta=lambda s, v: None, tags=(OpTags.DONT_DCE,))
check_literal_like = make_prim(PrimIDs.CHECK_LITERAL_LIKE, "check_literal_like", meta=lambda x, v: None, tags=(OpTags.DONT_DCE,))


def _unpack_sequence_meta(x, n):
    return [_proxies.AnyProxy(None) for _ in range(n)]


unpack_sequence = make_prim(PrimIDs.UNPACK_SEQUENCE, "unpack_sequence", meta=_unpack_sequence_meta)
unpack_key = make_prim(PrimIDs.UNPACK_KEY, "unpack_key", meta=lambda d, key: _proxies.AnyProxy(None))
unpack_attr = make_prim(PrimIDs.UNPACK_ATTR, "unpack_attr", meta=lambda obj, name: _proxies.AnyProxy(None))
unpack_parameter = make_prim(PrimIDs.UNPACK_PARAMETER, "unpack_parameter", meta=lambda obj, name: _proxies.AnyProxy(None))
unpack_buffer = make_prim(PrimIDs.UNPACK_BUFFER, "unpack_buffer", meta=lambda obj, name: _proxies.AnyProxy(None))


# -----------------------------------------------------------------------------------------
# Helpers for metas
# -----------------------------------------------------------------------------------------
def _tensor_args(*args):
    return [a for a in args if isinstance(a, TensorProxy)]


def _check_same_shape(*args):
    ts = _tensor_args(*args)
    if not ts:
        return None
    shape = ts[0].shape
    for t in ts[1:]:
        check(t.shape == shape, lambda: f"Expected same shape, got {shape} and {t.shape}")
        shape = unify_shapes(shape, t.shape)
    return shape


def _check_same_device(*args):
    ts = _tensor_args(*args)
    if not ts:
        return None
    d = ts[0].device
    for t in ts[1:]:
        # cpu scalars (0-dim) may mix with gpu tensors
        if t.device != d and t.ndim != 0 and ts[0].ndim != 0:
            raise RuntimeError(f"Expected all tensors on the same device, got {d} and {t.device}")
    gpu = [t.device for t in ts if t.device.type != "cpu"]
    return gpu[0] if gpu else d


def _check_same_dtype(*args):
    ts = _tensor_args(*args)
    if not ts:
        return None
    d = ts[0].dtype
    for t in ts[1:]:
        check(t.dtype == d, lambda: f"Expected same dtype, got {d} and {t.dtype}")
    return d


class ELEMENTWISE_PRIM_OUTPUT_DTYPE_KIND(Enum):
    SAME = auto()
    ALWAYS_BOOL = auto()
    COMPLEX_TO_FLOAT = auto()


_unary_python = {
    PrimIDs.ABS: abs,
    PrimIDs.NEG: operator.neg,
    PrimIDs.EXP: math.exp,
    PrimIDs.LOG: math.log,
    PrimIDs.SQRT: math.sqrt,
    PrimIDs.SIN: math.sin,
    PrimIDs.COS: math.cos,
    PrimIDs.TANH: math.tanh,
    PrimIDs.FLOOR: math.floor,
    PrimIDs.CEIL: math.ceil,
    PrimIDs.TRUNC: math.trunc,
    PrimIDs.RECIPROCAL: lambda x: 1.0 / x,
    PrimIDs.RSQRT: lambda x: 1.0 / math.sqrt(x),
    PrimIDs.ERF: math.erf,
    PrimIDs.ERFC: math.erfc,
    PrimIDs.EXP2: lambda x: 2.0**x,
    PrimIDs.EXPM1: math.expm1,
    PrimIDs.LOG1P: math.log1p,
    PrimIDs.LOG2: math.log2,
    PrimIDs.LOG10: math.log10,
}


def _make_unary(id, name, kind=ELEMENTWISE_PRIM_OUTPUT_DTYPE_KIND.SAME, supported=None):
    def meta(a):
        if isinstance(a, TensorProxy):
            dtype = a.dtype
            if kind is ELEMENTWISE_PRIM_OUTPUT_DTYPE_KIND.ALWAYS_BOOL:
                dtype = torch.bool
            elif kind is ELEMENTWISE_PRIM_OUTPUT_DTYPE_KIND.COMPLEX_TO_FLOAT:
                dtype = dtypes.corresponding_real_dtype(dtype)
            return TensorProxy(like=a, dtype=dtype, requires_grad=False)
        # pure number: evaluate in python
        fn = _unary_python.get(id)
        check(fn is not None, lambda: f"prim {name} on a python number is not supported")
        return fn(pyval(a))

    return make_prim(id, name, meta=meta, tags=(OpTags.ELEMENTWISE,))


abs = _make_unary(PrimIDs.ABS, "abs")
acos = _make_unary(PrimIDs.ACOS, "acos")
acosh = _make_unary(PrimIDs.ACOSH, "acosh")
asin = _make_unary(PrimIDs.ASIN, "asin")
asinh = _make_unary(PrimIDs.ASINH, "asinh")
atan = _make_unary(PrimIDs.ATAN, "atan")
atanh = _make_unary(PrimIDs.ATANH, "atanh")
bitwise_not = _make_unary(PrimIDs.BITWISE_NOT, "bitwise_not")
ceil = _make_unary(PrimIDs.CEIL, "ceil")
cos = _make_unary(PrimIDs.COS, "cos")
cosh = _make_unary(PrimIDs.COSH, "cosh")
digamma = _make_unary(PrimIDs.DIGAMMA, "digamma")
erf = _make_unary(PrimIDs.ERF, "erf")
erfc = _make_unary(PrimIDs.ERFC, "erfc")
erfinv = _make_unary(PrimIDs.ERFINV, "erfinv")
erfcinv = _make_unary(PrimIDs.ERFCINV, "erfcinv")
ndtri = _make_unary(PrimIDs.NDTRI, "ndtri")
exp = _make_unary(PrimIDs.EXP, "exp")
exp2 = _make_unary(PrimIDs.EXP2, "exp2")
expm1 = _make_unary(PrimIDs.EXPM1, "expm1")
floor = _make_unary(PrimIDs.FLOOR, "floor")
isfinite = _make_unary(PrimIDs.ISFINITE, "isfinite", ELEMENTWISE_PRIM_OUTPUT_DTYPE_KIND.ALWAYS_BOOL)
lgamma = _make_unary(PrimIDs.LGAMMA, "lgamma")
log = _make_unary(PrimIDs.LOG, "log")
log10 = _make_unary(PrimIDs.LOG10, "log10")
log1p = _make_unary(PrimIDs.LOG1P, "log1p")
log2 = _make_unary(PrimIDs.LOG2, "log2")
neg = _make_unary(PrimIDs.NEG, "neg")
reciprocal = _make_unary(PrimIDs.RECIPROCAL, "reciprocal")
round = _make_unary(PrimIDs.ROUND, "round")
rsqrt = _make_unary(PrimIDs.RSQRT, "rsqrt")
sign = _make_unary(PrimIDs.SIGN, "sign")
signbit = _make_unary(PrimIDs.SIGNBIT, "signbit", ELEMENTWISE_PRIM_OUTPUT_DTYPE_KIND.ALWAYS_BOOL)
sin = _make_unary(PrimIDs.SIN, "sin")
sinh = _make_unary(PrimIDs.SINH, "sinh")
sqrt = _make_unary(PrimIDs.SQRT, "sqrt")
tan = _make_unary(PrimIDs.TAN, "tan")
tanh = _make_unary(PrimIDs.TANH, "tanh")
trunc = _make_unary(PrimIDs.TRUNC, "trunc")
real = _make_unary(PrimIDs.REAL, "real", ELEMENTWISE_PRIM_OUTPUT_DTYPE_KIND.COMPLEX_TO_FLOAT)
imag = _make_unary(PrimIDs.IMAG, "imag", ELEMENTWISE_PRIM_OUTPUT_DTYPE_KIND.COMPLEX_TO_FLOAT)

_binary_python = {
    PrimIDs.ADD: operator.add,
    PrimIDs.SUB: operator.sub,
    PrimIDs.MUL: operator.mul,
    PrimIDs.DIV: operator.truediv,
    PrimIDs.POW: operator.pow,
    PrimIDs.EQ: operator.eq,
    PrimIDs.NE: operator.ne,
    PrimIDs.LT: operator.lt,
    PrimIDs.LE: operator.le,
    PrimIDs.GT: operator.gt,
    PrimIDs.GE: operator.ge,
    PrimIDs.MAXIMUM: max,
    PrimIDs.MINIMUM: min,
    PrimIDs.BITWISE_AND: operator.and_,
    PrimIDs.BITWISE_OR: operator.or_,
    PrimIDs.BITWISE_XOR: operator.xor,
    PrimIDs.REMAINDER: operator.mod,
    PrimIDs.FMOD: math.fmod,
    PrimIDs.ATAN2: math.atan2,
}


def _make_binary(id, name, kind=ELEMENTWISE_PRIM_OUTPUT_DTYPE_KIND.SAME):
    def meta(a, b):
        ts = _tensor_args(a, b)
        if not ts:
            fn = _binary_python.get(id)
            check(fn is not None, lambda: f"prim {name} on python numbers is not supported")
            return fn(pyval(a), pyval(b))
        shape = _check_same_shape(a, b)
        device = _check_same_device(a, b)
        dtype = _check_same_dtype(a, b)
        if kind is ELEMENTWISE_PRIM_OUTPUT_DTYPE_KIND.ALWAYS_BOOL:
            dtype = torch.bool
        return TensorProxy(shape=shape, device=device, dtype=dtype, requires_grad=False)

    return make_prim(id, name, meta=meta, tags=(OpTags.ELEMENTWISE,))


add = _make_binary(PrimIDs.ADD, "add")
atan2 = _make_binary(PrimIDs.ATAN2, "atan2")
bitwise_and = _make_binary(PrimIDs.BITWISE_AND, "bitwise_and")
bitwise_or = _make_binary(PrimIDs.BITWISE_OR, "bitwise_or")
bitwise_xor = _make_binary(PrimIDs.BITWISE_XOR, "bitwise_xor")
bitwise_left_shift = _make_binary(PrimIDs.BITWISE_LEFT_SHIFT, "bitwise_left_shift")
bitwise_right_shift = _make_binary(PrimIDs.BITWISE_RIGHT_SHIFT, "bitwise_right_shift")
copysign = _make_binary(PrimIDs.COPYSIGN, "copysign")
div = _make_binary(PrimIDs.DIV, "div")
eq = _make_binary(PrimIDs.EQ, "eq", ELEMENTWISE_PRIM_OUTPUT_DTYPE_KIND.ALWAYS_BOOL)
fmod = _make_binary(PrimIDs.FMOD, "fmod")
ge = _make_binary(PrimIDs.GE, "ge", ELEMENTWISE_PRIM_OUTPUT_DTYPE_KIND.ALWAYS_BOOL)
gt = _make_binary(PrimIDs.GT, "gt", ELEMENTWISE_PRIM_OUTPUT_DTYPE_KIND.ALWAYS_BOOL)
le = _make_binary(PrimIDs.LE, "le", ELEMENTWISE_PRIM_OUTPUT_DTYPE_KIND.ALWAYS_BOOL)
lt = _make_binary(PrimIDs.LT, "lt", ELEMENTWISE_PRIM_OUTPUT_DTYPE_KIND.ALWAYS_BOOL)
maximum = _make_binary(PrimIDs.MAXIMUM, "maximum")
minimum = _make_binary(PrimIDs.MINIMUM, "minimum")
mul = _make_binary(PrimIDs.MUL, "mul")
ne = _make_binary(PrimIDs.NE, "ne", ELEMENTWISE_PRIM_OUTPUT_DTYPE_KIND.ALWAYS_BOOL)
nextafter = _make_binary(PrimIDs.NEXTAFTER, "nextafter")
pow = _make_binary(PrimIDs.POW, "pow")
remainder = _make_binary(PrimIDs.REMAINDER, "remainder")
sub = _make_binary(PrimIDs.SUB, "sub")
zeta = _make_binary(PrimIDs.ZETA, "zeta")


def _where_meta(pred, a, b):
    ts = _tensor_args(pred, a, b)
    check(len(ts) > 0, "where expects at least one tensor")
    shape = _check_same_shape(pred, a, b)
    device = _check_same_device(pred, a, b)
    if isinstance(pred, TensorProxy):
        check(pred.dtype == torch.bool, lambda: f"where predicate must be bool, got {pred.dtype}")
    dtype = _check_same_dtype(a, b)
    if dtype is None:
        dtype = dtypes.to_torch_dtype(dtypes.to_dtype(a))
    return TensorProxy(shape=shape, device=device, dtype=dtype)


where = make_prim(PrimIDs.WHERE, "where", meta=_where_meta, tags=(OpTags.ELEMENTWISE,))


# -----------------------------------------------------------------------------------------
# Data movement
# -----------------------------------------------------------------------------------------
def _convert_element_type_meta(a, dtype):
    if isinstance(a, TensorProxy):
        return TensorProxy(like=a, dtype=dtype, requires_grad=a.requires_grad and dtypes.is_inexact_dtype(dtype))
    v = pyval(a)
    pt = dtypes.dtype_to_numbertype(dtype)
    return pt(v)


convert_element_type = make_prim(
    PrimIDs.CONVERT_ELEMENT_TYPE, "convert_element_type", meta=_convert_element_type_meta, tags=(OpTags.ELEMENTWISE,)
)


def _device_put_meta(a, device):
    return TensorProxy(like=a, device=to_device(device))


device_put = make_prim(PrimIDs.DEVICE_PUT, "device_put", meta=_device_put_meta)


def _bitcast_meta(a, dtype):
    check(dtypes.itemsize(a.dtype) == dtypes.itemsize(dtype), "bitcast requires equal item sizes")
    return TensorProxy(like=a, dtype=dtype, requires_grad=False)


bitcast = make_prim(PrimIDs.BITCAST, "bitcast", meta=_bitcast_meta, tags=(NON_DIFFERENTIABLE_TAG,))


# -----------------------------------------------------------------------------------------
# Creation
# -----------------------------------------------------------------------------------------
def _full_meta(shape, fill_value, *, device, dtype):
    return TensorProxy(shape=tuple(shape), device=to_device(device), dtype=dtype, requires_grad=False)


full = make_prim(PrimIDs.FULL, "full", meta=_full_meta)


def _iota_meta(length, *, start, step, device, dtype):
    n = length if isinstance(length, SymInt) else int(length)
    return TensorProxy(shape=(n,), device=to_device(device), dtype=dtype, requires_grad=False)


iota = make_prim(PrimIDs.IOTA, "iota", meta=_iota_meta)


def _uniform_meta(shape, minval, maxval, *, device, dtype):
    return TensorProxy(shape=tuple(shape), device=to_device(device), dtype=dtype, requires_grad=False)


uniform = make_prim(PrimIDs.UNIFORM, "uniform", meta=_uniform_meta, tags=(OpTags.RANDOM_OP,))


def _uniform_philox_meta(shape, minval, maxval, *, device, dtype, seed, offset):
    return TensorProxy(shape=tuple(shape), device=to_device(device), dtype=dtype, requires_grad=False)


uniform_philox = make_prim(PrimIDs.UNIFORM_PHILOX, "uniform_philox", meta=_uniform_philox_meta)


def _get_rng_seed_offset_meta(numel):
    return _proxies.IntegerProxy(None), _proxies.IntegerProxy(None)


# advances the framework's Philox counter (a side effect: never CSE'd or DCE'd, a fusion barrier)
get_rng_seed_offset = make_prim(PrimIDs.GET_RNG_SEED_OFFSET, "get_rng_seed_offset", meta=_get_rng_seed_offset_meta,
                                tags=(OpTags.DONT_DCE, OpTags.RANDOM_OP))


def _randn_meta(shape, *, device, dtype):
    return TensorProxy(shape=tuple(shape), device=to_device(device), dtype=dtype, requires_grad=False)


randn = make_prim(PrimIDs.RANDN, "randn", meta=_randn_meta, tags=(OpTags.RANDOM_OP,))


def _empty_meta(shape, *, device, dtype):
    return TensorProxy(shape=tuple(shape), device=to_device(device), dtype=dtype, requires_grad=False)


empty = make_prim(PrimIDs.EMPTY, "empty", meta=_empty_meta)


def _tensor_from_sequence_meta(seq, *, dtype, device):
    t = torch.tensor(seq, dtype=dtype, device="meta")
    return TensorProxy(shape=tuple(t.shape), device=to_device(device), dtype=t.dtype)


tensor_from_sequence = make_prim(PrimIDs.TENSOR_FROM_SEQUENCE, "tensor_from_sequence", meta=_tensor_from_sequence_meta)


# -----------------------------------------------------------------------------------------
# Shape ops
# -----------------------------------------------------------------------------------------
def _broadcast_in_dim_meta(a, shape, broadcast_dimensions):
    shape = tuple(s if isinstance(s, SymInt) else int(s) for s in shape)
    check(len(broadcast_dimensions) == a.ndim, lambda: f"broadcast_in_dim: {broadcast_dimensions} vs ndim {a.ndim}")
    for i, d in enumerate(broadcast_dimensions):
        check(a.shape[i] == shape[d] or a.shape[i] == 1, lambda: f"Cannot broadcast {a.shape} to {shape}")
    return TensorProxy(like=a, shape=shape)


broadcast_in_dim = make_prim(PrimIDs.BROADCAST_IN_DIM, "broadcast_in_dim", meta=_broadcast_in_dim_meta, tags=(OpTags.SHAPE_OP,))


def _cat_meta(tensors, dim):
    check(len(tensors) > 0, "cat expects at least one tensor")
    t0 = tensors[0]
    shape = list(t0.shape)
    total = 0
    for t in tensors:
        check(t.ndim == t0.ndim, "cat: tensors must have the same rank")
        for i in range(t.ndim):
            if i != dim:
                check(t.shape[i] == shape[i], lambda: f"cat: shape mismatch {t.shape} vs {t0.shape}")
        total += t.shape[dim]
    shape[dim] = total
    dtype = _check_same_dtype(*tensors)
    return TensorProxy(like=t0, shape=tuple(shape), dtype=dtype)


cat = make_prim(PrimIDs.CAT, "cat", meta=_cat_meta)


def _flip_meta(a, dims):
    return TensorProxy(like=a)


flip = make_prim(PrimIDs.FLIP, "flip", meta=_flip_meta, tags=(OpTags.SHAPE_OP,))


def _pad_meta(a, padding_value, padding_config):
    shape = []
    for s, (lo, hi, interior) in zip(a.shape, padding_config):
        shape.append(lo + hi + s + max(s - 1, 0) * interior)
    return TensorProxy(like=a, shape=tuple(shape))


pad = make_prim(PrimIDs.PAD, "pad", meta=_pad_meta)


def _reshape_meta(a, shape):
    shape = tuple(s if isinstance(s, SymInt) else int(s) for s in shape)
    check(math.prod(shape) == math.prod(a.shape), lambda: f"Cannot reshape {a.shape} to {shape}")
    return TensorProxy(like=a, shape=shape)


reshape = make_prim(PrimIDs.RESHAPE, "reshape", meta=_reshape_meta, tags=(OpTags.SHAPE_OP,))


def _slice_meta(a, start_indices, end_indices, strides=None):
    if strides is None:
        strides = [1] * a.ndim
    shape = []
    for s, e, st, l in zip(start_indices, end_indices, strides, a.shape):
        check(0 <= s <= e <= l, lambda: f"slice: invalid bounds {start_indices}, {end_indices} for {a.shape}")
        shape.append((e - s + st - 1) // st)
    return TensorProxy(like=a, shape=tuple(shape))


slice_prim = make_prim(PrimIDs.SLICE, "slice_prim", meta=_slice_meta, tags=(OpTags.SHAPE_OP,))


def _squeeze_meta(a, dims):
    dims = tuple(dims)
    shape = tuple(s for i, s in enumerate(a.shape) if i not in dims)
    for d in dims:
        check(a.shape[d] == 1, lambda: f"squeeze: dim {d} of {a.shape} is not 1")
    return TensorProxy(like=a, shape=shape)


squeeze = make_prim(PrimIDs.SQUEEZE, "squeeze", meta=_squeeze_meta, tags=(OpTags.SHAPE_OP,))


def _transpose_meta(a, permutation):
    check(sorted(permutation) == list(range(a.ndim)), lambda: f"transpose: invalid permutation {permutation}")
    return TensorProxy(like=a, shape=tuple(a.shape[p] for p in permutation))


transpose = make_prim(PrimIDs.TRANSPOSE, "transpose", meta=_transpose_meta, tags=(OpTags.SHAPE_OP,))


def _take_meta(a, indices, dim):
    shape = list(a.shape)
    shape[dim:dim + 1] = list(indices.shape)
    return TensorProxy(like=a, shape=tuple(shape))


take = make_prim(PrimIDs.TAKE, "take", meta=_take_meta)


def _take_along_axis_meta(a, indices, dim):
    return TensorProxy(like=a, shape=tuple(indices.shape))


take_along_axis = make_prim(PrimIDs.TAKE_ALONG_AXIS, "take_along_axis", meta=_take_along_axis_meta)


def _index_add_meta(a, indices, value, dim):
    return TensorProxy(like=a)


index_add = make_prim(PrimIDs.INDEX_ADD, "index_add", meta=_index_add_meta)


def _index_put_meta(a, indices, values, accumulate):
    return TensorProxy(like=a)


index_put = make_prim(PrimIDs.INDEX_PUT, "index_put", meta=_index_put_meta)


def _scatter_add_meta(a, index, value, dim):
    return TensorProxy(like=a)


scatter_add = make_prim(PrimIDs.SCATTER_ADD, "scatter_add", meta=_scatter_add_meta)


def _scatter_meta(a, index, src, dim):
    return TensorProxy(like=a)


scatter = make_prim(PrimIDs.SCATTER, "scatter", meta=_scatter_meta)


# -----------------------------------------------------------------------------------------
# Reductions
# -----------------------------------------------------------------------------------------
def _reduced_shape(shape, dims):
    return tuple(s for i, s in enumerate(shape) if i not in dims)


def _reduction_meta(a, dims, *, output_dtype=None):
    dims = tuple(sorted(dims))
    for d in dims:
        check(0 <= d < max(a.ndim, 1), lambda: f"reduction dim {d} out of range for {a.shape}")
    return TensorProxy(like=a, shape=_reduced_shape(a.shape, dims), dtype=output_dtype or a.dtype)


amax = make_prim(PrimIDs.AMAX, "amax", meta=_reduction_meta, tags=(OpTags.REDUCTION_OP,))
amin = make_prim(PrimIDs.AMIN, "amin", meta=_reduction_meta, tags=(OpTags.REDUCTION_OP,))
prod = make_prim(PrimIDs.PROD, "prod", meta=_reduction_meta, tags=(OpTags.REDUCTION_OP,))
sum = make_prim(PrimIDs.SUM, "sum", meta=_reduction_meta, tags=(OpTags.REDUCTION_OP,))


def _var_meta(a, dims, *, correction):
    dims = tuple(sorted(dims))
    return TensorProxy(like=a, shape=_reduced_shape(a.shape, dims), dtype=dtypes.corresponding_real_dtype(a.dtype))


var = make_prim(PrimIDs.VAR, "var", meta=_var_meta, tags=(OpTags.REDUCTION_OP,))


def _var_mean_meta(a, dims, *, correction):
    dims = tuple(sorted(dims))
    shape = _reduced_shape(a.shape, dims)
    v = TensorProxy(like=a, shape=shape, dtype=dtypes.corresponding_real_dtype(a.dtype))
    m = TensorProxy(like=a, shape=shape)
    return v, m


var_mean = make_prim(PrimIDs.VAR_MEAN, "var_mean", meta=_var_mean_meta, tags=(OpTags.REDUCTION_OP,))


def _argmax_meta(a, dim):
    shape = () if dim is None else _reduced_shape(a.shape, (dim,))
    return TensorProxy(like=a, shape=shape, dtype=torch.int64, requires_grad=False)


argmax = make_prim(PrimIDs.ARGMAX, "argmax", meta=_argmax_meta, tags=(OpTags.REDUCTION_OP, NON_DIFFERENTIABLE_TAG))
argmin = make_prim(PrimIDs.ARGMIN, "argmin", meta=_argmax_meta, tags=(OpTags.REDUCTION_OP, NON_DIFFERENTIABLE_TAG))


def _topk_meta(a, k, dim, largest, sorted):
    shape = list(a.shape)
    shape[dim] = k
    return TensorProxy(like=a, shape=tuple(shape)), TensorProxy(like=a, shape=tuple(shape), dtype=torch.int64, requires_grad=False)


topk = make_prim(PrimIDs.TOPK, "topk", meta=_topk_meta, tags=(OpTags.REDUCTION_OP,))


def _sort_meta(a, dim, descending, stable):
    return TensorProxy(like=a), TensorProxy(like=a, dtype=torch.int64, requires_grad=False)


sort = make_prim(PrimIDs.SORT, "sort", meta=_sort_meta)


def _cumsum_meta(a, dim, *, dtype=None):
    return TensorProxy(like=a, dtype=dtype or a.dtype)


cumsum = make_prim(PrimIDs.CUMSUM, "cumsum", meta=_cumsum_meta)


# -----------------------------------------------------------------------------------------
# Linear algebra / NN
# -----------------------------------------------------------------------------------------
def _matmul_meta(a, b):
    # torch.matmul's shape rules written out (a meta-device call would turn symbolic dims into ints)
    check(a.ndim >= 1 and b.ndim >= 1, "matmul: both arguments need at least one dimension")
    check(a.dtype == b.dtype, lambda: f"matmul: dtype mismatch {a.dtype} vs {b.dtype}")
    device = _check_same_device(a, b)
    ka = a.shape[-1]
    kb = b.shape[0] if b.ndim == 1 else b.shape[-2]
    check(ka == kb, lambda: f"matmul: {tuple(a.shape)} @ {tuple(b.shape)} shape mismatch")
    if a.ndim == 1 and b.ndim == 1:
        shape = ()
    elif b.ndim == 1:
        shape = tuple(a.shape[:-1])
    elif a.ndim == 1:
        shape = tuple(b.shape[:-2]) + (b.shape[-1],)
    else:
        from ..clang import compute_broadcast_shape

        batch = compute_broadcast_shape(tuple(a.shape[:-2]), tuple(b.shape[:-2])) or ()
        shape = tuple(batch) + (a.shape[-2], b.shape[-1])
    return TensorProxy(shape=shape, device=device, dtype=a.dtype)


matmul = make_prim(PrimIDs.MATMUL, "matmul", meta=_matmul_meta, tags=(OpTags.MATMUL_OP,))


def _linear_meta(a, w, bias):
    check(a.shape[-1] == w.shape[-1], lambda: f"linear: {a.shape} @ {w.shape}^T shape mismatch")
    check(w.ndim == 2, "linear weight must be 2D")
    if bias is not None:
        check(bias.shape == (w.shape[0],), lambda: f"linear: bias shape {bias.shape}")
    check(a.dtype == w.dtype, lambda: f"linear: dtype mismatch {a.dtype} vs {w.dtype}")
    device = _check_same_device(a, w)
    return TensorProxy(shape=tuple(a.shape[:-1]) + (w.shape[0],), device=device, dtype=a.dtype)


linear = make_prim(PrimIDs.LINEAR, "linear", meta=_linear_meta, tags=(OpTags.MATMUL_OP,))


def _grouped_mm_meta(a, b, offsets):
    # a: [M, K], b: [G, K, N], offsets [G] -> [M, N]
    if a.ndim == 2 and b.ndim == 3:
        shape = (a.shape[0], b.shape[2])
    elif a.ndim == 2 and b.ndim == 2:
        shape = (offsets.shape[0], a.shape[0], b.shape[1])
    else:
        shape = (a.shape[0], a.shape[1], b.shape[-1])
    return TensorProxy(like=a, shape=shape)


_grouped_mm = make_prim(PrimIDs.GROUPED_MM, "_grouped_mm", meta=_grouped_mm_meta, tags=(OpTags.MATMUL_OP,))


def _embedding_meta(a, weight, *, padding_idx=-1, max_norm=None, norm_type=2.0, scale_grad_by_freq=False, sparse=False):
    check(not dtypes.is_float_dtype(a.dtype), "embedding indices must be integers")
    return TensorProxy(like=weight, shape=tuple(a.shape) + (weight.shape[1],))


embedding = make_prim(PrimIDs.EMBEDDING, "embedding", meta=_embedding_meta)


def _embedding_backward_meta(grad, indices, num_weights, padding_idx, scale_grad_by_freq, sparse):
    return TensorProxy(like=grad, shape=(num_weights, grad.shape[-1]))


embedding_backward = make_prim(PrimIDs.EMBEDDING_BACKWARD, "embedding_backward", meta=_embedding_backward_meta)


def _convolution_meta(a, weight, bias, stride, padding, dilation, transposed, output_padding, groups):
    ta = torch.empty(a.shape, dtype=a.dtype, device="meta")
    tw = torch.empty(weight.shape, dtype=weight.dtype, device="meta")
    tb = None if bias is None else torch.empty(bias.shape, dtype=bias.dtype, device="meta")
    out = torch.convolution(ta, tw, tb, stride, padding, dilation, transposed, output_padding, groups)
    return TensorProxy(like=a, shape=tuple(out.shape))


convolution = make_prim(PrimIDs.CONVOLUTION, "convolution", meta=_convolution_meta)


# -----------------------------------------------------------------------------------------
# Memory
# -----------------------------------------------------------------------------------------
def _copy__meta(copy_from, copy_to):
    check(copy_from.shape == copy_to.shape, lambda: f"copy_: shape mismatch {copy_from.shape} vs {copy_to.shape}")
    return TensorProxy(like=copy_to)


copy_ = make_prim(PrimIDs.COPY_, "copy_", meta=_copy__meta, tags=(OpTags.DONT_DCE, OpTags.IN_PLACE))
copy_.written_args = (1,)


def written_args(bsym) -> list:
    """The proxy arguments an ``IN_PLACE`` bound symbol actually writes.

    A symbol declares them with a ``written_args`` attribute: positional indices or keyword names
    (``copy_`` writes its destination, ``index_copy_inplace`` its buffer, the fused RoPE+KV-cache
    kernel its two caches).  An ``IN_PLACE`` symbol that declares nothing is taken to write every
    tensor argument (conservative).  Non-``IN_PLACE`` symbols write nothing."""
    sym = bsym.sym
    if OpTags.IN_PLACE not in getattr(sym, "tags", ()):
        return []
    idx = getattr(sym, "written_args", None)
    if idx is None:
        return [a for a in bsym.flat_proxy_args if isinstance(a, _proxies.TensorProxy)]
    out = []
    for i in idx:
        a = bsym.args[i] if isinstance(i, int) and i < len(bsym.args) else bsym.kwargs.get(i) if isinstance(i, str) else None
        if isinstance(a, _proxies.TensorProxy):
            out.append(a)
    return out


def _item_meta(a):
    pt = dtypes.dtype_to_numbertype(a.dtype)
    return NumberProxy(None, pt)


item = make_prim(PrimIDs.ITEM, "item", meta=_item_meta, tags=(OpTags.DEVICE_SYNC_OP, NON_DIFFERENTIABLE_TAG))


def _shallow_copy_meta(a):
    return TensorProxy(like=a)


shallow_copy = make_prim(PrimIDs.SHALLOW_COPY, "shallow_copy", meta=_shallow_copy_meta)


def is_elementwise(sym) -> bool:
    return OpTags.ELEMENTWISE in sym.tags


ALL_ELEMENTWISE_UNARY = {
    PrimIDs.ABS, PrimIDs.ACOS, PrimIDs.ACOSH, PrimIDs.ASIN, PrimIDs.ASINH, PrimIDs.ATAN, PrimIDs.ATANH,
    PrimIDs.BITWISE_NOT, PrimIDs.CEIL, PrimIDs.COS, PrimIDs.COSH, PrimIDs.DIGAMMA, PrimIDs.ERF, PrimIDs.ERFC,
    PrimIDs.ERFINV, PrimIDs.ERFCINV, PrimIDs.NDTRI, PrimIDs.EXP, PrimIDs.EXP2, PrimIDs.EXPM1, PrimIDs.FLOOR, PrimIDs.ISFINITE, PrimIDs.LGAMMA,
    PrimIDs.LOG, PrimIDs.LOG10, PrimIDs.LOG1P, PrimIDs.LOG2, PrimIDs.NEG, PrimIDs.RECIPROCAL, PrimIDs.ROUND,
    PrimIDs.RSQRT, PrimIDs.SIGN, PrimIDs.SIGNBIT, PrimIDs.SIN, PrimIDs.SINH, PrimIDs.SQRT, PrimIDs.TAN,
    PrimIDs.TANH, PrimIDs.TRUNC, PrimIDs.REAL, PrimIDs.IMAG,
}
