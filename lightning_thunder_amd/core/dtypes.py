"""Dtype lattice used by the trace IR.

Capability parity with the reference's ``thunder/core/dtypes.py`` (``dtype`` :55,
``to_dtype`` :290, ``to_torch_dtype`` :544).  The reference keeps its own dtype
objects with "strong"/"weak" variants; here the IR stores ``torch.dtype``
directly (PyTorch-ROCm is the only runtime) and the weak/strong distinction is
expressed by Python number *types* (``int``/``float``/``complex``/``bool``)
flowing through type promotion, exactly as torch does it.
"""
from __future__ import annotations

from numbers import Number

import torch

bool8 = torch.bool
uint8 = torch.uint8
int8 = torch.int8
int16 = torch.int16
int32 = torch.int32
int64 = torch.int64
bfloat16 = torch.bfloat16
float16 = torch.float16
float32 = torch.float32
float64 = torch.float64
complex32 = torch.complex32
complex64 = torch.complex64
complex128 = torch.complex128
# CDNA4 (gfx950) implements the OCP fp8 encodings; the fnuz variants are kept
# for checkpoint interchange with MI300-era tooling only.
float8_e4m3fn = torch.float8_e4m3fn
float8_e5m2 = torch.float8_e5m2
float8_e4m3fnuz = torch.float8_e4m3fnuz
float8_e5m2fnuz = torch.float8_e5m2fnuz

float8_dtypes = (float8_e4m3fn, float8_e5m2, float8_e4m3fnuz, float8_e5m2fnuz)
# Microscaling (OCP MX) storage types, both native to the CDNA4 block-scaled MFMA
# (v_mfma_scale_f32_*_f8f6f4): packed fp4 e2m1 (two values per byte) and the E8M0 power-of-two
# block scale.  Tensors of these types are storage (quantized weights, scales); arithmetic happens
# in the kernels that consume them.
float4_e2m1fn_x2 = getattr(torch, "float4_e2m1fn_x2", None)
float8_e8m0fnu = getattr(torch, "float8_e8m0fnu", None)
mx_storage_dtypes = tuple(d for d in (float4_e2m1fn_x2, float8_e8m0fnu) if d is not None)
low_precision_dtypes = (bfloat16, float16, complex32) + float8_dtypes + mx_storage_dtypes
float_dtypes = (bfloat16, float16, float32, float64) + float8_dtypes
complex_dtypes = (complex32, complex64, complex128)
signed_int_dtypes = (int8, int16, int32, int64)
int_dtypes = (uint8,) + signed_int_dtypes
all_dtypes = (bool8,) + int_dtypes + float_dtypes + complex_dtypes + mx_storage_dtypes

_short_names = {
    bool8: "b8",
    uint8: "ui8",
    int8: "i8",
    int16: "i16",
    int32: "i32",
    int64: "i64",
    bfloat16: "bf16",
    float16: "f16",
    float32: "f32",
    float64: "f64",
    complex32: "c32",
    complex64: "c64",
    complex128: "c128",
    float8_e4m3fn: "f8_e4m3fn",
    float8_e5m2: "f8_e5m2",
    float8_e4m3fnuz: "f8_e4m3fnuz",
    float8_e5m2fnuz: "f8_e5m2fnuz",
}
if float4_e2m1fn_x2 is not None:
    _short_names[float4_e2m1fn_x2] = "f4_e2m1x2"
if float8_e8m0fnu is not None:
    _short_names[float8_e8m0fnu] = "f8_e8m0"

number_types = (bool, int, float, complex)


def short_name(dtype) -> str:
    if isinstance(dtype, type):
        return dtype.__name__
    return _short_names.get(dtype, str(dtype).replace("torch.", ""))


def is_dtype(x) -> bool:
    return isinstance(x, torch.dtype) or x in number_types


def is_boolean_dtype(d) -> bool:
    return d is torch.bool or d is bool


def is_unsigned_dtype(d) -> bool:
    return d is torch.uint8 or d is bool or d is torch.bool


def is_integer_dtype(d) -> bool:
    """Includes booleans, like the reference (``dtypes.is_integer_dtype``)."""
    if d in (bool, int):
        return True
    return isinstance(d, torch.dtype) and (not d.is_floating_point) and (not d.is_complex)


def is_exact_dtype(d) -> bool:
    return is_integer_dtype(d)


def is_nonboolean_integer_dtype(d) -> bool:
    return is_integer_dtype(d) and not is_boolean_dtype(d)


def is_float_dtype(d) -> bool:
    if d is float:
        return True
    return isinstance(d, torch.dtype) and d.is_floating_point


def is_complex_dtype(d) -> bool:
    if d is complex:
        return True
    return isinstance(d, torch.dtype) and d.is_complex


def is_inexact_dtype(d) -> bool:
    return is_float_dtype(d) or is_complex_dtype(d)


def is_low_precision_dtype(d) -> bool:
    return d in low_precision_dtypes


def is_float8_dtype(d) -> bool:
    return d in float8_dtypes


def is_mx_storage_dtype(d) -> bool:
    """Packed fp4 (e2m1 x2) or E8M0 scale storage."""
    return d in mx_storage_dtypes


def is_weak_dtype(d) -> bool:
    """Python number types behave like the reference's "weak" dtypes in promotion."""
    return d in number_types


def itemsize(d) -> int:
    if d in number_types:
        return {bool: 1, int: 8, float: 8, complex: 16}[d]
    return _itemsize_cache[d]


_itemsize_cache = {d: torch.empty((), dtype=d, device="meta").element_size() for d in all_dtypes if d is not complex32}
_itemsize_cache[complex32] = 4


def to_dtype(x, *, true_dtype: bool = False):
    """Maps values, tensors, proxies, python types and torch dtypes to a dtype."""
    if x is None:
        return None
    if isinstance(x, torch.dtype):
        return x
    if x in number_types:
        return x
    if isinstance(x, torch.Tensor):
        return x.dtype
    if isinstance(x, bool):
        return bool
    if isinstance(x, int):
        return int
    if isinstance(x, float):
        return float
    if isinstance(x, complex):
        return complex
    dt = getattr(x, "dtype", None)
    if dt is not None:
        return dt
    pt = getattr(x, "python_type", None)
    if pt is not None:
        return pt
    raise ValueError(f"Cannot compute a dtype from {x} of type {type(x)}")


def to_torch_dtype(x) -> torch.dtype | None:
    if x is None:
        return None
    if isinstance(x, torch.dtype):
        return x
    if x is bool:
        return torch.bool
    if x is int:
        return torch.int64
    if x is float:
        return torch.get_default_dtype()
    if x is complex:
        return torch.complex64 if torch.get_default_dtype() is torch.float32 else torch.complex128
    if isinstance(x, str):
        return getattr(torch, x)
    return to_dtype(x)


def dtype_to_numbertype(d):
    if d in number_types:
        return d
    if is_boolean_dtype(d):
        return bool
    if is_integer_dtype(d):
        return int
    if is_float_dtype(d):
        return float
    if is_complex_dtype(d):
        return complex
    raise ValueError(f"Unknown dtype {d}")


def numbertype_of(x) -> type:
    if isinstance(x, bool):
        return bool
    if isinstance(x, int):
        return int
    if isinstance(x, float):
        return float
    if isinstance(x, complex):
        return complex
    pt = getattr(x, "python_type", None)
    if pt is not None:
        return pt
    raise ValueError(f"{x} is not a number")


def corresponding_real_dtype(d):
    return {complex32: float16, complex64: float32, complex128: float64, complex: float}.get(d, d)


def corresponding_complex_dtype(d):
    return {float16: complex32, float32: complex64, float64: complex128, float: complex, bfloat16: complex64}.get(d, d)


def is_number(x) -> bool:
    return isinstance(x, Number) and not isinstance(x, torch.Tensor)


# Category ranks for torch-style type promotion
_BOOL, _INT, _FLOAT, _COMPLEX = 0, 1, 2, 3


def category(d) -> int:
    if is_boolean_dtype(d):
        return _BOOL
    if is_integer_dtype(d):
        return _INT
    if is_float_dtype(d):
        return _FLOAT
    return _COMPLEX


def promote_tensor_and_number_dtypes(tensor_dtypes, number_types_) -> torch.dtype:
    """torch's result_type semantics: tensors (dim>=0) dominate numbers of the same category."""
    result = None
    for d in tensor_dtypes:
        result = d if result is None else torch.promote_types(result, d)
    if result is None:
        # only numbers: use python promotion then map to default torch dtype
        cat = max(category(t) for t in number_types_)
        return to_torch_dtype([bool, int, float, complex][cat])
    tcat = category(result)
    for nt in number_types_:
        ncat = category(nt)
        if ncat > tcat:
            if ncat == _FLOAT:
                result = torch.get_default_dtype() if tcat < _FLOAT else result
            elif ncat == _COMPLEX:
                result = corresponding_complex_dtype(result if tcat == _FLOAT else torch.get_default_dtype())
            elif ncat == _INT:
                result = torch.int64
            tcat = ncat
    return result


__all__ = [
    "bool8", "uint8", "int8", "int16", "int32", "int64", "bfloat16", "float16", "float32", "float64",
    "complex32", "complex64", "complex128", "float8_e4m3fn", "float8_e5m2", "float8_e4m3fnuz", "float8_e5m2fnuz",
    "to_dtype", "to_torch_dtype", "is_float_dtype", "is_integer_dtype", "is_complex_dtype", "is_boolean_dtype",
    "is_low_precision_dtype", "is_float8_dtype", "is_mx_storage_dtype", "itemsize", "short_name",
    "float4_e2m1fn_x2", "float8_e8m0fnu", "mx_storage_dtypes",
]
