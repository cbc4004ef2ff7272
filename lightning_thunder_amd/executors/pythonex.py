"""The Python executor: prologue guards, unpacking, returns, deletes (parity: reference
``thunder/executors/pythonex.py:21-414``).

Prologue guard checks raise ``ThunderCacheMiss`` so a failing guard simply moves the
cache probe on to the next entry.
"""
from __future__ import annotations

import torch

from ..core import prims
from ..core.prims import PrimIDs
from ..extend import OperatorExecutor, register_executor, add_always_executor

ex = OperatorExecutor("python")
register_executor(ex)
add_always_executor(ex)

python_executor = ex


class ThunderCacheMiss(Exception):
    pass


def _unpack_sequence(x, n):
    if len(x) != n:
        raise ThunderCacheMiss(f"sequence length mismatch: {len(x)} vs {n}")
    return x


def _unpack_attr(o, n):
    try:
        return getattr(o, n)
    except AttributeError as e:  # a guarded attribute disappeared: not this cache entry
        raise ThunderCacheMiss(str(e)) from None


def _unpack_key(d, k):
    try:
        return d[k]
    except (KeyError, IndexError, TypeError) as e:
        raise ThunderCacheMiss(f"key {k!r}: {e}") from None


_DEV_STR: dict = {}


def _check_tensor(t, shape, device, dtype, requires_grad):
    if not isinstance(t, torch.Tensor):
        raise ThunderCacheMiss(f"expected a tensor, got {type(t)}")
    if None in shape:  # symbolic dims (cache="symbolic values"): rank and static dims here
        ok = t.ndim == len(shape) and all(n is None or n == m for n, m in zip(shape, t.shape))
    else:
        ok = t.shape == shape
    dev = t.device
    ds = _DEV_STR.get(dev)
    if ds is None:
        ds = _DEV_STR[dev] = str(dev)
    if not ok or t.dtype != dtype or ds != device or t.requires_grad != requires_grad:
        raise ThunderCacheMiss(
            f"tensor metadata mismatch: {tuple(t.shape)},{t.dtype},{t.device},{t.requires_grad} vs {shape},{dtype},{device},{requires_grad}"
        )


def _check_number(n, value):
    if type(n) is not type(value) or (n != value and not (n != n and value != value)):
        raise ThunderCacheMiss(f"number mismatch: {n!r} vs {value!r}")


def _check_number_type(n, typ):
    if type(n) is not typ:
        raise ThunderCacheMiss(f"number type mismatch: {type(n).__name__} vs {typ.__name__}")


def _check_len(x, n):
    if len(x) != n:
        raise ThunderCacheMiss(f"length mismatch: {len(x)} vs {n}")


def _check_none(x):
    if x is not None:
        raise ThunderCacheMiss("expected None")


def _check_string(s, v):
    if s != v:
        raise ThunderCacheMiss(f"string mismatch {s!r} vs {v!r}")


def _check_literal_like(x, v):
    if type(x) is not type(v) or x != v:
        raise ThunderCacheMiss(f"value mismatch {x!r} vs {v!r}")


for prim, fn, name in (
    (prims.check_tensor_shape_and_metadata, _check_tensor, "check_tensor_metadata"),
    (prims.check_number_type_and_value, _check_number, "check_number_type_and_value"),
    (prims.check_number_type, _check_number_type, "check_number_type"),
    (prims.check_len, _check_len, "check_len"),
    (prims.check_none, _check_none, "check_none"),
    (prims.check_string_value, _check_string, "check_string_value"),
    (prims.check_literal_like, _check_literal_like, "check_literal_like"),
    (prims.unpack_key, _unpack_key, "unpack_key"),
    (prims.unpack_attr, _unpack_attr, "unpack_attr"),
    (prims.unpack_parameter, lambda o, n: o._parameters[n], "unpack_parameter"),
    (prims.unpack_buffer, lambda o, n: o._buffers[n], "unpack_buffer"),
    (prims.unpack_sequence, _unpack_sequence, "unpack_sequence"),
):
    op = ex.register_operator(name, like=prim, fn=fn)
    ex.register_implementation(prim, op)

# Return, del, comment and unpack_trivial print themselves as python statements.
for prim in (prims.python_return, prims.python_del, prims.comment, prims.unpack_trivial):
    ex.register_implementation(prim, prim)


def _get_rng_seed_offset(numel):
    from ..core.rng import seed_offset_for

    return seed_offset_for(int(numel))  # GraphRngInt values while a hipGraph region captures


_rng_op = ex.register_operator("get_rng_seed_offset", like=prims.get_rng_seed_offset, fn=_get_rng_seed_offset)
ex.register_implementation(prims.get_rng_seed_offset, _rng_op)
