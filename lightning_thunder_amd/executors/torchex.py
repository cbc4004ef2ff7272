"""The PyTorch-ROCm ATen executor — the always-available fallback (parity: reference
``thunder/executors/torchex.py:37-2400``).

* Every ``ltorch`` symbol that was registered from a torch callable is replayed by
  calling that callable with the recorded arguments, so claimed programs call ATen
  (and hipBLASLt for GEMMs) directly — generated traces read ``torch.nn.functional.linear(...)``.
* Every prim has an ATen implementation here.
* Auto-registered opaque ops call their original torch callable.
* Distributed prims lower to RCCL through ``torch.distributed`` (registered by
  ``distributed/prims.py``).
"""
from __future__ import annotations

import math
from typing import Any, Callable

import torch

from ..core import prims
from ..core.prims import PrimIDs
from ..core.proxies import TensorProxy
from ..core.symbol import Symbol
from ..extend import OperatorExecutor, register_executor, add_always_executor, add_default_executor

ex = OperatorExecutor("torch", version=torch.__version__)
register_executor(ex)
add_always_executor(ex)

torch_executor = ex
pytorch_executor = ex


def _register_prim(prim: Symbol, fn: Callable, *, name: str | None = None, checker=None):
    op = ex.register_operator(name or f"torch_{prim.name}", like=prim, fn=fn)
    ex.register_implementation(prim, op, checker=checker)
    return op


# =========================================================================================
# Prims
# =========================================================================================
def _convert_element_type(a, dtype):
    if isinstance(a, torch.Tensor):
        return a.to(dtype)
    return a


_register_prim(prims.convert_element_type, _convert_element_type, name="convert_element_type")


def _device_put(a, device):
    return a.to(device)


_register_prim(prims.device_put, _device_put, name="device_put")
_register_prim(prims.bitcast, lambda a, dtype: a.view(dtype), name="bitcast")


def _full(shape, fill_value, *, device, dtype):
    return torch.full(shape, fill_value, device=device, dtype=dtype)


_register_prim(prims.full, _full, name="full")


def _iota(length, *, start, step, device, dtype):
    return torch.arange(start, start + step * length, step, device=device, dtype=dtype)[:length]


_register_prim(prims.iota, _iota, name="iota")


def _uniform(shape, minval, maxval, *, device, dtype):
    t = torch.empty(shape, device=device, dtype=dtype)
    return t.uniform_(minval, maxval)


_register_prim(prims.uniform, _uniform, name="uniform")


def _uniform_philox(shape, minval, maxval, *, device, dtype, seed, offset):
    # the framework's Philox (core/rng.py): bit-identical to hipfuse's inline generator
    from ..core.rng import philox_uniform_torch

    u = philox_uniform_torch(tuple(shape), seed, offset, device)  # GraphRngInt kept: graph-safe seed / base
    if minval != 0.0 or maxval != 1.0:
        u = u * (maxval - minval) + minval
    return u.to(dtype)


_register_prim(prims.uniform_philox, _uniform_philox, name="uniform_philox")
_register_prim(prims.randn, lambda shape, *, device, dtype: torch.randn(shape, device=device, dtype=dtype), name="randn")
_register_prim(prims.empty, lambda shape, *, device, dtype: torch.empty(shape, device=device, dtype=dtype), name="empty")
_register_prim(
    prims.tensor_from_sequence, lambda seq, *, dtype, device: torch.tensor(seq, dtype=dtype, device=device), name="tensor_from_sequence"
)


def _broadcast_in_dim(a, shape, broadcast_dimensions):
    s = [1] * len(shape)
    for i, d in enumerate(broadcast_dimensions):
        s[d] = a.shape[i]
    v = a.reshape(s)
    return v.expand(shape)


_register_prim(prims.broadcast_in_dim, _broadcast_in_dim, name="broadcast_in_dim")
_register_prim(prims.cat, lambda tensors, dim: torch.cat(tensors, dim), name="cat_prim")
_register_prim(prims.flip, lambda a, dims: torch.flip(a, dims), name="flip_prim")


def _pad(a, padding_value, padding_config):
    if all(interior == 0 for _, _, interior in padding_config) and all(lo >= 0 and hi >= 0 for lo, hi, _ in padding_config):
        pads = []
        for lo, hi, _ in reversed(padding_config):
            pads += [lo, hi]
        return torch.nn.functional.pad(a, pads, value=padding_value)
    shape = [lo + hi + s + max(s - 1, 0) * it for s, (lo, hi, it) in zip(a.shape, padding_config)]
    out = torch.full(shape, padding_value, dtype=a.dtype, device=a.device)
    idx = tuple(slice(lo, lo + s + max(s - 1, 0) * it, it + 1) for s, (lo, hi, it) in zip(a.shape, padding_config))
    out[idx] = a
    return out


_register_prim(prims.pad, _pad, name="pad_prim")
_register_prim(prims.reshape, lambda a, shape: a.reshape(shape), name="reshape_prim")


def _slice(a, start_indices, end_indices, strides=None):
    if strides is None:
        strides = [1] * a.ndim
    return a[tuple(slice(s, e, st) for s, e, st in zip(start_indices, end_indices, strides))]


_register_prim(prims.slice_prim, _slice, name="slice_prim")
_register_prim(prims.squeeze, lambda a, dims: a.squeeze(tuple(dims)) if dims else a, name="squeeze_prim")
_register_prim(prims.transpose, lambda a, permutation: a.permute(permutation), name="transpose_prim")
_register_prim(prims.take, lambda a, indices, dim: _take(a, indices, dim), name="take")


def _take(a, indices, dim):
    if indices.ndim == 1:
        return torch.index_select(a, dim, indices)
    flat = torch.index_select(a, dim, indices.reshape(-1))
    shape = list(a.shape)
    shape[dim:dim + 1] = list(indices.shape)
    return flat.reshape(shape)


_register_prim(prims.take_along_axis, lambda a, indices, dim: torch.gather(a, dim, indices), name="take_along_axis")
_register_prim(prims.index_add, lambda a, indices, value, dim: torch.index_add(a, dim, indices, value), name="index_add_prim")
_register_prim(
    prims.index_put, lambda a, indices, values, accumulate: torch.index_put(a, tuple(indices), values, accumulate), name="index_put_prim"
)
_register_prim(prims.scatter_add, lambda a, index, value, dim: torch.scatter_add(a, dim, index, value), name="scatter_add_prim")
_register_prim(prims.scatter, lambda a, index, src, dim: torch.scatter(a, dim, index, src), name="scatter_prim")

# elementwise unary
_unary_map = {
    prims.abs: torch.abs, prims.acos: torch.acos, prims.acosh: torch.acosh, prims.asin: torch.asin,
    prims.asinh: torch.asinh, prims.atan: torch.atan, prims.atanh: torch.atanh, prims.bitwise_not: torch.bitwise_not,
    prims.ceil: torch.ceil, prims.cos: torch.cos, prims.cosh: torch.cosh, prims.digamma: torch.digamma,
    prims.erf: torch.erf, prims.erfc: torch.erfc, prims.erfinv: torch.erfinv, prims.erfcinv: lambda a: torch.erfinv(1 - a),
    prims.ndtri: torch.special.ndtri, prims.exp: torch.exp,
    prims.exp2: torch.exp2, prims.expm1: torch.expm1, prims.floor: torch.floor, prims.isfinite: torch.isfinite,
    prims.lgamma: torch.lgamma, prims.log: torch.log, prims.log10: torch.log10, prims.log1p: torch.log1p,
    prims.log2: torch.log2, prims.neg: torch.neg, prims.reciprocal: torch.reciprocal, prims.round: torch.round,
    prims.rsqrt: torch.rsqrt, prims.sign: torch.sign, prims.signbit: torch.signbit, prims.sin: torch.sin,
    prims.sinh: torch.sinh, prims.sqrt: torch.sqrt, prims.tan: torch.tan, prims.tanh: torch.tanh,
    prims.trunc: torch.trunc, prims.real: torch.real, prims.imag: torch.imag,
}
for _p, _f in _unary_map.items():
    _register_prim(_p, _f, name=f"{_p.name}_prim")


def _div(a, b):
    def is_int(x):
        if isinstance(x, torch.Tensor):
            return not x.is_floating_point() and not x.is_complex()
        return isinstance(x, int)

    if is_int(a) and is_int(b):
        return torch.div(a, b, rounding_mode="floor")
    return torch.true_divide(a, b)


_binary_map = {
    prims.add: torch.add, prims.atan2: torch.atan2, prims.bitwise_and: torch.bitwise_and,
    prims.bitwise_or: torch.bitwise_or, prims.bitwise_xor: torch.bitwise_xor,
    prims.bitwise_left_shift: torch.bitwise_left_shift, prims.bitwise_right_shift: torch.bitwise_right_shift,
    prims.copysign: torch.copysign, prims.div: _div, prims.eq: torch.eq, prims.fmod: torch.fmod,
    prims.ge: torch.ge, prims.gt: torch.gt, prims.le: torch.le, prims.lt: torch.lt,
    prims.maximum: torch.maximum, prims.minimum: torch.minimum, prims.mul: torch.mul, prims.ne: torch.ne,
    prims.nextafter: torch.nextafter, prims.pow: torch.pow, prims.remainder: torch.remainder, prims.sub: torch.sub,
    prims.zeta: torch.special.zeta,
}


def _wrap_binary(f):
    def fn(a, b):
        # maximum/minimum/etc. need tensors on both sides
        if not isinstance(a, torch.Tensor) and f in (torch.maximum, torch.minimum, torch.atan2, torch.copysign, torch.nextafter, torch.special.zeta):
            a = torch.tensor(a, dtype=b.dtype, device=b.device)
        if not isinstance(b, torch.Tensor) and f in (torch.maximum, torch.minimum, torch.atan2, torch.copysign, torch.nextafter, torch.special.zeta):
            b = torch.tensor(b, dtype=a.dtype, device=a.device)
        if not isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor) and f in (torch.add, torch.mul, torch.eq, torch.ne, torch.bitwise_and, torch.bitwise_or, torch.bitwise_xor):
            return f(b, a)
        if not isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor):
            a = torch.tensor(a, dtype=b.dtype, device=b.device)
        return f(a, b)

    return fn


for _p, _f in _binary_map.items():
    _register_prim(_p, _wrap_binary(_f), name=f"{_p.name}_prim")


def _where(pred, a, b):
    return torch.where(pred, a, b)


_register_prim(prims.where, _where, name="where_prim")

# reductions
_register_prim(prims.sum, lambda a, dims, *, output_dtype=None: torch.sum(a, dims, dtype=output_dtype) if dims else a, name="sum_prim")
_register_prim(prims.prod, lambda a, dims, *, output_dtype=None: _prod(a, dims), name="prod_prim")


def _prod(a, dims):
    for d in sorted(dims, reverse=True):
        a = torch.prod(a, d)
    return a


_register_prim(prims.amax, lambda a, dims, *, output_dtype=None: torch.amax(a, dims) if dims else a, name="amax_prim")
_register_prim(prims.amin, lambda a, dims, *, output_dtype=None: torch.amin(a, dims) if dims else a, name="amin_prim")
_register_prim(prims.var, lambda a, dims, *, correction: torch.var(a, dims, correction=correction), name="var_prim")
_register_prim(prims.var_mean, lambda a, dims, *, correction: torch.var_mean(a, dims, correction=correction), name="var_mean_prim")
_register_prim(prims.argmax, lambda a, dim: torch.argmax(a, dim), name="argmax_prim")
_register_prim(prims.argmin, lambda a, dim: torch.argmin(a, dim), name="argmin_prim")
_register_prim(prims.topk, lambda a, k, dim, largest, sorted: tuple(torch.topk(a, k, dim, largest, sorted)), name="topk_prim")
_register_prim(prims.sort, lambda a, dim, descending, stable: tuple(torch.sort(a, dim=dim, descending=descending, stable=stable)), name="sort_prim")
_register_prim(prims.cumsum, lambda a, dim, *, dtype=None: torch.cumsum(a, dim, dtype=dtype), name="cumsum_prim")

# linear algebra / nn
_register_prim(prims.matmul, torch.matmul, name="matmul")
_register_prim(prims.linear, torch.nn.functional.linear, name="linear")
def _grouped_mm_impl(a, b, offsets):
    if a.is_cuda and hasattr(torch, "_grouped_mm") and a.dtype == torch.bfloat16:
        return torch._grouped_mm(a, b, offsets)
    # reference loop (CPU): group g owns rows/K-slices [offsets[g-1], offsets[g])
    ends = offsets.tolist()
    starts = [0] + ends[:-1]
    if a.dim() == 2 and b.dim() == 3:
        out = a.new_zeros((a.shape[0], b.shape[2]))
        for g, (s, e) in enumerate(zip(starts, ends)):
            out[s:e] = a[s:e] @ b[g]
        return out
    if a.dim() == 2 and b.dim() == 2:  # shared dim grouped: [G, M, N]
        return torch.stack([a[:, s:e] @ b[s:e] for s, e in zip(starts, ends)])
    raise NotImplementedError("grouped_mm layout")


_register_prim(prims._grouped_mm, _grouped_mm_impl, name="grouped_mm")


def _embedding(a, weight, *, padding_idx=-1, max_norm=None, norm_type=2.0, scale_grad_by_freq=False, sparse=False):
    return torch.nn.functional.embedding(a, weight, None if padding_idx == -1 else padding_idx, max_norm, norm_type, scale_grad_by_freq, sparse)


_register_prim(prims.embedding, _embedding, name="embedding_prim")


def _embedding_backward(grad, indices, num_weights, padding_idx, scale_grad_by_freq, sparse):
    return torch.ops.aten.embedding_backward(grad, indices, num_weights, padding_idx, scale_grad_by_freq, sparse)


_register_prim(prims.embedding_backward, _embedding_backward, name="embedding_backward")
_register_prim(prims.convolution, torch.convolution, name="convolution")


def _copy_(copy_from, copy_to):
    copy_to.copy_(copy_from)
    return copy_to


_register_prim(prims.copy_, _copy_, name="copy_")
_register_prim(prims.item, lambda a: a.item(), name="item")
_register_prim(prims.shallow_copy, lambda a: a.clone(), name="shallow_copy")


# =========================================================================================
# ltorch symbols: replay the original torch callable
# =========================================================================================
_NO_DIRECT_TORCH = {"torch.checkpoint", "torch.setitem_", "torch.detach"}


def _add(a, b, *, alpha=None):
    return torch.add(a, b) if alpha is None else torch.add(a, b, alpha=alpha)


def _sub(a, b, *, alpha=None):
    return torch.sub(a, b) if alpha is None else torch.sub(a, b, alpha=alpha)


def _var(a, dim=None, unbiased=None, keepdim=False, *, correction=None):
    if correction is None:
        correction = 1 if unbiased is None or unbiased else 0
    return torch.var(a, dim, correction=correction, keepdim=keepdim)


def _var_mean(a, dim=None, unbiased=None, keepdim=False, *, correction=None):
    if correction is None:
        correction = 1 if unbiased is None or unbiased else 0
    return torch.var_mean(a, dim, correction=correction, keepdim=keepdim)


def _number_first(fn, commutative: bool):
    """torch binary ops reject a python number as the first operand; compiler-created calls may pass one."""

    def adapter(a, b, **kwargs):
        if not isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor):
            if commutative and not kwargs:
                return fn(b, a)
            a = torch.tensor(a, device=b.device)
        return fn(a, b, **kwargs)

    adapter.__name__ = getattr(fn, "__name__", "binary")
    return adapter


# ltorch signatures that differ from the canonical torch callable (used for compiler-created calls)
_canonical_overrides = {
    "torch.add": _number_first(_add, True),
    "torch.sub": _number_first(_sub, False),
    "torch.var": _var,
    "torch.var_mean": _var_mean,
    "torch.mul": _number_first(torch.mul, True),
    "torch.true_divide": _number_first(torch.true_divide, False),
    "torch.div": _number_first(torch.div, False),
    "torch.floor_divide": _number_first(torch.floor_divide, False),
    "torch.remainder": _number_first(torch.remainder, False),
    "torch.pow": _number_first(torch.pow, False),
    "torch.eq": _number_first(torch.eq, True),
    "torch.ne": _number_first(torch.ne, True),
    "torch.lt": _number_first(torch.lt, False),
    "torch.le": _number_first(torch.le, False),
    "torch.gt": _number_first(torch.gt, False),
    "torch.ge": _number_first(torch.ge, False),
    "torch.maximum": _number_first(torch.maximum, False),
    "torch.minimum": _number_first(torch.minimum, False),
    "torch.bitwise_and": _number_first(torch.bitwise_and, True),
    "torch.bitwise_or": _number_first(torch.bitwise_or, True),
    "torch.bitwise_xor": _number_first(torch.bitwise_xor, True),
    "torch.reshape": torch.Tensor.reshape,
    "torch.permute": torch.Tensor.permute,
    "torch.flip": torch.Tensor.flip,
}


def _register_ltorch():
    from .. import torch as ltorch
    from ..core.symbol import _symbol_registry

    seen = set()
    for sym in list(_symbol_registry.values()):
        if not (isinstance(sym.id, str) and sym.id.startswith("torch.")):
            continue
        if sym.id in _NO_DIRECT_TORCH or sym.id in seen:
            continue
        tfn = getattr(sym, "torch_fn", None)
        if tfn is None:
            continue
        seen.add(sym.id)
        op = ex.register_operator(f"torch_{sym.name}", like=sym, fn=_canonical_overrides.get(sym.id, tfn))
        op.replay_torch = True
        ex.register_implementation(sym, op)

    # detach as its own op
    op = ex.register_operator("detach", like=ltorch.detach, fn=torch.Tensor.detach)
    ex.register_implementation(ltorch.detach, op)


_register_ltorch()


# =========================================================================================
# Fused attention through ATen (fallback when the HIP flash-attention kernel does not apply)
# (parity: reference thunder/executors/sdpaex.py:34-568)
# =========================================================================================
def _sdpa_fwd_meta(q, k, v, is_causal, scale):
    B, H, L, E = q.shape
    out = TensorProxy(like=q, shape=(B, H, L, v.shape[-1]))
    lse = TensorProxy(like=q, shape=(B, H, L), dtype=torch.float32, requires_grad=False)
    return out, lse


def _sdpa_fwd_impl(q, k, v, is_causal, scale):
    r = torch.ops.aten._scaled_dot_product_flash_attention(q, k, v, 0.0, is_causal, False, scale=scale)
    return r[0], r[1]


def _sdpa_bwd_meta(g, q, k, v, out, lse, is_causal, scale):
    return TensorProxy(like=q), TensorProxy(like=k), TensorProxy(like=v)


def _sdpa_bwd_impl(g, q, k, v, out, lse, is_causal, scale):
    L, S = q.shape[-2], k.shape[-2]
    zero = torch.empty((), dtype=torch.int64, device="cpu")
    r = torch.ops.aten._scaled_dot_product_flash_attention_backward(
        g.contiguous(), q, k, v, out, lse, None, None, L, S, 0.0, is_causal, zero, zero, scale=scale
    )
    return r[0], r[1], r[2]


aten_sdpa_fwd = ex.register_operator("aten_flash_sdpa_fwd", meta=_sdpa_fwd_meta, fn=_sdpa_fwd_impl)
aten_sdpa_bwd = ex.register_operator("aten_flash_sdpa_bwd", meta=_sdpa_bwd_meta, fn=_sdpa_bwd_impl)


def _sdpa_checker(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False, *, scale=None, enable_gqa=False):
    if attn_mask is not None or dropout_p != 0.0:
        return False
    if query.device.type != "cuda" or query.dtype not in (torch.bfloat16, torch.float16):
        return False
    if query.ndim != 4 or key.dtype != query.dtype or value.dtype != query.dtype:
        return False
    return query.shape[-1] <= 256 and query.shape[-1] % 8 == 0


def _expand_kv(query, key, value):
    from .. import torch as ltorch

    rep = query.shape[-3] // key.shape[-3]
    if rep > 1:
        key = ltorch.repeat_interleave(key, rep, -3)
        value = ltorch.repeat_interleave(value, rep, -3)
    return key, value


def _sdpa_grad(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False, *, scale=None, enable_gqa=False):
    from .. import torch as ltorch

    if not _sdpa_checker(query, key, value, attn_mask, dropout_p, is_causal, scale=scale, enable_gqa=enable_gqa):
        return None
    sc = scale if scale is not None else 1.0 / math.sqrt(query.shape[-1])
    k, v = _expand_kv(query, key, value)
    out, lse = aten_sdpa_fwd(query, k, v, is_causal, sc)

    def bwd(g):
        dq, dk, dv = aten_sdpa_bwd(g, query, k, v, out, lse, is_causal, sc)
        rep = query.shape[-3] // key.shape[-3]
        if rep > 1:
            shp = tuple(key.shape)
            dk = ltorch.sum(ltorch.reshape(dk, shp[:-3] + (shp[-3], rep) + shp[-2:]), -3)
            dv = ltorch.sum(ltorch.reshape(dv, shp[:-3] + (shp[-3], rep) + shp[-2:]), -3)
        return dq, dk, dv

    return out, bwd


def _sdpa_exec(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False, *, scale=None, enable_gqa=False):
    sc = scale if scale is not None else 1.0 / math.sqrt(query.shape[-1])
    k, v = _expand_kv(query, key, value)
    out, _ = aten_sdpa_fwd(query, k, v, is_causal, sc)
    return out


def _register_sdpa():
    from .. import torch as ltorch

    # keep the plain replay for forward-only use; add the fused grad transform
    impl = ex.implmap.get(ltorch.scaled_dot_product_attention.id)
    ex.register_implementation(ltorch.scaled_dot_product_attention, impl.symbol if impl else None,
                               grad_transform=_sdpa_grad, checker=None)
    ex._sdpa_grad_checker = _sdpa_checker


_register_sdpa()


def register_opaque(sym: Symbol, fn: Callable) -> None:
    op = ex.register_operator(f"torch_{sym.name}", like=sym, fn=fn)
    ex.register_implementation(sym, op)


def register_torch_op(name: str, fn: Callable, *, meta: Callable | None = None, like: Symbol | None = None) -> Symbol:
    """Registers an extra torch-backed operator (used by transforms that need ATen calls)."""
    return ex.register_operator(name, fn=fn, meta=meta, like=like)


# no_autocast decorator applied to generated programs (reference: executors/torchex.py no_autocast)
def no_autocast(fn):
    import functools

    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        if torch.is_autocast_enabled():
            with torch.autocast("cuda", enabled=False), torch.autocast("cpu", enabled=False):
                return fn(*args, **kwargs)
        return fn(*args, **kwargs)

    return wrapper
