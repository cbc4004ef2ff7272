"""K3 flash attention wrappers (kernels in ``csrc/attention_fwd.hip`` / ``attention_bwd.hip``)."""
from __future__ import annotations

import math

import torch

from ._lib import require, dcode, ptr, stream_ptr, check, register_signature, c_int, c_void_p, c_float

register_signature("lta_attn_fwd", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                    c_int, c_int, c_float, c_int, c_void_p])
register_signature("lta_attn_bwd", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                    c_float, c_int, c_void_p])

SUPPORTED_HEAD_DIMS = (64, 128)


def supported(q, k, v) -> bool:
    return (
        q.dtype in (torch.bfloat16, torch.float16)
        and k.dtype == q.dtype
        and v.dtype == q.dtype
        and q.ndim == 4
        and q.shape[-1] in SUPPORTED_HEAD_DIMS
        and k.shape[-1] == q.shape[-1]
        and v.shape[-1] == q.shape[-1]
        and q.shape[1] % k.shape[1] == 0
        and k.shape[1] == v.shape[1]
    )


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


def attn_fwd(q, k, v, causal: bool, scale: float | None = None):
    """q [B, Hq, T, D], k/v [B, Hkv, S, D] -> (o [B, Hq, T, D], lse [B, Hq, T] fp32)."""
    lib = require()
    q, k, v = _c(q), _c(k), _c(v)
    B, Hq, T, D = q.shape
    Hkv, S = k.shape[1], k.shape[2]
    sc = scale if scale is not None else 1.0 / math.sqrt(D)
    o = torch.empty_like(q)
    lse = torch.empty((B, Hq, T), device=q.device, dtype=torch.float32)
    rc = lib.lta_attn_fwd(dcode(q), ptr(q), ptr(k), ptr(v), ptr(o), ptr(lse), B, Hq, Hkv, T, S, D, float(sc), int(causal),
                          stream_ptr(q.device))
    check(rc, "lta_attn_fwd")
    return o, lse


def attn_bwd(do, q, k, v, o, lse, causal: bool, scale: float | None = None):
    """Returns (dq, dk, dv) with dk/dv summed over the query heads of each kv group."""
    lib = require()
    do, q, k, v, o = _c(do), _c(q), _c(k), _c(v), _c(o)
    B, Hq, T, D = q.shape
    Hkv, S = k.shape[1], k.shape[2]
    sc = scale if scale is not None else 1.0 / math.sqrt(D)
    dq = torch.empty_like(q)
    dk = torch.empty_like(k)
    dv = torch.empty_like(v)
    delta = torch.empty((B, Hq, T), device=q.device, dtype=torch.float32)
    rc = lib.lta_attn_bwd(dcode(q), ptr(do), ptr(q), ptr(k), ptr(v), ptr(o), ptr(lse), ptr(delta), ptr(dq), ptr(dk),
                          ptr(dv), None, B, Hq, Hkv, T, S, D, float(sc), int(causal), stream_ptr(q.device))
    check(rc, "lta_attn_bwd")
    return dq, dk, dv
