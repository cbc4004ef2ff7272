"""Wrappers for K6 (qkv split + RoPE), SwiGLU and K7 (cross entropy) kernels."""
from __future__ import annotations

import ctypes

import torch

from ._lib import require, dcode, ptr, stream_ptr, check, register_signature, c_int, c_int64, c_void_p, c_float

register_signature("lta_qkv_rope_fwd", [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_int, c_int, c_int, c_int, c_int, c_int, c_void_p])
register_signature("lta_qkv_rope_cache_fwd", [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p])
register_signature("lta_qkv_rope_bwd", [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_int, c_int, c_int, c_int, c_int, c_int, c_void_p])
register_signature("lta_swiglu_fwd", [c_int, c_void_p, c_void_p, c_void_p, c_int64, c_void_p])
register_signature("lta_swiglu_bwd", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p])
register_signature("lta_ce_fwd", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64,
                                  c_int, c_float, c_void_p])
register_signature("lta_ce_bwd", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64,
                                  c_int64, c_int, c_float, c_void_p])
register_signature("lta_ce_fwd_w", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64,
                                    c_int64, c_int, c_float, c_void_p])
register_signature("lta_ce_bwd_w", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                    c_int64, c_int64, c_int, c_float, c_void_p])


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


def qkv_rope_fwd(qkv, cos, sin, n_head: int, n_query_groups: int, head_size: int, rope_n: int):
    lib = require()
    qkv = _c(qkv)
    B, T, _ = qkv.shape
    cos = _c(cos[:T])
    sin = _c(sin[:T])
    if cos.dtype != sin.dtype:
        sin = sin.to(cos.dtype)
    if cos.dtype not in (torch.float32, qkv.dtype):
        cos, sin = cos.float(), sin.float()
    q = torch.empty((B, n_head, T, head_size), device=qkv.device, dtype=qkv.dtype)
    k = torch.empty((B, n_query_groups, T, head_size), device=qkv.device, dtype=qkv.dtype)
    v = torch.empty_like(k)
    rc = lib.lta_qkv_rope_fwd(dcode(qkv), dcode(cos), ptr(qkv), ptr(cos), ptr(sin), ptr(q), ptr(k), ptr(v), B, T,
                              n_head, n_query_groups, head_size, rope_n, stream_ptr(qkv.device))
    check(rc, "lta_qkv_rope_fwd")
    return q, k, v


def qkv_rope_cache_supported(qkv, kc, vc, pos, n_query_groups: int, head_size: int) -> bool:
    """Static caches [B, ng, S, hs] (head dim contiguous, 16-byte aligned rows) and int64 positions."""
    B, T, _ = qkv.shape
    for c in (kc, vc):
        if c.dtype != qkv.dtype or c.dim() != 4 or tuple(c.shape[:2]) != (B, n_query_groups) or c.shape[3] != head_size:
            return False
        if c.stride(3) != 1 or any(st % 8 for st in c.stride()[:3]) or c.data_ptr() % 16:
            return False
    return pos.dtype == torch.int64 and pos.dim() == 1 and pos.numel() == T and pos.is_contiguous()


def qkv_rope_cache_fwd(qkv, cos, sin, n_head: int, n_query_groups: int, head_size: int, rope_n: int, kc, vc, pos):
    """qkv split + RoPE with k / v written in place into the static caches ``kc`` / ``vc`` at rows
    ``pos`` (the decode step's ``index_copy_`` fused into the same launch).  Returns (q, kc, vc)."""
    lib = require()
    qkv = _c(qkv)
    B, T, _ = qkv.shape
    cos = _c(cos[:T])
    sin = _c(sin[:T])
    if cos.dtype != sin.dtype:
        sin = sin.to(cos.dtype)
    if cos.dtype not in (torch.float32, qkv.dtype):
        cos, sin = cos.float(), sin.float()
    q = torch.empty((B, n_head, T, head_size), device=qkv.device, dtype=qkv.dtype)
    st = (ctypes.c_int64 * 6)(*kc.stride()[:3], *vc.stride()[:3])
    rc = lib.lta_qkv_rope_cache_fwd(dcode(qkv), dcode(cos), ptr(qkv), ptr(cos), ptr(sin), ptr(q), ptr(kc), ptr(vc),
                                    ptr(pos), st, B, T, n_head, n_query_groups, head_size, rope_n,
                                    stream_ptr(qkv.device))
    check(rc, "lta_qkv_rope_cache_fwd")
    return q, kc, vc


def qkv_rope_bwd(dq, dk, dv, cos, sin, n_head: int, n_query_groups: int, head_size: int, rope_n: int):
    lib = require()
    dq, dk, dv = _c(dq), _c(dk), _c(dv)
    B, _, T, _ = dq.shape
    cos = _c(cos[:T])
    sin = _c(sin[:T])
    if cos.dtype != sin.dtype:
        sin = sin.to(cos.dtype)
    if cos.dtype not in (torch.float32, dq.dtype):
        cos, sin = cos.float(), sin.float()
    dqkv = torch.empty((B, T, (n_head + 2 * n_query_groups) * head_size), device=dq.device, dtype=dq.dtype)
    rc = lib.lta_qkv_rope_bwd(dcode(dq), dcode(cos), ptr(dq), ptr(dk), ptr(dv), ptr(cos), ptr(sin), ptr(dqkv), B, T,
                              n_head, n_query_groups, head_size, rope_n, stream_ptr(dq.device))
    check(rc, "lta_qkv_rope_bwd")
    return dqkv


def swiglu_fwd(a, b):
    lib = require()
    a, b = _c(a), _c(b)
    y = torch.empty_like(a)
    check(lib.lta_swiglu_fwd(dcode(a), ptr(a), ptr(b), ptr(y), a.numel(), stream_ptr(a.device)), "lta_swiglu_fwd")
    return y


def swiglu_bwd(g, a, b):
    lib = require()
    g, a, b = _c(g), _c(a), _c(b)
    da = torch.empty_like(a)
    db = torch.empty_like(b)
    check(lib.lta_swiglu_bwd(dcode(a), ptr(g), ptr(a), ptr(b), ptr(da), ptr(db), a.numel(), stream_ptr(a.device)),
          "lta_swiglu_bwd")
    return da, db


_REDUCTION = {"none": 0, "mean": 1, "sum": 2}


def _ce_weight(weight):
    return None if weight is None else _c(weight.to(torch.float32))


def cross_entropy_fwd(logits, target, ignore_index: int = -100, reduction: str = "mean", label_smoothing: float = 0.0,
                      weight=None):
    """Returns (loss [in logits dtype; per-row when reduction='none'], lse [rows] fp32, stats [2] fp32).
    ``weight``: optional [V] class weights (torch semantics: 'mean' divides by the kept rows' target
    weights; stats[1] holds that sum)."""
    lib = require()
    logits = _c(logits)
    target = _c(target.to(torch.int64))
    rows, V = logits.shape
    loss_rows = torch.empty(rows, device=logits.device, dtype=torch.float32)
    lse = torch.empty(rows, device=logits.device, dtype=torch.float32)
    stats = torch.empty(2, device=logits.device, dtype=torch.float32)
    r = _REDUCTION[reduction]
    w = _ce_weight(weight)
    check(lib.lta_ce_fwd_w(dcode(logits), ptr(logits), ptr(target), ptr(w), ptr(loss_rows), ptr(lse), ptr(stats), rows,
                           V, int(ignore_index), r, float(label_smoothing), stream_ptr(logits.device)), "lta_ce_fwd")
    if r == 0:
        loss = loss_rows.to(logits.dtype)
    else:
        loss = stats[0].to(logits.dtype)
    return loss, lse, stats


def ce_row_stats(logits, target_local, ignore_index: int = -100):
    """Per-row fp32 ``(lse, lse - x[target])`` of ``logits`` [rows, V] in ONE pass of the hand CE kernel
    (rows whose ``target_local`` is ``ignore_index`` get 0 in the second output) — the local half of
    a vocab-parallel cross-entropy."""
    lib = require()
    logits = _c(logits)
    target = _c(target_local.to(torch.int64))
    rows, V = logits.shape
    loss_rows = torch.empty(rows, device=logits.device, dtype=torch.float32)
    lse = torch.empty(rows, device=logits.device, dtype=torch.float32)
    check(lib.lta_ce_fwd_w(dcode(logits), ptr(logits), ptr(target), None, ptr(loss_rows), ptr(lse), None, rows, V,
                           int(ignore_index), 0, 0.0, stream_ptr(logits.device)), "lta_ce_fwd")
    return lse, loss_rows


def cross_entropy_bwd(g, logits, target, lse, stats, ignore_index: int = -100, reduction: str = "mean",
                      label_smoothing: float = 0.0, weight=None):
    lib = require()
    logits = _c(logits)
    target = _c(target.to(torch.int64))
    rows, V = logits.shape
    gs = _c(g.float().reshape(-1))
    dl = torch.empty_like(logits)
    w = _ce_weight(weight)
    check(lib.lta_ce_bwd_w(dcode(logits), ptr(logits), ptr(target), ptr(w), ptr(lse), ptr(gs), ptr(stats), ptr(dl), rows,
                           V, int(ignore_index), _REDUCTION[reduction], float(label_smoothing),
                           stream_ptr(logits.device)), "lta_ce_bwd")
    return dl
