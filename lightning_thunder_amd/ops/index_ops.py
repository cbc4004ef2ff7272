"""Python side of csrc/index_ops.hip: sort / argsort / topk / cumsum / index_add / embedding
backward on the HIP kernels (the reference's nvFuser/ATen coverage is
``thunder/executors/nvfuserex_impl.py`` embedding/index_put/scatter/topk/argsort/cumsum).

Every entry handles any ``dim`` by moving it last (one copy when it is not already the innermost
dimension) and returns tensors shaped like the torch op's.  The ``*_supported`` predicates state
each kernel's limits on real tensors; the HIP executor's checkers apply the same limits to proxies,
so a call these kernels cannot take stays on torch.
"""
from __future__ import annotations

import torch

from ._lib import require, stream_ptr, check, register_signature, c_int, c_int64, c_float, c_void_p

register_signature("lta_sort_rows", [c_int, c_void_p, c_int64, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p])
register_signature("lta_topk_rows", [c_int, c_void_p, c_int64, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p])
register_signature("lta_cumsum_rows", [c_int, c_void_p, c_int64, c_void_p, c_int, c_int64, c_int, c_void_p])
register_signature("lta_sort_index_keys", [c_void_p, c_int, c_void_p, c_void_p])
register_signature("lta_index_rows_sum", [c_int, c_void_p, c_int64, c_void_p, c_int, c_void_p, c_int64, c_void_p, c_int64,
                                          c_int64, c_int64, c_int64, c_int, c_float, c_void_p])

SORT_MAX = 16384  # keys per row that fit the LDS bitonic sort (lta_sort_max)
TOPK_WAVE_MAX = 2048  # row length of the one-wave-per-row top-k
_CODE = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2, torch.int32: 4, torch.int64: 5}
_SORT_DTYPES = (torch.float32, torch.float16, torch.bfloat16, torch.int32)
_ROW_DTYPES = (torch.float32, torch.float16, torch.bfloat16)


def _rows(x: torch.Tensor, dim: int):
    """x with ``dim`` moved last as a [R, N] view with unit inner stride (copy if needed)."""
    d = dim % x.ndim if x.ndim else 0
    xm = x.movedim(d, -1) if x.ndim else x.reshape(1)
    if xm.stride(-1) != 1 or not xm.is_contiguous():
        xm = xm.contiguous()
    n = xm.shape[-1]
    return xm.reshape(-1, n), xm.shape, d


def _back(t: torch.Tensor, lead_shape, d: int, ndim: int) -> torch.Tensor:
    t = t.reshape(*lead_shape[:-1], t.shape[-1])
    if ndim == 0:
        return t.reshape(())
    return t.movedim(-1, d).contiguous() if d != ndim - 1 else t


def sort_supported(x: torch.Tensor, dim: int) -> bool:
    lim = SORT_MAX // 2 if x.dtype == torch.int64 else SORT_MAX
    return (x.is_cuda and (x.dtype in _SORT_DTYPES or x.dtype == torch.int64) and x.numel() > 0
            and 1 <= (x.shape[dim] if x.ndim else 1) <= lim)


def sort(x: torch.Tensor, dim: int = -1, descending: bool = False, stable: bool = True):
    """Stable sort (ties keep their original order on every run; NaN sorts as the largest)."""
    x2, shp, d = _rows(x, dim)
    R, N = x2.shape
    vals = torch.empty((R, N), dtype=x.dtype, device=x.device)
    idx = torch.empty((R, N), dtype=torch.int64, device=x.device)
    check(require().lta_sort_rows(_CODE[x.dtype], x2.data_ptr(), x2.stride(0), vals.data_ptr(), idx.data_ptr(), R, N,
                                  N, int(bool(descending)), stream_ptr(x.device)), "lta_sort_rows")
    return _back(vals, shp, d, x.ndim), _back(idx, shp, d, x.ndim)


def argsort(x: torch.Tensor, dim: int = -1, descending: bool = False, stable: bool = True) -> torch.Tensor:
    return sort(x, dim, descending, stable)[1]


def topk_supported(x: torch.Tensor, k: int, dim: int) -> bool:
    if not (x.is_cuda and x.dtype in _SORT_DTYPES and x.numel() > 0 and x.ndim >= 1):
        return False
    n = x.shape[dim]
    return 1 <= k <= n and n <= SORT_MAX


def topk(x: torch.Tensor, k: int, dim: int = -1, largest: bool = True, sorted: bool = True):
    """Top-k along ``dim``, always sorted (largest first / smallest first), ties to the lower index.
    Rows of <= 2048 take the one-wave-per-row selection kernel (MoE routing shapes), longer rows
    the LDS sort."""
    x2, shp, d = _rows(x, dim)
    R, N = x2.shape
    vals = torch.empty((R, k), dtype=x.dtype, device=x.device)
    idx = torch.empty((R, k), dtype=torch.int64, device=x.device)
    lib = require()
    if N <= TOPK_WAVE_MAX and k <= 64:
        rc = lib.lta_topk_rows(_CODE[x.dtype], x2.data_ptr(), x2.stride(0), vals.data_ptr(), idx.data_ptr(), R, N, k,
                               int(bool(largest)), stream_ptr(x.device))
        check(rc, "lta_topk_rows")
    else:
        rc = lib.lta_sort_rows(_CODE[x.dtype], x2.data_ptr(), x2.stride(0), vals.data_ptr(), idx.data_ptr(), R, N, k,
                               int(bool(largest)), stream_ptr(x.device))
        check(rc, "lta_sort_rows")
    return _back(vals, shp, d, x.ndim), _back(idx, shp, d, x.ndim)


def cumsum_supported(x: torch.Tensor, dim: int, dtype=None) -> bool:
    if not x.is_cuda or x.numel() == 0 or x.numel() >= 2**31:
        return False
    if x.dtype in _ROW_DTYPES:
        return dtype in (None, x.dtype)
    return x.dtype in (torch.int32, torch.int64) and dtype in (None, torch.int64, torch.int32)


def cumsum(x: torch.Tensor, dim: int, dtype=None) -> torch.Tensor:
    """Inclusive scan along ``dim``: float inputs accumulate in fp32 and keep their dtype; integer
    inputs accumulate in int64 and give int64 (torch's promotion) or ``dtype=torch.int32``."""
    x2, shp, d = _rows(x, dim)
    R, N = x2.shape
    if x.dtype in (torch.int32, torch.int64):
        out_dtype = torch.int32 if dtype == torch.int32 else torch.int64
    else:
        out_dtype = x.dtype
    y = torch.empty((R, N), dtype=out_dtype, device=x.device)
    check(require().lta_cumsum_rows(_CODE[x.dtype], x2.data_ptr(), x2.stride(0), y.data_ptr(), R, N,
                                    int(out_dtype == torch.int32), stream_ptr(x.device)), "lta_cumsum_rows")
    return _back(y, shp, d, x.ndim)


def _sorted_index_keys(index: torch.Tensor) -> torch.Tensor:
    """(index << 32 | position) sorted ascending: the rows' contributions in position order."""
    idx = index.reshape(-1)
    if idx.dtype != torch.int64:
        idx = idx.to(torch.int64)
    idx = idx.contiguous()
    n = idx.numel()
    if n <= SORT_MAX:
        keys = torch.empty(n, dtype=torch.int64, device=index.device)
        check(require().lta_sort_index_keys(idx.data_ptr(), n, keys.data_ptr(), stream_ptr(index.device)),
              "lta_sort_index_keys")
        return keys
    # longer index lists: the composite keys are unique, so any sort gives the same order
    comp = (idx << 32) | torch.arange(n, device=index.device, dtype=torch.int64)
    return torch.sort(comp).values


def _aligned(t: torch.Tensor) -> torch.Tensor:
    return t if t.data_ptr() % 16 == 0 else t.clone()


def _rows_sum_ok(src: torch.Tensor, D: int) -> bool:
    vec = 16 // src.element_size()
    return src.dtype in _ROW_DTYPES and D % vec == 0


def embedding_backward_supported(grad: torch.Tensor, indices: torch.Tensor, num_weights: int, sparse: bool) -> bool:
    if sparse or not grad.is_cuda or grad.ndim < 1 or indices.dtype not in (torch.int32, torch.int64):
        return False
    D = grad.shape[-1]
    return (_rows_sum_ok(grad, D) and 0 < num_weights < 2**31 and indices.numel() < 2**31
            and indices.numel() * D == grad.numel())


def embedding_backward(grad: torch.Tensor, indices: torch.Tensor, num_weights: int, padding_idx: int = -1,
                       scale_grad_by_freq: bool = False) -> torch.Tensor:
    """Dense embedding weight gradient, deterministic: each weight row sums its tokens' gradient rows
    in token order (no float atomics), rows with no token and the padding row are zero."""
    D = grad.shape[-1]
    g2 = grad.reshape(-1, D)
    if g2.stride(1) != 1 or g2.stride(0) % (16 // g2.element_size()):
        g2 = g2.contiguous()
    g2 = _aligned(g2)
    keys = _sorted_index_keys(indices)
    out = torch.empty((num_weights, D), dtype=grad.dtype, device=grad.device)
    check(require().lta_index_rows_sum(_CODE[grad.dtype], g2.data_ptr(), g2.stride(0), keys.data_ptr(), keys.numel(),
                                       None, 0, out.data_ptr(), D, num_weights, D,
                                       padding_idx if padding_idx is not None and padding_idx >= 0 else -1,
                                       int(bool(scale_grad_by_freq)), 1.0, stream_ptr(grad.device)),
          "lta_index_rows_sum")
    return out


def index_add_supported(a: torch.Tensor, index: torch.Tensor, src: torch.Tensor, dim: int) -> bool:
    if not (a.is_cuda and a.ndim >= 1 and dim % a.ndim == 0 and a.dtype == src.dtype and index.ndim <= 1):
        return False
    if index.dtype not in (torch.int32, torch.int64) or src.ndim != a.ndim or a.numel() == 0:
        return False
    D = a.numel() // a.shape[0]
    return (_rows_sum_ok(a, D) and src.shape[1:] == a.shape[1:] and src.shape[0] == index.numel()
            and a.shape[0] < 2**31)


def index_add(a: torch.Tensor, index: torch.Tensor, src: torch.Tensor, alpha: float = 1.0) -> torch.Tensor:
    """``torch.index_add(a, 0, index, src, alpha=alpha)`` out of place, deterministic (contributions
    to one row added in index order, in fp32, then rounded once)."""
    V = a.shape[0]
    D = a.numel() // V
    a2 = _aligned(a.reshape(V, D).contiguous())
    s2 = _aligned(src.reshape(-1, D).contiguous())
    out = torch.empty_like(a2)
    if index.numel() == 0:
        out.copy_(a2)
        return out.reshape(a.shape)
    keys = _sorted_index_keys(index)
    check(require().lta_index_rows_sum(_CODE[a.dtype], s2.data_ptr(), D, keys.data_ptr(), keys.numel(), a2.data_ptr(),
                                       D, out.data_ptr(), D, V, D, -1, 0, float(alpha), stream_ptr(a.device)),
          "lta_index_rows_sum")
    return out.reshape(a.shape)
