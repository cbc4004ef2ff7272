"""Python bindings of the hand-written CDNA4 GEMMs (``csrc/gemm.hip``, K2)."""
from __future__ import annotations

import os as _os

import torch

import ctypes

from ._lib import require, stream_ptr, check, register_signature, dcode, c_int, c_void_p, c_float

ACT = {None: 0, "none": 0, "gelu_tanh": 1, "gelu": 2, "gelu_erf": 2, "silu": 3, "relu": 4}
TILE_M, TILE_N, TILE_K = 256, 256, 64

register_signature("lta_gemm_nt_bf16", [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                        c_int, c_int, c_int, c_float, c_int, c_void_p])
register_signature("lta_gemm_nt_bf16_v", [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                          c_int, c_int, c_int, c_float, c_int, c_int, c_void_p])


def _rowmajor_2d(t: torch.Tensor) -> bool:
    return t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0


def gemm_nt_supported(a: torch.Tensor, b: torch.Tensor, bias=None, residual=None) -> bool:
    """a [M,K] and b [N,K] bf16 on the GPU with tile-divisible shapes."""
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or not a.is_cuda:
        return False
    if not (_rowmajor_2d(a) and _rowmajor_2d(b)):
        return False
    M, K = a.shape
    N = b.shape[0]
    if M % TILE_M or N % TILE_N or K % TILE_K or b.shape[1] != K:
        return False
    if bias is not None and (bias.dtype != torch.bfloat16 or bias.numel() != N or not bias.is_contiguous()):
        return False
    if residual is not None and (residual.dtype != torch.bfloat16 or tuple(residual.shape) != (M, N)
                                 or not _rowmajor_2d(residual)):
        return False
    return True


def gemm_nt(a: torch.Tensor, b: torch.Tensor, *, bias=None, residual=None, act=None, alpha: float = 1.0,
            out: torch.Tensor | None = None, variant: int | None = None) -> torch.Tensor:
    """``act(alpha * a @ b.T + bias) + residual`` with the hand-written MFMA kernel.

    ``variant`` (``LTA_GEMM_VARIANT``): 0 (default) the 2-buffer glds loop, 1 the 8-phase pipelined
    loop (K % 128 == 0; 6-11 % slower on the Llama shapes, profiles/gemm_microbench.json)."""
    lib = require()
    M, K = a.shape
    N = b.shape[0]
    if variant is None:
        variant = int(_os.environ.get("LTA_GEMM_VARIANT", "0"))
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    rc = lib.lta_gemm_nt_bf16_v(a.data_ptr(), b.data_ptr(), out.data_ptr(),
                                None if bias is None else bias.data_ptr(),
                                None if residual is None else residual.data_ptr(), M, N, K, a.stride(0), b.stride(0),
                                out.stride(0), 0 if residual is None else residual.stride(0), alpha, ACT[act], variant,
                                stream_ptr(a.device))
    check(rc, "lta_gemm_nt_bf16")
    return out


# ---------------------------------------------------------------------------------------------
# linear with per-shape kernel selection
# ---------------------------------------------------------------------------------------------
import os as _os

_choice: dict = {}


def _timeit(fn, iters: int = 5) -> float:
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def _torch_linear(x2, w, bias, residual, act):
    y = torch.nn.functional.linear(x2, w, bias)
    if act == "gelu_tanh":
        y = torch.nn.functional.gelu(y, approximate="tanh")
    elif act in ("gelu", "gelu_erf"):
        y = torch.nn.functional.gelu(y)
    elif act == "silu":
        y = torch.nn.functional.silu(y)
    elif act == "relu":
        y = torch.relu(y)
    if residual is not None:
        y = y + residual
    return y


register_signature("lta_gemv_nt", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_float, c_void_p, c_void_p,
                                    c_void_p, c_int, c_int, c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                    ctypes.c_int64, c_int, c_void_p])
GEMV_MAX_M = 8


def gemv_supported(x: torch.Tensor, w: torch.Tensor, bias=None, residual=None) -> bool:
    """Decode-shaped linear: x [M <= 8, K] and w [N, K] (bf16/fp16, K % 8 == 0, 16-byte aligned rows)."""
    if x.dtype not in (torch.bfloat16, torch.float16) or w.dtype != x.dtype or not x.is_cuda:
        return False
    if x.dim() != 2 or w.dim() != 2 or not 1 <= x.shape[0] <= GEMV_MAX_M or w.shape[1] != x.shape[1]:
        return False
    if x.shape[1] % 8 or x.stride(1) != 1 or w.stride(1) != 1 or x.stride(0) % 8 or w.stride(0) % 8:
        return False
    if x.data_ptr() % 16 or w.data_ptr() % 16:
        return False
    if bias is not None and (bias.dtype != x.dtype or bias.numel() != w.shape[0] or not bias.is_contiguous()):
        return False
    if residual is not None and (residual.dtype != x.dtype or tuple(residual.shape) != (x.shape[0], w.shape[0])
                                 or residual.stride(1) != 1):
        return False
    return True


def gemv_nt(x: torch.Tensor, w: torch.Tensor, *, bias=None, residual=None, act=None, gate_weight=None,
            norm: bool = False, norm_weight=None, eps: float = 1e-5) -> torch.Tensor:
    """``act(x @ w.T + bias) + residual`` for M <= 8 rows with the weight-streaming kernel (``csrc/gemv.hip``).

    ``norm=True`` first replaces x by ``rmsnorm(x) * norm_weight``; ``gate_weight`` (same shape as w)
    makes the result ``act(x @ w.T) * (x @ gate_weight.T)`` (SwiGLU/GeGLU up-projection pair)."""
    lib = require()
    M, K = x.shape
    N = w.shape[0]
    if gate_weight is not None:
        assert gate_weight.shape == w.shape and gate_weight.stride() == w.stride() and bias is None and residual is None
    if norm_weight is not None:
        assert norm_weight.numel() == K and norm_weight.is_contiguous() and norm_weight.dtype == x.dtype
    out = torch.empty((M, N), dtype=x.dtype, device=x.device)
    rc = lib.lta_gemv_nt(dcode(x), x.data_ptr(), w.data_ptr(), None if gate_weight is None else gate_weight.data_ptr(),
                         None if norm_weight is None else norm_weight.data_ptr(), int(norm), float(eps),
                         None if bias is None else bias.data_ptr(), None if residual is None else residual.data_ptr(),
                         out.data_ptr(), M, N, K, x.stride(0), w.stride(0), out.stride(0),
                         0 if residual is None else residual.stride(0), ACT[act], stream_ptr(x.device))
    check(rc, "lta_gemv_nt")
    return out


def linear(x: torch.Tensor, w: torch.Tensor, bias=None, residual=None, act=None) -> torch.Tensor:
    """``act(x @ w.T + bias) + residual`` choosing, once per shape, the faster of the hand-written
    kernel (MFMA GEMM, or the weight-streaming GEMV for M <= 8; epilogue fused) and hipBLASLt +
    separate epilogue (``LTA_GEMM=hip|torch|auto``)."""
    K = x.shape[-1]
    N = w.shape[0]
    x2 = x.reshape(-1, K)
    r2 = None if residual is None else residual.reshape(-1, N)
    mode = _os.environ.get("LTA_GEMM", "auto")
    if mode != "torch" and gemv_supported(x2, w, bias, r2):
        return gemv_nt(x2, w, bias=bias, residual=r2, act=act).reshape(*x.shape[:-1], N)
    ok = gemm_nt_supported(x2, w, bias, r2)
    if not ok or mode == "torch":
        return _torch_linear(x2, w, bias, r2, act).reshape(*x.shape[:-1], N)
    key = (x2.shape[0], N, K, bias is not None, residual is not None, act)
    use = True if mode == "hip" else _choice.get(key)
    if use is None:
        if torch.cuda.is_current_stream_capturing():
            use = True
        else:
            t_h = _timeit(lambda: gemm_nt(x2, w, bias=bias, residual=r2, act=act))
            t_t = _timeit(lambda: _torch_linear(x2, w, bias, r2, act))
            use = t_h <= t_t
        _choice[key] = use
    if use:
        y = gemm_nt(x2, w, bias=bias, residual=r2, act=act)
    else:
        y = _torch_linear(x2, w, bias, r2, act)
    return y.reshape(*x.shape[:-1], N)


def selection_table() -> dict:
    """(M, N, K, bias, residual, act) -> True if the HIP kernel was selected."""
    return dict(_choice)


# ---------------------------------------------------------------------------------------------
# K10 grouped GEMM (mixture of experts)
# ---------------------------------------------------------------------------------------------
from ._lib import c_int64  # noqa: E402

register_signature("lta_gemm_grouped_nt_bf16", [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                                c_int64, c_void_p])


def grouped_nt_supported(a: torch.Tensor, b: torch.Tensor, offs: torch.Tensor) -> bool:
    """a [M, K]; b [G, K, N] given as the transpose of a K-contiguous [G, N, K] weight."""
    if not (a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.dim() == 2 and b.dim() == 3):
        return False
    G, K, N = b.shape
    if a.shape[1] != K or N % TILE_N or K % TILE_K or offs.dtype != torch.int32 or offs.numel() != G:
        return False
    return a.is_contiguous() and b.stride(1) == 1 and b.stride(2) == K and a.data_ptr() % 16 == 0


def grouped_mm(a: torch.Tensor, b: torch.Tensor, offs: torch.Tensor) -> torch.Tensor:
    """out[M, N] = a[rows of group g] @ b[g] (offs: int32 cumulative row ends)."""
    if not grouped_nt_supported(a, b, offs):
        return torch._grouped_mm(a, b, offs)
    lib = require()
    G, K, N = b.shape
    M = a.shape[0]
    out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    check(lib.lta_gemm_grouped_nt_bf16(a.data_ptr(), b.data_ptr(), out.data_ptr(), offs.data_ptr(), G, M, N, K,
                                       b.stride(0), stream_ptr(a.device)), "lta_gemm_grouped_nt_bf16")
    return out
