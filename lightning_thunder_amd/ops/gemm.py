"""Python bindings of the hand-written CDNA4 GEMMs (``csrc/gemm.hip``, K2)."""
from __future__ import annotations

import os as _os

import torch

import ctypes
import functools

from ._lib import require, stream_ptr, check, register_signature, dcode, c_int, c_void_p, c_float, c_int64

ACT = {None: 0, "none": 0, "gelu_tanh": 1, "gelu": 2, "gelu_erf": 2, "silu": 3, "relu": 4}
TILE_M, TILE_N, TILE_K = 256, 256, 64

register_signature("lta_gemm_nt_bf16", [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                        c_int, c_int, c_int, c_float, c_int, c_void_p])
register_signature("lta_gemm_nt_bf16_v", [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                          c_int, c_int, c_int, c_float, c_int, c_int, c_void_p])


def _rowmajor_2d(t: torch.Tensor) -> bool:
    return t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0


def gemm_nt_supported(a: torch.Tensor, b: torch.Tensor, bias=None, residual=None) -> bool:
    """a [M,K] and b [N,K] bf16 on the GPU with tile-divisible shapes (the 8-wave kernel)."""
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or not a.is_cuda:
        return False
    M, K = a.shape
    N = b.shape[0]
    if M % TILE_M or N % TILE_N or K % TILE_K:
        return False
    return nt_epilogue_ok(a, b, bias, residual)


def nt_epilogue_ok(a: torch.Tensor, b: torch.Tensor, bias=None, residual=None) -> bool:
    """Row-major a [M,K], b [N,K] and a bias / residual the NT epilogues read (bf16, contiguous)."""
    if not (_rowmajor_2d(a) and _rowmajor_2d(b)):
        return False
    M, K = a.shape
    N = b.shape[0]
    if b.shape[1] != K:
        return False
    # 16-byte vector bias loads in the epilogues and the split-K fixup: a bias view at an odd offset
    # (a slice of a fused qkv bias) takes the library path
    if bias is not None and (bias.dtype != torch.bfloat16 or bias.numel() != N or not bias.is_contiguous()
                             or bias.data_ptr() % 16):
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
# K2 v2: the 4-wave 256x256 kernel (csrc/gemm4.hip), every training layout through one entry
# ---------------------------------------------------------------------------------------------
register_signature("lta_gemm4_bf16", [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                      c_int, c_int, c_int, c_float, c_int, c_int, c_int, c_int, c_void_p])
register_signature("lta_gemm4_bf16_splitk", [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                             c_int, c_float, c_int, c_int, c_int, c_void_p, c_int64, c_void_p])
register_signature("lta_gemm4_bf16_ws", [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                         c_int, c_int, c_int, c_float, c_int, c_int, c_int, c_int, c_void_p, c_int64,
                                         c_void_p])

# wave-quantisation tail of plain products: the last partial wave (<= 128 of 256 CUs' tiles, e.g. the
# 1376-tile Llama-2-7B gate/up forward and wgrad) runs as two K halves per tile + an fp32 fixup
# (csrc/gemm4.hip launch4_tail); LTA_GEMM_TAIL_SPLIT=0 turns it off
_TAIL_SPLIT = _os.environ.get("LTA_GEMM_TAIL_SPLIT", "1") != "0"


_CUS: dict = {}
_WS: dict = {}


def _device_cus(device) -> int:
    """Compute units of ``device`` (the kernel reads the same attribute: hipDeviceAttributeMultiprocessorCount)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx not in _CUS:
        _CUS[idx] = int(torch.cuda.get_device_properties(idx).multi_processor_count)
    return _CUS[idx]


def _tail_workspace(M: int, N: int, K: int, device):
    if not _TAIL_SPLIT or K % 256:
        return None
    cus = _device_cus(device)
    nwg = -(-M // 256) * -(-N // 256)
    tail = nwg % cus
    if nwg <= cus or tail == 0 or 2 * tail > cus:
        return None
    return _workspace(2 * tail * 256 * 256, device)


# under-filled grids of plain products (at most half a wave of 256 x 256 tiles: the wgrad / dgrad of
# narrow layers, e.g. GPT-2-medium's d = 1024) split K over ksplit slices + an fp32 fixup
# (csrc/gemm4.hip launch4_splitk); LTA_GEMM_SPLITK=0 turns it off
_SPLITK = _os.environ.get("LTA_GEMM_SPLITK", "1") != "0"
# static cost model of the split (MI355X, profiles/gemm_splitk_gpt2.txt): a K-tile of a 256 x 256 tile
# takes ~1.3 us, prologue + epilogue ~4.5 us; every slice writes and the fixup reads a 256 KiB fp32
# partial per tile at ~5 TB/s; the fixup launch ~3 us
_KT_US, _FIXED_US, _PARTIAL_US, _LAUNCH_US = 1.3, 4.5, 2 * 262144 / 5e6, 3.0


@functools.lru_cache(maxsize=4096)
def splitk_factor(M: int, N: int, K: int, cus: int) -> int:
    """K slices per tile for a plain product (0: no split) whose grid is at most half a wave of
    ``cus`` workgroups: the slice count (grid <= one wave, >= one 128-deep K pair per slice) the
    cost model above rates fastest, if it beats the unsplit grid."""
    if not _SPLITK or K % 128:
        return 0
    nwg = -(-M // 256) * -(-N // 256)
    if 2 * nwg > cus:
        return 0
    pairs = K // 128
    best, best_t = 0, 2 * pairs * _KT_US + _FIXED_US
    for s in range(2, min(64, cus // nwg, pairs) + 1):
        t = 2 * -(-pairs // s) * _KT_US + _FIXED_US + nwg * s * _PARTIAL_US + _LAUNCH_US
        if t < best_t:
            best, best_t = s, t
    return best


def _workspace(need: int, device):
    """fp32 scratch of >= ``need`` elements: one cached buffer per (device, stream), grown to the largest
    request (its consumer, the fixup, runs right behind the producer on the same stream, so reuse is
    ordered); inside a graph capture a fresh allocation from the graph's pool (the graph keeps the
    pointer, which a later, larger request must never replace)."""
    if torch.cuda.is_current_stream_capturing():
        return torch.empty(need, dtype=torch.float32, device=device)
    key = (device.index, torch.cuda.current_stream(device).cuda_stream)
    ws = _WS.get(key)
    if ws is None or ws.numel() < need:
        ws = torch.empty(need, dtype=torch.float32, device=device)
        _WS[key] = ws
    return ws


GEMM4_MIN_M = 64
_FWD_LIB = _os.environ.get("LTA_GEMM_FWD_LIB", "0") == "1"


def gemm4_layout(a: torch.Tensor, b: torch.Tensor):
    """(at, bt, lda, ldb) of ``a [M,K] @ b [K,N]`` for ``lta_gemm4_bf16``, or None when the operands
    are not bf16 2-D GPU tensors with one unit-stride dim and 16-B aligned rows, or K % 128 != 0.
    M and N need not divide the 256 x 256 tile (edge tiles clamp their operand rows and mask their
    stores; N % 8 == 0 for whole 16-B output chunks); M < GEMM4_MIN_M goes elsewhere (a 256-row
    tile would be mostly idle)."""
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or not a.is_cuda or a.dim() != 2 or b.dim() != 2:
        return None
    M, K = a.shape
    N = b.shape[1]
    if b.shape[0] != K or M < GEMM4_MIN_M or N % 8 or K % 128 or N == 0 or K == 0:
        return None
    la, lb = _operand_layout(a, M, K), _operand_layout(b, K, N)
    if la is None or lb is None:
        return None
    at = 0 if la[0] == 1 else 1
    bt = 1 if lb[0] == 1 else 0
    if at and M % 8:  # an MN-major A is staged in 16-B row pieces (the kernel returns -2 otherwise)
        return None
    # 32-bit buffer offsets
    if (K if at else M) * la[1] * 2 >= 2 ** 31 or (K if bt else N) * lb[1] * 2 >= 2 ** 31:
        return None
    return at, bt, la[1], lb[1]


def matmul4(a: torch.Tensor, b: torch.Tensor, *, bias=None, residual=None, act=None, alpha: float = 1.0,
            out: torch.Tensor | None = None, variant: int = 1) -> torch.Tensor:
    """``act(alpha * a @ b + bias) + residual`` on the 4-wave MFMA kernel.  ``a``/``b`` may be
    transposed views (the backward GEMMs read dY^T / W / X in place); bias and act only for the
    forward layout (a row-major, b = W^T)."""
    lay = gemm4_layout(a, b)
    if lay is None:
        raise ValueError(f"matmul4: unsupported operands {tuple(a.shape)}{a.stride()} @ {tuple(b.shape)}{b.stride()}")
    at, bt, lda, ldb = lay
    M, K = a.shape
    N = b.shape[1]
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    if residual is not None:
        assert residual.shape == (M, N) and residual.stride(1) == 1 and residual.dtype == torch.bfloat16
    if bias is not None:
        assert bias.dtype == torch.bfloat16 and bias.numel() == N and bias.is_contiguous()
        bias = _aligned_bias(bias)
    plain = bias is None and residual is None and act is None and variant == 1
    # the K split also carries a bias (added in the fixup, forward layout)
    splittable = residual is None and act is None and variant == 1 and (
        bias is None or (not at and not bt and bias.data_ptr() % 16 == 0))
    ks = splitk_factor(M, N, K, _device_cus(a.device)) if splittable else 0
    if ks:
        nwg = -(-M // 256) * -(-N // 256)
        ws = _workspace(ks * nwg * 256 * 256, a.device)
        rc = require().lta_gemm4_bf16_splitk(a.data_ptr(), b.data_ptr(), out.data_ptr(),
                                             None if bias is None else bias.data_ptr(), M, N, K, lda, ldb,
                                             out.stride(0), alpha, at, bt, ks, ws.data_ptr(), ws.numel() * 4,
                                             stream_ptr(a.device))
        check(rc, "lta_gemm4_bf16_splitk")
        return out
    ws = _tail_workspace(M, N, K, a.device) if plain else None
    if ws is not None:
        rc = require().lta_gemm4_bf16_ws(a.data_ptr(), b.data_ptr(), out.data_ptr(), None, None, M, N, K, lda, ldb,
                                         out.stride(0), 0, alpha, ACT[act], at, bt, variant, ws.data_ptr(),
                                         ws.numel() * 4, stream_ptr(a.device))
        check(rc, "lta_gemm4_bf16_ws")
        return out
    rc = require().lta_gemm4_bf16(a.data_ptr(), b.data_ptr(), out.data_ptr(),
                                  None if bias is None else bias.data_ptr(),
                                  None if residual is None else residual.data_ptr(), M, N, K, lda, ldb, out.stride(0),
                                  0 if residual is None else residual.stride(0), alpha, ACT[act], at, bt, variant,
                                  stream_ptr(a.device))
    check(rc, "lta_gemm4_bf16")
    return out


# ---------------------------------------------------------------------------------------------
# linear / matmul dispatch (static rules, no run-time timing)
# ---------------------------------------------------------------------------------------------

# Library GEMM solutions pre-selected on MI355X for the shapes of the Llama-2-7B training step
# (PyTorch TunableOp results: rocBLAS / hipBLASLt solution per (layout, M, N, K), measured with
# rotating buffers on random data by scripts/tunable_probe.py on this image).  OPT-IN
# (``LTA_TUNED_GEMMS=1``): TunableOp is a process-wide switch that also changes every GEMM of user
# code, so the framework never turns it on by itself; the hand-written kernels (csrc/gemm4.hip)
# are the default GEMM path.  When enabled, the shipped table is read first and TunableOp is
# switched on only if the table matched this stack (validators: PyTorch / HIP / rocBLAS / hipBLASLt
# versions, arch); tuning and write-on-exit stay off.
TUNED_GEMMS = _os.path.join(_os.path.dirname(__file__), "tuned", "gemm_mi355x_bf16.csv")
_tuned_state: dict = {}


def enable_tuned_gemms() -> bool:
    """Load the shipped TunableOp results once per process when ``LTA_TUNED_GEMMS=1``.  Returns
    whether they are active; on any mismatch TunableOp's state is left exactly as it was."""
    if "active" in _tuned_state:
        return _tuned_state["active"]
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        return False  # never switch TunableOp on inside a graph capture; the next eager call will
    active = False
    tun = getattr(torch.cuda, "tunable", None)
    if (_os.environ.get("LTA_TUNED_GEMMS", "0") == "1" and torch.version.hip is not None and tun is not None
            and _os.path.exists(TUNED_GEMMS) and torch.cuda.is_available()):
        prev = None
        try:
            prev = (tun.is_enabled(), tun.tuning_is_enabled())
            if tun.read_file(TUNED_GEMMS):
                if hasattr(tun, "write_file_on_exit"):
                    tun.write_file_on_exit(False)
                tun.tuning_enable(False)
                tun.enable(True)
                active = True
        except Exception:  # an older/newer stack without the API: library defaults
            active = False
        if not active and prev is not None:
            try:
                tun.enable(prev[0])
                tun.tuning_enable(prev[1])
            except Exception:
                pass
    _tuned_state["active"] = active
    return active


def _torch_linear(x2, w, bias, residual, act):
    if residual is not None and act is None and bias is None and x2.dim() == 2:
        return torch.addmm(residual, x2, w.t())  # hipBLASLt with beta = 1: the add rides in the GEMM
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


register_signature("lta_gemv_group", [c_int, c_void_p, c_void_p, c_int, c_float, c_int, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_int, c_int, ctypes.c_int64, c_void_p])


def gemv_group(x: torch.Tensor, weights, *, norm: bool = False, norm_weight=None, eps: float = 1e-5,
               packed: bool = False):
    """``[x' @ w.T for w in weights]`` (<= 3 weights sharing x, e.g. attention q / k / v) in ONE
    weight-streaming launch; ``x' = rmsnorm(x) * norm_weight`` when ``norm``.  ``packed``: the
    outputs are adjacent column ranges of one [M, sum N] tensor (returned alone), e.g. the fused
    qkv row a RoPE kernel splits."""
    assert 1 <= len(weights) <= 3
    lib = require()
    M, K = x.shape
    if packed:
        total = sum(w.shape[0] for w in weights)
        buf = torch.empty((M, total), dtype=x.dtype, device=x.device)
        outs, off = [], 0
        for w in weights:
            outs.append(buf[:, off:off + w.shape[0]])
            off += w.shape[0]
    else:
        outs = [torch.empty((M, w.shape[0]), dtype=x.dtype, device=x.device) for w in weights]
    n = len(weights)
    ws = (ctypes.c_void_p * 3)(*[w.data_ptr() for w in weights], *([None] * (3 - n)))
    ys = (ctypes.c_void_p * 3)(*[o.data_ptr() for o in outs], *([None] * (3 - n)))
    ns = (ctypes.c_int * 3)(*[w.shape[0] for w in weights], *([0] * (3 - n)))
    ldw = (ctypes.c_int64 * 3)(*[w.stride(0) for w in weights], *([0] * (3 - n)))
    ldy = (ctypes.c_int64 * 3)(*[o.stride(0) for o in outs], *([0] * (3 - n)))
    rc = lib.lta_gemv_group(dcode(x), x.data_ptr(), None if norm_weight is None else norm_weight.data_ptr(), int(norm),
                            float(eps), n, ctypes.cast(ws, c_void_p), ctypes.cast(ys, c_void_p), ctypes.cast(ns, c_void_p),
                            ctypes.cast(ldw, c_void_p), ctypes.cast(ldy, c_void_p), M, K, x.stride(0),
                            stream_ptr(x.device))
    check(rc, "lta_gemv_group")
    return buf if packed else outs


_backend_counts: dict = {}


def _count(backend: str) -> None:
    _backend_counts[backend] = _backend_counts.get(backend, 0) + 1


def last_gemm_backend_counts(reset: bool = False) -> dict:
    """How many GEMM calls each backend served since the last reset: ``gemm4`` (csrc/gemm4.hip),
    ``gemm`` (csrc/gemm.hip, K % 128 != 0), ``gemv`` (decode rows), ``torch`` (library fallback:
    shapes no hand kernel tiles, or ``LTA_GEMM=torch``)."""
    out = dict(_backend_counts)
    if reset:
        _backend_counts.clear()
    return out


def gemm4_variant(at: int, bt: int, M: int, N: int, K: int) -> int:
    """Static, deterministic kernel-variant table (no run-time timing: every process runs the same
    kernels, so numerics never depend on a benchmark's noise).  Variant = the LDS-DMA split of
    csrc/gemm4.hip (how many of a K-tile's 16 LDS-DMA loads issue in the second half of the previous
    tile).  Variant 1 (8 / 8) is the fastest or within 1 % of it on all 18 Llama-2-7B training GEMMs
    in profiles/gemm4_microbench.json; a measured row below overrides it for one shape."""
    return _GEMM4_VARIANTS.get((at, bt, N, K), _GEMM4_VARIANTS.get((at, bt), 1))


# (at, bt[, N, K]) -> variant (profiles/gemm4_microbench.json)
_GEMM4_VARIANTS: dict = {}


# ---------------------------------------------------------------------------------------------
# launch plans: the dispatch decision of a GEMM call site depends only on its operands' shapes,
# strides, dtypes, 16-B alignment and the LTA_GEMM mode, which a compiled program repeats on every
# call; the plan caches that decision with the kernel's scalar arguments, so a repeated call costs the
# output allocation and one native launch (the host path of launch-bound programs, benchmarks/targets.py)
# ---------------------------------------------------------------------------------------------
_PLANS: dict = {}
_NO_PLAN = object()


def _remember(key, plan) -> None:
    if len(_PLANS) >= 8192:  # bounded: a program seeing ever new sizes re-dispatches instead of growing
        _PLANS.clear()
    _PLANS[key] = plan or _NO_PLAN


def _aligned_bias(bias):
    """The kernels read the bias with 8- / 16-byte vector loads (gemm4 epilogue, split-K fixup): a
    bias view at an element offset that is not a multiple of 8 (a slice of a fused qkv bias) is
    copied to a fresh, aligned buffer (N elements) instead of being read misaligned."""
    if bias is not None and bias.is_cuda and bias.data_ptr() % 16:
        return bias.contiguous().clone()
    return bias


def _tkey(t):
    return None if t is None else (t.shape, t.stride(), t.dtype, t.data_ptr() & 15)


def _gemm4_plan(M: int, N: int, K: int, lda: int, ldb: int, at: int, bt: int, variant: int, act_code: int,
                has_bias: bool, has_res: bool, ldr: int, out_shape, dev):
    """A plain / bias / residual / activation gemm4 launch (no K split, no tail split) as a closure."""
    fn = require().lta_gemm4_bf16
    bf16 = torch.bfloat16

    def run(a, b, bias, residual):
        _backend_counts["gemm4"] = _backend_counts.get("gemm4", 0) + 1
        out = torch.empty(out_shape, dtype=bf16, device=dev)
        rc = fn(a.data_ptr(), b.data_ptr(), out.data_ptr(), bias.data_ptr() if has_bias else None,
                residual.data_ptr() if has_res else None, M, N, K, lda, ldb, N, ldr, 1.0, act_code, at, bt, variant,
                stream_ptr(dev))
        if rc != 0:
            check(rc, "lta_gemm4_bf16")
        return out

    return run


def _gemm4_plain_plan(M, N, K, at, bt, lda, ldb, variant, bias, residual, act, out_shape, dev):
    """The plan of a gemm4 product, or None when this call takes a K split / tail split (workspace per call)."""
    plain = bias is None and residual is None and act is None and variant == 1
    splittable = residual is None and act is None and variant == 1 and (
        bias is None or (not at and not bt and bias.data_ptr() % 16 == 0))
    if splittable and splitk_factor(M, N, K, _device_cus(dev)):
        return None
    if plain and _TAIL_SPLIT and K % 256 == 0:
        cus = _device_cus(dev)
        nwg = -(-M // 256) * -(-N // 256)
        tail = nwg % cus
        if not (nwg <= cus or tail == 0 or 2 * tail > cus):
            return None
    return _gemm4_plan(M, N, K, lda, ldb, at, bt, variant, ACT[act], bias is not None, residual is not None,
                       0 if residual is None else residual.stride(0), out_shape, dev)


def linear(x: torch.Tensor, w: torch.Tensor, bias=None, residual=None, act=None) -> torch.Tensor:
    """``act(x @ w.T + bias) + residual`` on the hand-written kernels, chosen by a static rule:
    the weight-streaming GEMV for <= 8 rows, the 4-wave MFMA GEMM (csrc/gemm4.hip, any M >= 64,
    N % 8, K % 128: edge tiles), the 8-wave kernel (csrc/gemm.hip) when tile-divisible with K % 64,
    else torch (``LTA_GEMM=torch`` forces torch).  Repeated call sites run a cached launch plan."""
    bias = _aligned_bias(bias)
    key = ("lin", _tkey(x), _tkey(w), _tkey(bias), _tkey(residual), act, x.get_device(),
           _os.environ.get("LTA_GEMM", "auto"))
    plan = _PLANS.get(key)
    if plan is not None and plan is not _NO_PLAN and x.is_cuda:
        return plan(x, w, bias, residual)
    out = _linear_dispatch(x, w, bias, residual, act)
    if plan is None and x.is_cuda and not torch.cuda.is_current_stream_capturing():
        _remember(key, _linear_plan(x, w, bias, residual, act))
    return out


def _linear_plan(x, w, bias, residual, act):
    """The cached form of :func:`_linear_dispatch` for this call's operands (gemm4 launches only)."""
    if _os.environ.get("LTA_GEMM", "auto") == "torch":
        return None
    K = x.shape[-1]
    N = w.shape[0]
    x2 = x.reshape(-1, K)
    r2 = None if residual is None else residual.reshape(-1, N)
    if gemv_supported(x2, w, bias, r2):
        return None
    if _FWD_LIB and act is None and bias is None and x2.shape[0] >= 1024 and x2.dtype == torch.bfloat16:
        return None
    wt = w.t()
    lay = gemm4_layout(x2, wt)
    if lay is None or not nt_epilogue_ok(x2, w, bias, r2):
        return None
    at, bt, lda, ldb = lay
    M = x2.shape[0]
    if x2.data_ptr() != x.data_ptr() or (r2 is not None and r2.data_ptr() != residual.data_ptr()):
        return None  # a reshape that copied: the plan launches on the caller's tensors
    return _gemm4_plain_plan(M, N, K, at, bt, lda, ldb, gemm4_variant(0, 0, M, N, K), bias, r2, act,
                             tuple(x.shape[:-1]) + (N,), x.device)


def _linear_dispatch(x: torch.Tensor, w: torch.Tensor, bias=None, residual=None, act=None) -> torch.Tensor:
    K = x.shape[-1]
    N = w.shape[0]
    x2 = x.reshape(-1, K)
    r2 = None if residual is None else residual.reshape(-1, N)
    mode = _os.environ.get("LTA_GEMM", "auto")
    if mode != "torch":
        if gemv_supported(x2, w, bias, r2):
            _count("gemv")
            return gemv_nt(x2, w, bias=bias, residual=r2, act=act).reshape(*x.shape[:-1], N)
        if _FWD_LIB and act is None and bias is None and x2.shape[0] >= 1024 and x2.dtype == torch.bfloat16:
            # A/B hook: forward products with no epilogue but the residual on the library GEMM
            _count("torch")
            return _torch_linear(x2, w, bias, r2, act).reshape(*x.shape[:-1], N)
        wt = w.t()
        lay = gemm4_layout(x2, wt)
        if lay is not None and nt_epilogue_ok(x2, w, bias, r2):
            _count("gemm4")
            y = matmul4(x2, wt, bias=bias, residual=r2, act=act, variant=gemm4_variant(0, 0, x2.shape[0], N, K))
            return y.reshape(*x.shape[:-1], N)
        if gemm_nt_supported(x2, w, bias, r2):
            _count("gemm")
            return gemm_nt(x2, w, bias=bias, residual=r2, act=act).reshape(*x.shape[:-1], N)
    _count("torch")
    return _torch_linear(x2, w, bias, r2, act).reshape(*x.shape[:-1], N)


# ---------------------------------------------------------------------------------------------
# general-layout bf16 matmul (the backward GEMMs: dgrad = g @ W, wgrad = g^T @ x)
# ---------------------------------------------------------------------------------------------
register_signature("lta_gemm_bf16_layout", [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                            c_int, c_int, c_float, c_int, c_int, c_void_p])


def _operand_layout(t: torch.Tensor, rows: int, cols: int):
    """(contiguous dim, pitch) of a 2-D [rows, cols] operand with 16-byte aligned rows, or None."""
    if t.dim() != 2 or t.data_ptr() % 16:
        return None
    s0, s1 = t.stride()
    if s1 == 1 and s0 % 8 == 0 and s0 >= cols:
        return 1, s0
    if s0 == 1 and s1 % 8 == 0 and s1 >= rows:
        return 0, s1
    return None


def matmul_layout(a: torch.Tensor, b: torch.Tensor):
    """(at, bt, lda, ldb) of ``a [M,K] @ b [K,N]`` for ``lta_gemm_bf16_layout``, or None."""
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or not a.is_cuda or a.dim() != 2 or b.dim() != 2:
        return None
    M, K = a.shape
    N = b.shape[1]
    if b.shape[0] != K or M % TILE_M or N % TILE_N or K % TILE_K:
        return None
    la, lb = _operand_layout(a, M, K), _operand_layout(b, K, N)
    if la is None or lb is None:
        return None
    at = 0 if la[0] == 1 else 1  # a row-major [M][K] -> K-major; column-major -> stored [K][M]
    bt = 1 if lb[0] == 1 else 0  # b row-major [K][N] -> stored [K][N]; column-major -> [N][K]
    return at, bt, la[1], lb[1]


def matmul_hip(a: torch.Tensor, b: torch.Tensor, *, residual: torch.Tensor | None = None,
               out: torch.Tensor | None = None) -> torch.Tensor:
    """``a @ b (+ residual)`` on the MFMA kernel, reading transposed operands through the
    hardware-transposing LDS read instead of materialising them (2-D bf16, tile-divisible)."""
    lay = matmul_layout(a, b)
    if lay is None:
        raise ValueError(f"matmul_hip: unsupported operands {tuple(a.shape)}{a.stride()} @ {tuple(b.shape)}{b.stride()}")
    at, bt, lda, ldb = lay
    M, K = a.shape
    N = b.shape[1]
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    if residual is not None:
        assert residual.shape == (M, N) and residual.stride(1) == 1 and residual.dtype == torch.bfloat16
    rc = require().lta_gemm_bf16_layout(a.data_ptr(), b.data_ptr(), out.data_ptr(),
                                        None if residual is None else residual.data_ptr(), M, N, K, lda, ldb,
                                        out.stride(0), 0 if residual is None else residual.stride(0), 1.0, at, bt,
                                        stream_ptr(a.device))
    check(rc, "lta_gemm_bf16_layout")
    return out


def _torch_mm(a, b, residual=None):
    return torch.matmul(a, b) if residual is None else torch.addmm(residual, a, b)


def matmul(a: torch.Tensor, b: torch.Tensor, residual: torch.Tensor | None = None) -> torch.Tensor:
    """``a @ b (+ residual)`` for the prim matmul (leading dims of ``a`` flattened) — the backward's
    dgrad / wgrad read their transposed operands in place.  Static rule as :func:`linear`: the
    4-wave kernel, else the 8-wave kernel, else torch.  Repeated call sites run a cached launch plan."""
    key = ("mm", _tkey(a), _tkey(b), _tkey(residual), a.get_device(), _os.environ.get("LTA_GEMM", "auto"))
    plan = _PLANS.get(key)
    if plan is not None and plan is not _NO_PLAN and a.is_cuda:
        return plan(a, b, None, residual)
    out = _matmul_dispatch(a, b, residual)
    if plan is None and a.is_cuda and not torch.cuda.is_current_stream_capturing():
        _remember(key, _matmul_plan(a, b, residual))
    return out


def _matmul_plan(a, b, residual):
    if _os.environ.get("LTA_GEMM", "auto") == "torch" or b.dim() != 2 or a.dim() < 2:
        return None
    a2 = a.reshape(-1, a.shape[-1]) if a.dim() > 2 else a
    if a2.data_ptr() != a.data_ptr():
        return None
    N = b.shape[1]
    r2 = None if residual is None else residual.reshape(-1, N)
    if r2 is not None and r2.data_ptr() != residual.data_ptr():
        return None
    if r2 is not None and not (r2.dtype == torch.bfloat16 and r2.stride(1) == 1 and r2.stride(0) % 8 == 0
                               and r2.data_ptr() % 16 == 0):
        return None
    lay = gemm4_layout(a2, b)
    if lay is None:
        return None
    at, bt, lda, ldb = lay
    M, K = a2.shape
    return _gemm4_plain_plan(M, N, K, at, bt, lda, ldb, gemm4_variant(at, bt, M, N, K), None, r2, None,
                             tuple(a.shape[:-1]) + (N,), a.device)


def _matmul_dispatch(a: torch.Tensor, b: torch.Tensor, residual: torch.Tensor | None = None) -> torch.Tensor:
    if a.dim() > 2 and b.dim() == 2:
        lead = a.shape[:-1]
        a2 = a.reshape(-1, a.shape[-1])
        r2 = None if residual is None else residual.reshape(-1, b.shape[1])
        return _matmul_dispatch(a2, b, r2).reshape(*lead, b.shape[1])
    mode = _os.environ.get("LTA_GEMM", "auto")
    res_ok = residual is None or (residual.dtype == torch.bfloat16 and residual.stride(1) == 1
                                  and residual.stride(0) % 8 == 0 and residual.data_ptr() % 16 == 0)
    if mode != "torch" and res_ok:
        lay = gemm4_layout(a, b)
        if lay is not None:
            _count("gemm4")
            return matmul4(a, b, residual=residual,
                           variant=gemm4_variant(lay[0], lay[1], a.shape[0], b.shape[1], a.shape[1]))
        if matmul_layout(a, b) is not None:
            _count("gemm")
            return matmul_hip(a, b, residual=residual)
    _count("torch")
    return _torch_mm(a, b, residual)


# ---------------------------------------------------------------------------------------------
# K10 grouped GEMM (mixture of experts)
# ---------------------------------------------------------------------------------------------
from ._lib import c_int64  # noqa: E402

register_signature("lta_gemm_grouped_nt_bf16", [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                                c_int64, c_void_p])


register_signature("lta_gemm4_grouped", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                         c_int, c_int, c_int, ctypes.c_int64, ctypes.c_int64, c_int, c_void_p])


def grouped_nt_supported(a: torch.Tensor, b: torch.Tensor, offs: torch.Tensor) -> bool:
    """a [M, K]; b [G, K, N] given as the transpose of a K-contiguous [G, N, K] weight."""
    if not (a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.dim() == 2 and b.dim() == 3):
        return False
    G, K, N = b.shape
    if a.shape[1] != K or N % TILE_N or K % TILE_K or offs.dtype != torch.int32 or offs.numel() != G:
        return False
    return a.is_contiguous() and b.stride(1) == 1 and b.stride(2) == K and a.data_ptr() % 16 == 0


def _grouped_b_layout(b: torch.Tensor):
    """(bt, ldb) of a [G, K, N] grouped operand read per group as [K][N]: bt = 0 when each group is
    stored [N][K] (K contiguous: an nn.Linear-style expert weight viewed transposed), 1 when stored
    [K][N] (N contiguous: the dgrad's W_g); None otherwise."""
    G, K, N = b.shape
    if b.data_ptr() % 16:
        return None
    if b.stride(1) == 1 and b.stride(2) % 8 == 0 and b.stride(2) >= K:
        return 0, b.stride(2)
    if b.stride(2) == 1 and b.stride(1) % 8 == 0 and b.stride(1) >= N:
        return 1, b.stride(1)
    return None


def grouped_rows_supported(a: torch.Tensor, b: torch.Tensor, offs: torch.Tensor) -> bool:
    """The 2-D x 3-D grouped form on the 4-wave kernel (mode 1): a [M, K] row-major, b [G, K, N] in
    either per-group layout, K % 128, N % 8."""
    if not (a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.dim() == 2 and b.dim() == 3):
        return False
    G, K, N = b.shape
    if a.shape[1] != K or K % 128 or N % 8 or offs is None or offs.dtype != torch.int32 or offs.numel() != G:
        return False
    if not (a.stride(1) == 1 and a.stride(0) % 8 == 0 and a.data_ptr() % 16 == 0):
        return False
    return _grouped_b_layout(b) is not None and b.stride(0) * G * 2 < 2 ** 62


def grouped_mm(a: torch.Tensor, b: torch.Tensor, offs: torch.Tensor) -> torch.Tensor:
    """MoE grouped GEMM (``torch._grouped_mm`` semantics), on hand kernels when the layout allows:
      * a [M, K] @ b [G, K, N] -> [M, N]: rows [offs[g-1], offs[g]) of ``a`` times ``b[g]`` (forward,
        and the dgrad ``dY @ W_g`` whose b is the expert weight itself);
      * a [K, M] @ b [M, N] -> [G, K, N]: per group the product over its rows (the wgrad
        ``x_g^T dY_g``), written straight in the expert weight's [G, N, K] layout and returned as
        its transposed view;
    ``offs``: int32 cumulative row ends."""
    if a.dim() == 2 and b.dim() == 2:
        return grouped_mm_wgrad(a, b, offs)
    if grouped_rows_supported(a, b, offs):
        G, K, N = b.shape
        M = a.shape[0]
        bt, ldb = _grouped_b_layout(b)
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
        _count("gemm4")
        check(require().lta_gemm4_grouped(1, a.data_ptr(), b.data_ptr(), out.data_ptr(), offs.data_ptr(), G, M, N, K,
                                          a.stride(0), ldb, N, b.stride(0), 0, bt, stream_ptr(a.device)),
              "lta_gemm4_grouped")
        return out
    if grouped_nt_supported(a, b, offs):
        lib = require()
        G, K, N = b.shape
        M = a.shape[0]
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
        _count("gemm")
        check(lib.lta_gemm_grouped_nt_bf16(a.data_ptr(), b.data_ptr(), out.data_ptr(), offs.data_ptr(), G, M, N, K,
                                           b.stride(0), stream_ptr(a.device)), "lta_gemm_grouped_nt_bf16")
        return out
    _count("torch")
    return torch._grouped_mm(a, b, offs)


def grouped_wgrad_supported(a: torch.Tensor, b: torch.Tensor, offs: torch.Tensor) -> bool:
    """a [K, M] viewed from a row-major [M, K] (token rows), b [M, N] row-major."""
    if not (a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.dim() == 2 and b.dim() == 2):
        return False
    K, M = a.shape
    N = b.shape[1]
    if b.shape[0] != M or K % 8 or N % 8 or offs is None or offs.dtype != torch.int32:
        return False
    return (a.stride(0) == 1 and a.stride(1) % 8 == 0 and b.stride(1) == 1 and b.stride(0) % 8 == 0
            and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0)


def grouped_mm_wgrad(a: torch.Tensor, b: torch.Tensor, offs: torch.Tensor) -> torch.Tensor:
    """[G, K, N] = per group g: a[:, rows of g] @ b[rows of g] — the MoE wgrad.  Computed as
    C'[g] = b_g^T a_g^T, i.e. [G][N][K] (the expert weight's own layout, so its gradient needs no
    transposing copy) on the 4-wave kernel's grouped-reduction mode, returned transposed."""
    if not grouped_wgrad_supported(a, b, offs):
        _count("torch")
        return torch._grouped_mm(a, b, offs)
    K, M = a.shape
    N = b.shape[1]
    G = offs.numel()
    out = torch.empty((G, N, K), dtype=torch.bfloat16, device=a.device)
    _count("gemm4")
    # C'[g] [N][K] = b_g^T . a_g^T: A operand = b stored [rows][N] (at = 1), B operand = a's storage
    # [rows][K] (bt = 1)
    check(require().lta_gemm4_grouped(2, b.data_ptr(), a.data_ptr(), out.data_ptr(), offs.data_ptr(), G, N, K, M,
                                      b.stride(0), a.stride(1), K, 0, N * K, 1, stream_ptr(a.device)),
          "lta_gemm4_grouped")
    return out.transpose(1, 2)


# ---------------------------------------------------------------------------------------------
# fused SwiGLU GEMMs (csrc/gemm4.hip lta_gemm4_swiglu): the LLaMA MLP gate/up pair and its backward
# ---------------------------------------------------------------------------------------------
register_signature("lta_gemm4_swiglu", [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p])


def _fused_swiglu_on() -> bool:
    """SwiGLU in the GEMM epilogues is OPT-IN (``LTA_FUSED_SWIGLU=1``): measured on the Llama-2-7B
    step (profiles/fused_epilogue_ab.txt: 169.3 ms fused vs 168.4 ms unfused) the
    one-workgroup-per-CU kernel exposes its epilogue, and the third output (gate-up: 581 us per layer)
    or the per-tile a / b loads (down-projection dgrad + swiglu backward: 382 us per layer) cost about
    what the separate streaming passes they remove cost."""
    return _os.environ.get("LTA_FUSED_SWIGLU", "0") == "1"


def _plain_2d(t: torch.Tensor) -> bool:
    return (t.dim() == 2 and t.dtype == torch.bfloat16 and t.is_cuda and t.stride(1) == 1 and t.stride(0) % 8 == 0
            and t.data_ptr() % 16 == 0)


def gate_up_supported(x2: torch.Tensor, w1: torch.Tensor, w2: torch.Tensor) -> bool:
    if _os.environ.get("LTA_GEMM", "auto") == "torch" or not _fused_swiglu_on():
        return False
    if not (_plain_2d(x2) and _plain_2d(w1) and _plain_2d(w2)) or w1.shape != w2.shape or w1.stride() != w2.stride():
        return False
    M, K = x2.shape
    Nh = w1.shape[0]
    return (w1.shape[1] == K and M >= GEMM4_MIN_M and Nh % 128 == 0 and K % 128 == 0 and Nh > 0
            and M * x2.stride(0) * 2 < 2 ** 31 and Nh * w1.stride(0) * 2 < 2 ** 31)


def gate_up_swiglu(x: torch.Tensor, w1: torch.Tensor, w2: torch.Tensor, need_ab: bool = True):
    """``a = x W1^T, b = x W2^T, y = silu(a) * b`` -> ``(a, b, y)`` (``a``/``b`` None when not
    ``need_ab``).  One launch of the gate-up GEMM when supported, else linear + linear + swiglu with
    the same rounding points."""
    K = x.shape[-1]
    Nh = w1.shape[0]
    x2 = x.reshape(-1, K)
    lead = x.shape[:-1]
    if gate_up_supported(x2, w1, w2):
        M = x2.shape[0]
        y = torch.empty((M, Nh), dtype=torch.bfloat16, device=x.device)
        a = torch.empty_like(y) if need_ab else None
        b = torch.empty_like(y) if need_ab else None
        _count("gemm4")
        rc = require().lta_gemm4_swiglu(x2.data_ptr(), w1.data_ptr(), w2.data_ptr(),
                                        None if a is None else a.data_ptr(), None if b is None else b.data_ptr(),
                                        y.data_ptr(), None, None, M, Nh, K, x2.stride(0), w1.stride(0), Nh, 1,
                                        stream_ptr(x.device))
        check(rc, "lta_gemm4_swiglu")
        r = (lambda t: None if t is None else t.reshape(*lead, Nh))
        return r(a), r(b), r(y)
    from .fused import swiglu_fwd

    a = linear(x, w1)
    b = linear(x, w2)
    return a, b, swiglu_fwd(a, b)


def matmul_swiglu_bwd(dy: torch.Tensor, w: torch.Tensor, a: torch.Tensor, b: torch.Tensor):
    """``g = dy @ w`` (the dgrad of the MLP down-projection, ``w`` = its weight viewed [K, N]) then the
    SwiGLU backward ``(da, db)`` of ``y = silu(a) * b``, with ``g`` kept on chip when supported."""
    N = w.shape[1]
    dy2 = dy.reshape(-1, dy.shape[-1])
    a2, b2 = a.reshape(-1, N), b.reshape(-1, N)
    lay = gemm4_layout(dy2, w) if _os.environ.get("LTA_GEMM", "auto") != "torch" else None
    if (lay is not None and lay[0] == 0 and lay[1] == 1 and _fused_swiglu_on() and N % 256 == 0 and dy2.shape[1] % 128 == 0
            and a2.is_contiguous() and b2.is_contiguous() and a2.data_ptr() % 16 == 0 and b2.data_ptr() % 16 == 0
            and a2.dtype == torch.bfloat16 and b2.dtype == torch.bfloat16 and a2.shape[0] == dy2.shape[0]):
        M, K = dy2.shape
        da = torch.empty((M, N), dtype=torch.bfloat16, device=dy.device)
        db = torch.empty_like(da)
        _count("gemm4")
        rc = require().lta_gemm4_swiglu(dy2.data_ptr(), w.data_ptr(), None, da.data_ptr(), db.data_ptr(), None,
                                        a2.data_ptr(), b2.data_ptr(), M, N, K, lay[2], lay[3], N, 2,
                                        stream_ptr(dy.device))
        check(rc, "lta_gemm4_swiglu")
        return da.reshape(a.shape), db.reshape(b.shape)
    from .fused import swiglu_bwd

    g = matmul(dy, w)
    return swiglu_bwd(g.reshape(a.shape), a, b)


register_signature("lta_gemm4_qkv_rope", [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p])


_HALVES_EQUAL: dict = {}


def _rope_halves_equal(cos: torch.Tensor, sin: torch.Tensor, T: int) -> bool:
    """The fused epilogue reads cos / sin once per (d, d + 64) pair: true for rotate-half caches
    built as cat(freqs, freqs) (LitGPT / HF).  Checked once per cache buffer (not per call)."""
    try:
        key = (cos.data_ptr(), sin.data_ptr(), tuple(cos.shape), tuple(sin.shape), cos._version, sin._version, T)
    except RuntimeError:  # inference tensors carry no version counter
        key = (cos.data_ptr(), sin.data_ptr(), tuple(cos.shape), tuple(sin.shape), T)
    hit = _HALVES_EQUAL.get(key)
    if hit is None:
        if torch.cuda.is_current_stream_capturing():
            return False
        c, s_ = cos[:T], sin[:T]
        hit = bool(torch.equal(c[:, :64], c[:, 64:]) and torch.equal(s_[:, :64], s_[:, 64:]))
        if len(_HALVES_EQUAL) > 64:
            _HALVES_EQUAL.clear()
        _HALVES_EQUAL[key] = hit
    return hit


def linear_qkv_rope(x: torch.Tensor, w: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, n_head: int,
                    n_query_groups: int, head_size: int, rope_n: int):
    """``q, k, v = qkv_split_rope(x @ w.T)`` for a ``[q heads | k heads | v heads]`` projection: one
    launch of the GEMM whose epilogue applies the rotate-half RoPE and stores the [B, H, T, D]
    head layouts (csrc/gemm4.hip EPI 3) when supported, else the GEMM then csrc/rope.hip."""
    B, T, K = x.shape
    x2 = x.reshape(-1, K)
    nq = n_head + 2 * n_query_groups
    ok = (_os.environ.get("LTA_GEMM", "auto") != "torch" and _os.environ.get("LTA_FUSED_QKV_ROPE", "1") != "0"
          and head_size == 128 and rope_n == 128 and nq % 2 == 0 and tuple(w.shape) == (nq * 128, K)
          and _plain_2d(x2) and _plain_2d(w) and x2.shape[0] >= GEMM4_MIN_M and K % 128 == 0
          and cos.dtype == torch.float32 and sin.dtype == torch.float32 and cos.shape[-1] == 128
          and sin.shape[-1] == 128 and cos.shape[0] >= T and sin.shape[0] >= T
          and cos.dim() == 2 and sin.dim() == 2
          and x2.shape[0] * x2.stride(0) * 2 < 2 ** 31 and w.shape[0] * w.stride(0) * 2 < 2 ** 31)
    if ok and _rope_halves_equal(cos, sin, T):
        c = cos[:T].contiguous()
        s = sin[:T].contiguous()
        q = torch.empty((B, n_head, T, 128), dtype=torch.bfloat16, device=x.device)
        k = torch.empty((B, n_query_groups, T, 128), dtype=torch.bfloat16, device=x.device)
        v = torch.empty_like(k)
        _count("gemm4")
        rc = require().lta_gemm4_qkv_rope(x2.data_ptr(), w.data_ptr(), c.data_ptr(), s.data_ptr(), q.data_ptr(),
                                          k.data_ptr(), v.data_ptr(), x2.shape[0], K, x2.stride(0), w.stride(0), T,
                                          n_head, n_query_groups, stream_ptr(x.device))
        check(rc, "lta_gemm4_qkv_rope")
        return q, k, v
    from .fused import qkv_rope_fwd

    return qkv_rope_fwd(linear(x, w), cos, sin, n_head, n_query_groups, head_size, rope_n)
