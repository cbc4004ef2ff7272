"""K3 flash attention wrappers (kernels in ``csrc/attention_fwd.hip`` / ``attention_bwd.hip``)."""
from __future__ import annotations

import ctypes
import math
import os

import torch

from ._lib import require, dcode, ptr, stream_ptr, check, register_signature, c_int, c_int64, c_void_p, c_float

register_signature("lta_attn_fwd", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                    c_int, c_int, c_float, c_int, c_void_p])
register_signature("lta_attn_bwd", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                    c_float, c_int, c_void_p])
register_signature("lta_attn_fwd_s", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                      c_int, c_int, c_int, c_float, c_int, c_void_p, c_void_p])
register_signature("lta_attn_bwd_s", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                                      c_float, c_int, c_void_p, c_void_p])

register_signature("lta_attn_fwd_ex", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                       c_int, c_int, c_int, c_float, c_int, c_void_p, c_void_p, c_int, c_int, c_float,
                                       ctypes.c_uint64, ctypes.c_uint64, c_void_p])
register_signature("lta_attn_bwd_ex", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_float,
                                       c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_float, ctypes.c_uint64,
                                       ctypes.c_uint64, c_void_p])

register_signature("lta_attn_fwd_ex2", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                        c_int, c_int, c_int, c_float, c_int, c_void_p, c_void_p, c_int, c_int, c_float,
                                        ctypes.c_uint64, ctypes.c_uint64, c_void_p, c_void_p])
register_signature("lta_attn_bwd_ex2", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_float,
                                        c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_float, ctypes.c_uint64,
                                        ctypes.c_uint64, c_void_p, c_void_p])
register_signature("lta_attn_bwd_rope", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_float,
                                         c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         ctypes.c_int64, c_int, c_void_p])
register_signature("lta_attn_bwd_rope_ds", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                            c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                            c_int, c_float, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                            c_void_p, ctypes.c_int64, c_void_p, ctypes.c_int64, c_int, c_void_p])
register_signature("lta_attn_bwd_ex3", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_float,
                                        c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_float, ctypes.c_uint64,
                                        ctypes.c_uint64, c_void_p, c_void_p, c_void_p])

SUPPORTED_HEAD_DIMS = (64, 96, 128, 256)  # the kernels' compile-time head dims
# Other head dims up to 256 (multiples of 8) run zero-padded to the next kernel head dim, as the
# reference pads for aten flash (thunder/executors/sdpaex.py:45-59): zero columns of Q / K leave
# Q K^T unchanged, zero columns of V give zero columns of O (sliced off), the scale stays the
# caller's (1 / sqrt(D) of the real D), and the padded gradient columns are exactly zero.
# D = 256 (Gemma; cuDNN's limit, thunder/executors/cudnn_sdpa.py:339-363) runs 32-key tiles at one
# workgroup per CU with the accumulators in the AGPR file; additive / boolean masks and dropout are
# compiled into those kernels as for the smaller head dims (no spills: 248-256 VGPRs + AGPRs).
MAX_PADDED_HEAD_DIM = 256
PLAIN_ONLY_HEAD_DIM = 256  # above this head dim the kernels would take no additive mask / dropout


def padded_head_dim(D: int) -> int | None:
    if D in SUPPORTED_HEAD_DIMS:
        return D
    if D % 8 or D <= 0 or D > MAX_PADDED_HEAD_DIM:
        return None
    return next(d for d in SUPPORTED_HEAD_DIMS if d >= D)


def _pad_d(t: torch.Tensor, Dp: int) -> torch.Tensor:
    return t if t.shape[-1] == Dp else torch.nn.functional.pad(t, (0, Dp - t.shape[-1]))


def prepare_mask(mask: torch.Tensor, B: int, Hq: int, Tq: int, Sk: int):
    """Additive fp32 image of an SDPA mask for the kernels: ``[Bm, Hm, Tq, Skp]`` (Bm in {1, B},
    Hm in {1, Hq}, key dim padded to a multiple of 64 with -inf).  A boolean mask (True = attend)
    becomes 0 / -inf.  Returns (image, mask_b, mask_h)."""
    m = mask
    while m.dim() < 4:
        m = m.unsqueeze(0)
    mb = m.shape[0] == B and B > 1
    mh = m.shape[1] == Hq and Hq > 1
    m = m.expand(B if mb else 1, Hq if mh else 1, Tq, Sk)
    skp = (Sk + 63) // 64 * 64
    out = torch.full((m.shape[0], m.shape[1], Tq, skp), float("-inf"), device=m.device, dtype=torch.float32)
    if m.dtype == torch.bool:
        out[..., :Sk].masked_fill_(m, 0.0)
    else:
        out[..., :Sk].copy_(m)
    return out, int(mb), int(mh)


def supported(q, k, v) -> bool:
    return (
        q.dtype in (torch.bfloat16, torch.float16)
        and k.dtype == q.dtype
        and v.dtype == q.dtype
        and q.ndim == 4
        and padded_head_dim(q.shape[-1]) is not None
        and k.shape[-1] == q.shape[-1]
        and v.shape[-1] == q.shape[-1]
        and q.shape[1] % k.shape[1] == 0
        and k.shape[1] == v.shape[1]
    )


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


def _strides3(t):
    return (ctypes.c_int64 * 3)(*t.stride()[:3])


def _qkv_in_place(q, k, v):
    """q / k / v as the kernels read them: any [B, H, T] strides with the head dim contiguous and
    16-byte aligned rows in place (e.g. views into a fused qkv projection), else a contiguous copy;
    plus their (batch, head, token) strides for the kernels."""
    q, k, v = (t if _rows_ok(t) else t.contiguous() for t in (q, k, v))
    st = (ctypes.c_int64 * 9)(*q.stride()[:3], *k.stride()[:3], *v.stride()[:3])
    return q, k, v, st


def _grad_like(t):
    """An empty [B, H, T, D] gradient for ``t``: [B, T, H, D] memory (transposed view) when ``t`` is a
    head split of a token-major tensor (token stride > head stride), dense [B, H, T, D] otherwise."""
    B, H, T, D = t.shape
    if H > 1 and T > 1 and t.stride(2) > t.stride(1):
        return torch.empty((B, T, H, D), device=t.device, dtype=t.dtype).transpose(1, 2)
    return torch.empty((B, H, T, D), device=t.device, dtype=t.dtype)


def _rows_ok(t) -> bool:
    """Head dim contiguous, 16-byte aligned rows: any [B, H, T] strides are read in place."""
    return t.stride(-1) == 1 and all(s % 8 == 0 for s in t.stride()[:-1]) and t.data_ptr() % 16 == 0


register_signature("lta_attn_set_rng_state", [c_void_p])
register_signature("lta_attn_set_fp8_out", [c_void_p, c_void_p, c_float, c_void_p, c_void_p])
register_signature("lta_attn_fp8_out_used", [])


def _graph_rng(lib, dropout_p, seed, offset):
    """Dropout seeds drawn inside a hipGraph capture (core/rng.py GraphRngInt): hand the kernel the
    region's device RNG state; the offset stays relative to its base."""
    from ..core.rng import GraphRngInt

    if dropout_p > 0 and (type(seed) is GraphRngInt or type(offset) is GraphRngInt):
        st = (seed if type(seed) is GraphRngInt else offset).state
        lib.lta_attn_set_rng_state(st.data_ptr())
        return 0, int(offset)
    return seed, offset


def attn_fwd(q, k, v, causal: bool, scale: float | None = None, out_layout: str = "bshd", mask=None,
             dropout_p: float = 0.0, seed: int = 0, offset: int = 0, fp8_out=None):
    """q [B, Hq, T, D], k/v [B, Hkv, S, D] -> (o [B, Hq, T, D], lse [B, Hq, T] fp32).

    ``out_layout="bshd"`` (default) stores O as [B, T, Hq, D] and returns its [B, Hq, T, D]
    transposed view: the usual ``o.transpose(1, 2).reshape(B, T, Hq * D)`` before the output
    projection is then a view instead of a copy, and the backward reads it (and dO) in place.

    ``fp8_out`` = (q8 uint8 [B, T, Hq, D], amax_in, fmax, scale_out, amax_out): ask the kernel for an
    e4m3 copy of O as well (the FP8 output projection's input, delayed scaling; csrc AttnQ8).  Returns
    (o, lse, written) then; ``written`` is False when the launched kernel has no such output (the caller
    casts separately)."""
    if fp8_out is not None:
        lib = require()
        if out_layout != "bshd" or q.shape[-1] != 128 or mask is not None or dropout_p:
            return attn_fwd(q, k, v, causal, scale, out_layout, mask, dropout_p, seed, offset) + (False,)
        q8, amax_in, fmax, scale_out, amax_out = fp8_out
        lib.lta_attn_set_fp8_out(q8.data_ptr(), amax_in.data_ptr(), float(fmax), scale_out.data_ptr(),
                                 amax_out.data_ptr())
        try:
            o, lse = attn_fwd(q, k, v, causal, scale, out_layout)
        finally:
            used = bool(lib.lta_attn_fp8_out_used())
            lib.lta_attn_set_fp8_out(None, None, 0.0, None, None)  # never left armed for another call
        return o, lse, used
    lib = require()
    D0 = q.shape[-1]
    Dp = padded_head_dim(D0)
    if Dp is not None and Dp != D0:
        sc = scale if scale is not None else 1.0 / math.sqrt(D0)
        o, lse = attn_fwd(_pad_d(q, Dp), _pad_d(k, Dp), _pad_d(v, Dp), causal, sc, out_layout, mask, dropout_p, seed,
                          offset)
        return o[..., :D0], lse
    q, k, v, qkv_st = _qkv_in_place(q, k, v)
    B, Hq, T, D = q.shape
    Hkv, S = k.shape[1], k.shape[2]
    sc = scale if scale is not None else 1.0 / math.sqrt(D)
    if out_layout == "bshd":
        o = torch.empty((B, T, Hq, D), device=q.device, dtype=q.dtype).transpose(1, 2)
    else:
        o = torch.empty((B, Hq, T, D), device=q.device, dtype=q.dtype)
    lse = torch.empty((B, Hq, T), device=q.device, dtype=torch.float32)
    mimg, mb, mh = (None, 0, 0) if mask is None else prepare_mask(mask, B, Hq, T, S)
    seed, offset = _graph_rng(lib, dropout_p, seed, offset)
    rc = lib.lta_attn_fwd_ex2(dcode(q), ptr(q), ptr(k), ptr(v), ptr(o), ptr(lse), B, Hq, Hkv, T, S, D, float(sc),
                              int(causal), ctypes.cast(_strides3(o), c_void_p), ptr(mimg), mb, mh, float(dropout_p),
                              int(seed) & (2 ** 64 - 1), int(offset) & (2 ** 64 - 1), ctypes.cast(qkv_st, c_void_p),
                              stream_ptr(q.device))
    check(rc, "lta_attn_fwd")
    return o, lse


def attn_bwd(do, q, k, v, o, lse, causal: bool, scale: float | None = None, mask=None, dropout_p: float = 0.0,
             seed: int = 0, offset: int = 0, mask_grad: bool = False):
    """Returns (dq, dk, dv) with dk/dv summed over the query heads of each kv group; with
    ``mask_grad`` (a float mask) a 4th result: the mask's gradient, reduced to its shape."""
    lib = require()
    D0 = q.shape[-1]
    Dp = padded_head_dim(D0)
    if Dp is not None and Dp != D0:
        sc = scale if scale is not None else 1.0 / math.sqrt(D0)
        res = attn_bwd(_pad_d(do, Dp), _pad_d(q, Dp), _pad_d(k, Dp), _pad_d(v, Dp), _pad_d(o, Dp), lse, causal, sc, mask,
                       dropout_p, seed, offset, mask_grad)
        return (res[0][..., :D0], res[1][..., :D0], res[2][..., :D0]) + tuple(res[3:])
    q, k, v, qkv_st = _qkv_in_place(q, k, v)
    do = do if _rows_ok(do) else do.contiguous()
    o = o if _rows_ok(o) else o.contiguous()
    B, Hq, T, D = q.shape
    Hkv, S = k.shape[1], k.shape[2]
    sc = scale if scale is not None else 1.0 / math.sqrt(D)
    # gradients take their operand's (head, token) order: heads split from a [B, T, H*D] projection
    # get [B, T, H, D] gradients, so the transpose + reshape back to [B, T, H*D] is a view
    dq, dk, dv = _grad_like(q), _grad_like(k), _grad_like(v)
    gst = (ctypes.c_int64 * 9)(*dq.stride()[:3], *dk.stride()[:3], *dv.stride()[:3])
    delta = torch.empty((B, Hq, T), device=q.device, dtype=torch.float32)
    st = (ctypes.c_int64 * 6)(*do.stride()[:3], *o.stride()[:3])
    mimg, mb, mh = (None, 0, 0) if mask is None else prepare_mask(mask, B, Hq, T, S)
    dmask = None
    if mask_grad:
        assert mask is not None and mask.dtype != torch.bool
        dmask = torch.empty((B, Hq, T, S), device=q.device, dtype=torch.float32)
    seed, offset = _graph_rng(lib, dropout_p, seed, offset)
    part = None
    if Hq > Hkv and mask is None and dropout_p == 0:
        # GQA / MQA: the dK/dV pass splits each kv group's query heads over workgroups (D = 128 runs the
        # v4 kernel's 256-key blocks, other head dims the v1 kernel's 128-key blocks)
        part, nbytes, hs = _gqa_workspace(B, Hq, Hkv, S, q.device, D, 256 if D == 128 else 128)
        if part is not None:
            lib.lta_attn_set_gqa_workspace(part.data_ptr(), nbytes, hs)
    rc = lib.lta_attn_bwd_ex3(dcode(q), ptr(do), ptr(q), ptr(k), ptr(v), ptr(o), ptr(lse), ptr(delta), ptr(dq), ptr(dk),
                              ptr(dv), B, Hq, Hkv, T, S, D, float(sc), int(causal), ctypes.cast(st, c_void_p), ptr(mimg),
                              mb, mh, ptr(dmask), float(dropout_p), int(seed) & (2 ** 64 - 1),
                              int(offset) & (2 ** 64 - 1), ctypes.cast(qkv_st, c_void_p), ctypes.cast(gst, c_void_p),
                              stream_ptr(q.device))
    check(rc, "lta_attn_bwd")
    if not mask_grad:
        return dq, dk, dv
    # the mask broadcasts over some dims: its gradient is dS summed over them
    g = dmask
    shape = tuple(mask.shape)
    lead = g.dim() - len(shape)
    g = g.sum(tuple(range(lead))) if lead else g
    dims = tuple(i for i, n in enumerate(shape) if n == 1 and g.shape[i] != 1)
    if dims:
        g = g.sum(dims, keepdim=True)
    return dq, dk, dv, g.to(mask.dtype)


def _dq_from_ds(ws_bytes: int, device: torch.device | None = None) -> bool:
    """The RoPE'd backward computes dQ from the dS the dK/dV kernel stores (one B Hq T^2 bf16
    workspace, 1 GiB for a Llama-2-7B layer at T = 4096) instead of the dQ kernel's S / P / dP
    recompute: 59 us less per layer there (profiles/attn_dq_from_ds.txt).  On by default while the
    workspace fits LTA_ATTN_DS_MAX_GB (default 4) and at most half of what the device can still
    hand out (driver-free plus the caching allocator's unused reserve), so a run near the memory
    limit keeps the workspace-free recompute path; LTA_ATTN_DQ_FROM_DS=0 / 1 forces it off / on."""
    mode = os.environ.get("LTA_ATTN_DQ_FROM_DS", "auto")
    if mode in ("0", "1"):
        return mode == "1"
    if ws_bytes > float(os.environ.get("LTA_ATTN_DS_MAX_GB", "4")) * 2 ** 30:
        return False
    if device is None or device.type != "cuda":
        return True
    free, _ = torch.cuda.mem_get_info(device)
    spare = torch.cuda.memory_reserved(device) - torch.cuda.memory_allocated(device)
    return 2 * ws_bytes <= free + spare


def gqa_split(B: int, Hq: int, Hkv: int, S: int, keys_per_wg: int = 256) -> int:
    """How many workgroups share one kv group's query heads in the dK/dV pass.  The pass runs one
    workgroup per (batch, kv head, 256 keys): for GQA models (Mistral / Llama-3: 8 kv heads) that is
    128 workgroups at T = 4096, half of the 256 CUs, each sweeping 4 query heads.  Splitting the heads
    over workgroups (fp32 partial dK / dV rows, summed by one reduce launch) targets >= 2 waves of
    workgroups; LTA_ATTN_GQA_SPLIT caps it (1 = off)."""
    group = Hq // Hkv
    if group <= 1:
        return 1
    cap = int(os.environ.get("LTA_ATTN_GQA_SPLIT", "8"))
    n_wg = B * Hkv * ((S + keys_per_wg - 1) // keys_per_wg)
    best = 1
    for d in range(2, group + 1):
        if group % d or d > cap:
            continue
        best = d
        if n_wg * d >= 512:
            break
    return best if n_wg < 512 else 1


def _gqa_workspace(B, Hq, Hkv, S, device, D: int = 128, keys_per_wg: int = 256):
    hs = gqa_split(B, Hq, Hkv, S, keys_per_wg)
    if hs <= 1:
        return None, 0, 1
    ws = torch.empty(hs * B * Hkv * S * 2 * D, device=device, dtype=torch.float32)
    return ws, ws.numel() * 4, hs


register_signature("lta_attn_set_gqa_workspace", [c_void_p, c_int64, c_int])


def attn_bwd_rope(do, q, k, v, o, lse, causal: bool, scale, cos, sin, n_head: int, n_query_groups: int):
    """The attention backward and the backward of the rotate-half RoPE + qkv split in one pass:
    returns d(qkv) [B, T, (n_head + 2 n_query_groups) * 128], with dQ / dK rotated back in the
    dK/dV and dQ kernels' epilogues and stored (like dV) straight into their columns of the fused
    projection's gradient (no dq / dk / dv tensors, no separate RoPE-backward pass).  Falls back to
    ``attn_bwd`` + ``ops.fused.qkv_rope_bwd`` when the kernels do not cover the case."""
    lib = require()
    B, Hq, T, D = q.shape
    Hkv, S = k.shape[1], k.shape[2]
    sc = scale if scale is not None else 1.0 / math.sqrt(D)
    if D == 128 and S == T and Hq == n_head and Hkv == n_query_groups:
        qq, kk, vv, qkv_st = _qkv_in_place(q, k, v)
        dd = do if _rows_ok(do) else do.contiguous()
        oo = o if _rows_ok(o) else o.contiguous()
        cs = cos[:T].float().contiguous()
        sn = sin[:T].float().contiguous()
        W = (Hq + 2 * Hkv) * D
        dqkv = torch.empty((B, T, W), device=q.device, dtype=q.dtype)
        gst = (ctypes.c_int64 * 9)(T * W, D, W, T * W, D, W, T * W, D, W)
        delta = torch.empty((B, Hq, T), device=q.device, dtype=torch.float32)
        st = (ctypes.c_int64 * 6)(*dd.stride()[:3], *oo.stride()[:3])
        esz = dqkv.element_size()
        rc = -1
        n_ws = B * Hq * S * ((T + 255) // 256 * 256)
        part, part_bytes, hsplit = _gqa_workspace(B, Hq, Hkv, S, q.device)
        # the kernel's own shape rules (T == S checked above, T % 64) before the workspace is allocated
        if T > 0 and T % 64 == 0 and Hq % Hkv == 0 and _dq_from_ds(n_ws * esz, q.device):
            ws = torch.empty(n_ws, device=q.device, dtype=q.dtype)
            rc = lib.lta_attn_bwd_rope_ds(dcode(qq), ptr(dd), ptr(qq), ptr(kk), ptr(vv), ptr(oo), ptr(lse), ptr(delta),
                                          ptr(dqkv), ptr(dqkv) + Hq * D * esz, ptr(dqkv) + (Hq + Hkv) * D * esz, B, Hq,
                                          Hkv, T, S, D, float(sc), int(causal), ctypes.cast(st, c_void_p),
                                          ctypes.cast(qkv_st, c_void_p), ctypes.cast(gst, c_void_p), ptr(cs), ptr(sn),
                                          ptr(ws), ws.numel() * ws.element_size(), ptr(part), part_bytes, hsplit,
                                          stream_ptr(q.device))
            if rc != -1:
                check(rc, "lta_attn_bwd_rope_ds")
                return dqkv
        rc = lib.lta_attn_bwd_rope(dcode(qq), ptr(dd), ptr(qq), ptr(kk), ptr(vv), ptr(oo), ptr(lse), ptr(delta),
                                   ptr(dqkv), ptr(dqkv) + Hq * D * esz, ptr(dqkv) + (Hq + Hkv) * D * esz, B, Hq, Hkv, T,
                                   S, D, float(sc), int(causal), ctypes.cast(st, c_void_p), ctypes.cast(qkv_st, c_void_p),
                                   ctypes.cast(gst, c_void_p), ptr(cs), ptr(sn), ptr(part), part_bytes, hsplit,
                                   stream_ptr(q.device))
        if rc != -1:
            check(rc, "lta_attn_bwd_rope")
            return dqkv
    from .fused import qkv_rope_bwd

    dq, dk, dv = attn_bwd(do, q, k, v, o, lse, causal, sc)
    return qkv_rope_bwd(dq, dk, dv, cos, sin, n_head, n_query_groups, D, D)


# ------------------------------------------------------------------------------------------------
# K3d decode attention (csrc/decode_attention.hip): T <= 16 query rows against a long KV cache
# ------------------------------------------------------------------------------------------------
import ctypes  # noqa: E402

from ._lib import c_int64  # noqa: E402

register_signature("lta_decode_attn", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_float,
                                       c_int, c_void_p])

DECODE_MAX_QUERIES = 16


def _aligned_rows(t: torch.Tensor) -> torch.Tensor:
    """Head dim contiguous and every row start 16-byte aligned (the kernel uses 16-byte loads)."""
    ok = t.stride(-1) == 1 and all(s % 8 == 0 for s in t.stride()[:-1]) and t.data_ptr() % 16 == 0
    return t if ok else t.contiguous()


def decode_attn(q, k, v, mask=None, causal: bool = False, scale: float | None = None):
    """q [B, Hq, T, D] (T <= 16), k/v [B, Hkv, S, D], mask bool broadcastable to [B, Hq, T, S] -> [B, Hq, T, D]."""
    lib = require()
    q, k, v = _aligned_rows(q), _aligned_rows(k), _aligned_rows(v)
    B, Hq, T, D = q.shape
    Hkv, S = k.shape[1], k.shape[2]
    sc = scale if scale is not None else 1.0 / math.sqrt(D)
    if mask is not None:
        mask = torch.broadcast_to(mask, (B, Hq, T, S))
        ms = mask.stride()
    else:
        ms = (0, 0, 0, 0)
    rows = B * Hq * T
    # few rows (batch-1 decode): one row per workgroup with its 4 waves splitting the keys
    wsplit = rows < 256
    blocks = rows if wsplit else (rows + 3) // 4
    # split the cache so that a decode step still launches >= ~256 workgroups (flash-decoding)
    nsplit = max(1, min((256 + blocks - 1) // blocks, S // 256))  # a split is worth a combine launch from ~256 keys
    chunk = ((S + nsplit - 1) // nsplit + 63) // 64 * 64
    nsplit = (S + chunk - 1) // chunk
    o = torch.empty((B, Hq, T, D), device=q.device, dtype=q.dtype)
    ws_acc = ws_ml = None
    if nsplit > 1:
        ws_acc = torch.empty((nsplit, rows, D), device=q.device, dtype=torch.float32)
        ws_ml = torch.empty((nsplit, rows, 2), device=q.device, dtype=torch.float32)
    st = (ctypes.c_int64 * 13)(q.stride(0), q.stride(1), q.stride(2), k.stride(0), k.stride(1), k.stride(2),
                               v.stride(0), v.stride(1), v.stride(2), *ms)
    mptr = None if mask is None else mask.data_ptr()
    rc = lib.lta_decode_attn(dcode(q), ptr(q), ptr(k), ptr(v), mptr, ptr(o), ptr(ws_acc), ptr(ws_ml), B, Hq, Hkv, T, S, D,
                             ctypes.cast(st, ctypes.c_void_p), chunk, nsplit, int(causal), float(sc), int(wsplit),
                             stream_ptr(q.device))
    check(rc, "lta_decode_attn")
    return o
