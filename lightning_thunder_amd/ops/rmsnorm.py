"""K4 RMSNorm wrappers (kernels in ``csrc/rmsnorm.hip``)."""
from __future__ import annotations

import torch

from ._lib import require, dcode, ptr, stream_ptr, check, register_signature, c_int, c_int64, c_void_p

register_signature("lta_rmsnorm_bwd_res", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_int64, c_int64, c_int, c_void_p, c_void_p])


def _as_2d(x: torch.Tensor):
    cols = x.shape[-1]
    x2 = x.reshape(-1, cols)
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    return x2, x2.shape[0], cols


def rms_norm_fwd(x: torch.Tensor, weight: torch.Tensor | None, eps: float):
    lib = require()
    x2, rows, cols = _as_2d(x)
    w = None if weight is None else weight.contiguous()
    y = torch.empty_like(x2)
    rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
    rc = lib.lta_rmsnorm_fwd(dcode(x2), ptr(x2), ptr(w), ptr(y), ptr(rstd), rows, cols, float(eps), stream_ptr(x.device))
    check(rc, "lta_rmsnorm_fwd")
    return y.view(x.shape), rstd


def _bwd_blocks(rows: int) -> int:
    # workgroups per launch: LTA_RMS_BWD_BLOCKS (A/B knob), default ~2 per CU on MI355X (256 CUs),
    # at least one row each
    import os

    return max(1, min(rows, int(os.environ.get("LTA_RMS_BWD_BLOCKS", "512"))))


def rms_norm_bwd(dy: torch.Tensor, x: torch.Tensor, weight: torch.Tensor | None, rstd: torch.Tensor,
                 residual: torch.Tensor | None = None):
    """(dx, dw); ``residual`` (same shape as x) is added to dx in the same pass."""
    lib = require()
    x2, rows, cols = _as_2d(x)
    dy2, _, _ = _as_2d(dy)
    r2 = None if residual is None else _as_2d(residual)[0]
    w = None if weight is None else weight.contiguous()
    dx = torch.empty_like(x2)
    nblocks = _bwd_blocks(rows)
    dw = None if weight is None else torch.empty_like(w)
    ws = torch.empty((nblocks, cols), device=x.device, dtype=torch.float32) if weight is not None else None
    rc = lib.lta_rmsnorm_bwd_res(dcode(x2), ptr(dy2), ptr(x2), ptr(w), ptr(rstd), ptr(dx), ptr(dw), ptr(ws), rows, cols,
                                 nblocks, ptr(r2), stream_ptr(x.device))
    check(rc, "lta_rmsnorm_bwd")
    return dx.view(x.shape), dw


# ---------------------------------------------------------------------------------------------
# K5 LayerNorm (csrc/layernorm.hip)
# ---------------------------------------------------------------------------------------------
from ._lib import register_signature, c_int, c_int64, c_float, c_void_p  # noqa: E402

register_signature("lta_layernorm_fwd", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                         c_int64, c_float, c_void_p])
register_signature("lta_layernorm_bwd", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_int64, c_int64, c_int, c_void_p])
register_signature("lta_layernorm_bwd_res", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                             c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int, c_void_p, c_void_p])


def layer_norm_fwd(x: torch.Tensor, weight, bias, eps: float):
    lib = require()
    x2, rows, cols = _as_2d(x)
    w = None if weight is None else weight.contiguous()
    b = None if bias is None else bias.contiguous()
    y = torch.empty_like(x2)
    mean = torch.empty(rows, device=x.device, dtype=torch.float32)
    rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
    check(lib.lta_layernorm_fwd(dcode(x2), ptr(x2), ptr(w), ptr(b), ptr(y), ptr(mean), ptr(rstd), rows, cols,
                                float(eps), stream_ptr(x.device)), "lta_layernorm_fwd")
    return y.view(x.shape), mean, rstd


def layer_norm_bwd(dy: torch.Tensor, x: torch.Tensor, weight, mean, rstd, has_bias: bool,
                   residual: torch.Tensor | None = None):
    """(dx, dw, db); ``residual`` (same shape as x) is added to dx in the same pass."""
    lib = require()
    x2, rows, cols = _as_2d(x)
    dy2, _, _ = _as_2d(dy)
    r2 = None if residual is None else _as_2d(residual)[0]
    w = None if weight is None else weight.contiguous()
    dx = torch.empty_like(x2)
    nblocks = _bwd_blocks(rows)
    dw = None if weight is None else torch.empty_like(w)
    db = torch.empty(cols, device=x.device, dtype=x.dtype) if has_bias else None
    ws = torch.empty((nblocks, 2, cols), device=x.device, dtype=torch.float32) if (dw is not None or has_bias) else None
    check(lib.lta_layernorm_bwd_res(dcode(x2), ptr(dy2), ptr(x2), ptr(w), ptr(mean), ptr(rstd), ptr(dx), ptr(dw),
                                    ptr(db), ptr(ws), rows, cols, nblocks, ptr(r2), stream_ptr(x.device)),
          "lta_layernorm_bwd")
    return dx.view(x.shape), dw, db
