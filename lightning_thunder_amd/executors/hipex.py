"""hipex: the hand-written CDNA4 kernel executor (replaces the reference's cuDNN / sdpa / apex / TE /
Triton-CE executors: ``thunder/executors/{cudnnex,sdpaex,apexex,triton_crossentropy,transformer_engineex}.py``).

It claims high-level ltorch ops whole (RMSNorm, SDPA, cross-entropy, RoPE/qkv-split,
SwiGLU, ...) on HIP devices and provides *grad transforms* so autodiff saves exactly
what the fused backward kernels need (e.g. RMSNorm's per-row rstd, attention's LSE).
"""
from __future__ import annotations

import math

import torch

from ..core.proxies import TensorProxy
from ..extend import OperatorExecutor, register_executor, add_default_executor

ex = OperatorExecutor("hipex", version="0.1")
register_executor(ex)
add_default_executor(ex)

hipex = ex


def _gpu(*ts) -> bool:
    return all(t is None or (isinstance(t, TensorProxy) and t.device.type == "cuda") for t in ts)


_FLOAT16ISH = (torch.bfloat16, torch.float16, torch.float32)


# =========================================================================================
# K4 RMSNorm
# =========================================================================================
def _rms_fwd_meta(x, weight, eps):
    rows = 1
    for s in x.shape[:-1]:
        rows *= s
    return TensorProxy(like=x), TensorProxy(like=x, shape=(rows,), dtype=torch.float32, requires_grad=False)


def _rms_fwd_impl(x, weight, eps):
    from ..ops.rmsnorm import rms_norm_fwd

    return rms_norm_fwd(x, weight, eps)


def _rms_bwd_meta(dy, x, weight, rstd):
    return TensorProxy(like=x), (None if weight is None else TensorProxy(like=weight))


def _rms_bwd_impl(dy, x, weight, rstd):
    from ..ops.rmsnorm import rms_norm_bwd

    return rms_norm_bwd(dy, x, weight, rstd)


hip_rms_norm_fwd = ex.register_operator("hip_rms_norm_fwd", meta=_rms_fwd_meta, fn=_rms_fwd_impl)
hip_rms_norm_bwd = ex.register_operator("hip_rms_norm_bwd", meta=_rms_bwd_meta, fn=_rms_bwd_impl)


def _rms_checker(a, normalized_shape, weight=None, eps=None):
    if not _gpu(a, weight) or a.dtype not in _FLOAT16ISH:
        return False
    if len(normalized_shape) != 1 or normalized_shape[0] != a.shape[-1]:
        return False
    if weight is not None and (weight.dtype != a.dtype or tuple(weight.shape) != (a.shape[-1],)):
        return False
    return True


def _eps(a, eps):
    return torch.finfo(a.dtype).eps if eps is None else eps


def _rms_exec(a, normalized_shape, weight=None, eps=None):
    y, _ = hip_rms_norm_fwd(a, weight, _eps(a, eps))
    return y


def _rms_grad(a, normalized_shape, weight=None, eps=None):
    y, rstd = hip_rms_norm_fwd(a, weight, _eps(a, eps))

    def bwd(g):
        dx, dw = hip_rms_norm_bwd(g, a, weight, rstd)
        return dx, None, dw

    return y, bwd


def _register_all():
    from .. import torch as ltorch

    ex.register_implementation(ltorch.rms_norm, checker=_rms_checker, execution_transform=_rms_exec, grad_transform=_rms_grad)


_register_all()
