"""FP8 linear training (K8; reference: TransformerEngine executor + ``thunder/plugins/fp8.py``).

``FP8LinearTransform`` rewrites every eligible ``linear`` of the program (bf16 on the GPU, all
three GEMM dims multiples of 256) into ``fp8_linear`` *before* autodiff.  Its VJP is

    fwd:  qx, qx^T = cast_transpose(x, s_x)   (e4m3)      qw, qw^T = cast_transpose(w, s_w)
          y = gemm_nt_fp8(qx, qw) / (s_x s_w) + b
    bwd:  qdy, qdy^T = cast_transpose(dy, s_dy)  (e5m2)
          dx = gemm_nt_fp8(qdy, qw^T),  dw = gemm_nt_fp8(qdy^T, qx^T),  db = sum(dy)

so all three GEMMs run on the one hand-written block-scaled-MFMA NT kernel at 2x the bf16
MFMA rate, and the backward saves fp8 copies (half the bytes of bf16 activations).
Scaling is per-tensor "current" scaling (amax of the tensor being cast, computed on device,
no host synchronisation); e4m3 for activations/weights, e5m2 for gradients.
"""
from __future__ import annotations

import torch

from ..core.proxies import TensorProxy
from ..core.symbol import Symbol
from ..core.trace import from_trace, tracectx, TraceProvenance
from ..core.transform_common import Transform


def _fp8_linear_meta(x, w, bias=None):
    return TensorProxy(like=x, shape=tuple(x.shape[:-1]) + (w.shape[0],))


fp8_linear = Symbol("fp8_linear", _fp8_linear_meta, id="lta.fp8_linear", is_prim=True)


def eligible(x, w, bias=None) -> bool:
    if not all(isinstance(t, TensorProxy) for t in (x, w)):
        return False
    if x.device.type != "cuda" or x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or w.ndim != 2 or x.ndim < 2:
        return False
    if bias is not None and (not isinstance(bias, TensorProxy) or bias.dtype != torch.bfloat16):
        return False
    M = 1
    for s in x.shape[:-1]:
        M *= s
    N, K = w.shape
    return M % 256 == 0 and N % 256 == 0 and K % 256 == 0


class FP8LinearTransform(Transform):
    def __init__(self, recipe: str = "current", amax_history_len: int = 16, skip: tuple[str, ...] = ()):
        self.recipe = recipe
        self.amax_history_len = amax_history_len
        self.skip = skip
        self.n_converted = 0

    def transform_traces_pre_prologue(self, prologue_trace, computation_trace, epilogue_trace, **kwargs):
        from ..executors import hipex  # noqa: F401  (registers fp8_linear's implementation + VJP)

        new = from_trace(computation_trace)
        new.bound_symbols = []
        new.scopes = [new.bound_symbols]
        swap: dict = {}
        n = 0
        with tracectx(new):
            for b in computation_trace.bound_symbols:
                nb = b.swap_proxies(swap, skip_output=True)
                if b.sym.name == "linear" and len(nb.args) >= 2:
                    x, w = nb.args[0], nb.args[1]
                    bias = nb.args[2] if len(nb.args) > 2 else nb.kwargs.get("bias")
                    if eligible(x, w, bias) and not any(s in w.name for s in self.skip):
                        y = fp8_linear(x, w, bias)
                        swap[b.output.name] = y
                        n += 1
                        continue
                new.bound_symbols.append(nb)
        self.n_converted = n
        if not n:
            return prologue_trace, computation_trace, epilogue_trace
        new.set_provenance(TraceProvenance(f"FP8 linear ({n} linears -> e4m3/e5m2 GEMMs)"))
        return prologue_trace, new, epilogue_trace
