"""4-bit MXFP4 weight-quantized inference linears (CDNA4-native; the reference's 4-bit inference
path is bitsandbytes NF4, ``thunder/transforms/quantization.py:19-293``, which this framework also
has in ``transforms/quantization.py``).

``transform_module`` quantizes each ``nn.Linear`` weight once to OCP MXFP4 (e2m1 elements, one
E8M0 scale per 32 input features; ``ops/mxfp4.py``).  At run time:

* decode and short prompts (up to 32 rows): the weight-only GEMV (``csrc/mxfp4.hip``) streams
  the 4-bit weight (once per 8 rows) and multiplies bf16 activations — a quarter of the bf16
  weight bytes per token;
* prefill, ``activations="bf16"`` (default, W4A16): the weight is dequantized to bf16 and the
  product runs on the bf16 GEMM path;
* prefill, ``activations="mxfp4"`` (W4A4): the activation is MXFP4-quantized as well and the
  product runs on the block-scaled MFMA at the fp4 rate (``gemm_nt_mxfp4_kernel``), rows padded
  to the 256-row tile.

The op is a ``torch.library`` custom op (``lta::mxfp4_linear``), traced like any other op and
runnable eagerly; activation gradients flow through the dequantized weight (frozen base weights,
as for LoRA on a quantized model).
"""
from __future__ import annotations

import torch

from ..core.transform_common import Transform
from ..ops import mxfp4 as _mx


GEMV_ROWS = 32  # rows up to which the GEMV path is used


def _gpu(x: torch.Tensor) -> bool:
    return x.is_cuda and x.dtype == torch.bfloat16


@torch.library.custom_op("lta::mxfp4_linear", mutates_args=())
def mxfp4_linear(x: torch.Tensor, qweight: torch.Tensor, scales: torch.Tensor, bias: torch.Tensor | None = None,
                 fp4_activations: bool = False) -> torch.Tensor:
    N, K = qweight.shape[0], qweight.shape[1] * 2
    x2 = x.reshape(-1, K)
    M = x2.shape[0]
    if _gpu(x2) and M <= GEMV_ROWS:
        # decode and short prompts: the weight-only GEMV, 8 rows per pass over the 4-bit weight
        # (cheaper than dequantizing the weight to bf16 up to a few passes)
        y = torch.cat([_mx.gemv(x2[i:i + _mx.GEMV_MAX_ROWS], qweight, scales, bias)
                       for i in range(0, M, _mx.GEMV_MAX_ROWS)]) if M > _mx.GEMV_MAX_ROWS else \
            _mx.gemv(x2, qweight, scales, bias)
    elif _gpu(x2) and fp4_activations and N % 256 == 0 and K % 256 == 0:
        Mp = (M + 255) // 256 * 256
        xp = x2 if Mp == M else torch.cat([x2, x2.new_zeros(Mp - M, K)])
        qx, sx = _mx.quantize(xp)
        y = _mx.gemm_nt(qx, sx, qweight, scales, bias)[:M]
    else:
        w = _mx.dequantize(qweight, scales, x.dtype)
        y = torch.nn.functional.linear(x2, w, None if bias is None else bias.to(x.dtype))
    return y.reshape(*x.shape[:-1], N).to(x.dtype)


@mxfp4_linear.register_fake
def _mxfp4_linear_fake(x, qweight, scales, bias=None, fp4_activations=False):
    return x.new_empty((*x.shape[:-1], qweight.shape[0]))


def _setup(ctx, inputs, output):
    x, qweight, scales, bias, _ = inputs
    ctx.save_for_backward(qweight, scales)
    ctx.has_bias = bias is not None


def _backward(ctx, g):
    qweight, scales = ctx.saved_tensors
    gx = g @ _mx.dequantize(qweight, scales, g.dtype)
    gb = g.reshape(-1, g.shape[-1]).sum(0) if ctx.has_bias else None
    return gx, None, None, gb, None


mxfp4_linear.register_autograd(_backward, setup_context=_setup)


class _MXFP4Forward:
    def __init__(self, mod, fp4_activations: bool):
        self.mod = mod
        self.fp4_activations = fp4_activations

    def __call__(self, x):
        m = self.mod
        return mxfp4_linear(x, m.mxfp4_weight, m.mxfp4_scales, m.bias, self.fp4_activations)


class MXFP4InferenceTransform(Transform):
    """Quantizes ``nn.Linear`` weights (all, or those named in ``modules``; in-features a multiple
    of 32) to MXFP4 for inference.  ``activations``: ``"bf16"`` (weight-only) or ``"mxfp4"``."""

    def __init__(self, modules: list[str] | None = None, skip: tuple[str, ...] = ("lm_head",),
                 activations: str = "bf16"):
        if activations not in ("bf16", "mxfp4"):
            raise ValueError(f"activations must be 'bf16' or 'mxfp4', got {activations!r}")
        self.modules = modules
        self.skip = skip
        self.fp4_activations = activations == "mxfp4"
        self.quantized: list[str] = []

    def transform_module(self, model) -> None:
        for name, m in model._model.named_modules():
            if not isinstance(m, torch.nn.Linear) or hasattr(m, "mxfp4_weight"):
                continue
            if self.modules is not None and name not in self.modules:
                continue
            if any(name.endswith(s) for s in self.skip) or m.in_features % _mx.BLOCK:
                continue
            q, s = _mx.quantize(m.weight.detach())
            del m.weight
            m.register_buffer("mxfp4_weight", q)
            m.register_buffer("mxfp4_scales", s)
            m.forward = _MXFP4Forward(m, self.fp4_activations)
            self.quantized.append(name)

    def transform_state_dict_for_submodule(self, model, submodule_name, state_dict):
        if submodule_name not in self.quantized or "weight" not in state_dict:
            return state_dict
        sd = dict(state_dict)
        sd["mxfp4_weight"], sd["mxfp4_scales"] = _mx.quantize(sd.pop("weight"))
        return sd
