"""8-bit (FP8 e4m3) weight-quantized inference linears (parity: reference
``thunder/transforms/te_inference.py:17-113`` — ``TEInference8BitTransform``, ops ``te_linear_fp8`` /
``te_groupedmm_fp8``).

Weights are quantized once, in ``transform_module``, to OCP e4m3 with a per-tensor scale
(``q = fp8(w * 448 / amax(w))``).  At run time each call quantizes the activation with current
per-tensor scaling (one amax pass + one cast pass, ``ops/fp8.py``) and multiplies on the CDNA4
block-scaled MFMA fp8 GEMM (``csrc/gemm.hip`` ``gemm_nt_fp8_kernel``, the dequantisation
``1/(sx*sw)`` folded into the epilogue).  Rows are padded to the GEMM's 256-row tile so decode
(M = batch) runs on the same kernel; the weight is read from HBM in fp8, i.e. half the bytes of a
bf16 GEMV.  Grouped (MoE) experts (``GroupedLinear``, weight [G, N, K]) are quantized per expert
(one scale per expert) and run on the grouped fp8 MFMA kernel ``lta_gemm_grouped_nt_fp8``
(``lta::fp8_grouped_mm_inference``, the ``te_groupedmm_fp8`` counterpart): each workgroup finds
its (expert, row tile) from the device offsets, so routing needs no host synchronisation.

The quantized linear is a ``torch.library`` custom op (``lta::fp8_linear_inference``), so it is
traced as an ordinary op and also runs eagerly.  Activation gradients flow (the weights are
frozen), which is what LoRA-style fine-tuning on a quantized base needs.
"""
from __future__ import annotations

import torch

from ..core.transform_common import Transform

E4M3_MAX = 448.0


def quantize_weight_e4m3(w: torch.Tensor):
    """w [N, K] -> (uint8 storage of e4m3 values, fp32 scale tensor [])."""
    wf = w.detach().float()
    amax = wf.abs().amax().clamp_min(1e-12)
    scale = (E4M3_MAX / amax).to(torch.float32)
    q = (wf * scale).clamp(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn).view(torch.uint8)
    return q.contiguous(), scale.reshape(())


def dequantize_e4m3(q: torch.Tensor, scale: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    return (q.view(torch.float8_e4m3fn).float() / scale).to(dtype)


def _gpu_path(x2: torch.Tensor, K: int, N: int) -> bool:
    return x2.is_cuda and x2.dtype == torch.bfloat16 and K % 256 == 0 and N % 256 == 0


@torch.library.custom_op("lta::fp8_linear_inference", mutates_args=())
def fp8_linear_inference(x: torch.Tensor, qweight: torch.Tensor, w_scale: torch.Tensor,
                         bias: torch.Tensor | None = None) -> torch.Tensor:
    N, K = qweight.shape
    x2 = x.reshape(-1, K)
    if _gpu_path(x2, K, N):
        from ..ops import fp8 as f8

        M = x2.shape[0]
        Mp = (M + 255) // 256 * 256
        xp = x2 if Mp == M else torch.cat([x2, x2.new_zeros(Mp - M, K)])
        st = torch.zeros(2, dtype=torch.float32, device=x.device)
        f8.amax_into(xp if xp.is_contiguous() else xp.contiguous(), st[0])
        qx = f8.cast(xp.contiguous(), st[0], E4M3_MAX, st[1])
        y = f8.gemm_nt_fp8(qx, qweight, st[1:2], w_scale.reshape(1), 0, 0,
                           None if bias is None else bias.to(torch.bfloat16))
        y = y[:M]
    else:
        y = torch.nn.functional.linear(x2, dequantize_e4m3(qweight, w_scale, x.dtype),
                                       None if bias is None else bias.to(x.dtype))
    return y.reshape(*x.shape[:-1], N).to(x.dtype)


@fp8_linear_inference.register_fake
def _fp8_linear_inference_fake(x, qweight, w_scale, bias=None):
    return x.new_empty((*x.shape[:-1], qweight.shape[0]))


def _setup(ctx, inputs, output):
    x, qweight, w_scale, bias = inputs
    ctx.save_for_backward(qweight, w_scale)
    ctx.xdtype = x.dtype
    ctx.has_bias = bias is not None


def _backward(ctx, g):
    qweight, w_scale = ctx.saved_tensors
    gx = g @ dequantize_e4m3(qweight, w_scale, g.dtype)
    gb = g.reshape(-1, g.shape[-1]).sum(0) if ctx.has_bias else None
    return gx, None, None, gb


fp8_linear_inference.register_autograd(_backward, setup_context=_setup)


def quantize_experts_e4m3(w: torch.Tensor):
    """w [G, N, K] -> (uint8 e4m3 [G, N, K], fp32 scales [G]) with one scale per expert."""
    wf = w.detach().float()
    amax = wf.abs().amax(dim=(1, 2)).clamp_min(1e-12)
    scale = (E4M3_MAX / amax).to(torch.float32)
    q = (wf * scale[:, None, None]).clamp(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn).view(torch.uint8)
    return q.contiguous(), scale.contiguous()


@torch.library.custom_op("lta::fp8_grouped_mm_inference", mutates_args=())
def fp8_grouped_mm_inference(x: torch.Tensor, qweight: torch.Tensor, w_scale: torch.Tensor,
                             offsets: torch.Tensor) -> torch.Tensor:
    """``x [M, K]`` (rows grouped by expert, int32 row ends ``offsets``) times the fp8 experts
    ``qweight [G, N, K]`` -> bf16 [M, N]."""
    G, N, K = qweight.shape
    if x.is_cuda and x.dtype == torch.bfloat16 and K % 128 == 0 and N % 256 == 0 and x.shape[0] > 0:
        from ..ops import fp8 as f8

        xc = x.contiguous()
        st = torch.zeros(2, dtype=torch.float32, device=x.device)
        f8.amax_into(xc, st[0])
        qx = f8.cast(xc, st[0], E4M3_MAX, st[1])
        return f8.grouped_mm_fp8(qx, qweight, st[1], w_scale, offsets.to(torch.int32))
    w = (qweight.view(torch.float8_e4m3fn).float() / w_scale[:, None, None]).to(x.dtype)
    outs, start = [], 0
    for g, end in enumerate(offsets.tolist()):
        outs.append(x[start:end] @ w[g].t())
        start = end
    return torch.cat(outs) if outs else x.new_empty((0, N))


@fp8_grouped_mm_inference.register_fake
def _fp8_grouped_fake(x, qweight, w_scale, offsets):
    return x.new_empty((x.shape[0], qweight.shape[1]))


def _g_setup(ctx, inputs, output):
    x, qweight, w_scale, offsets = inputs
    ctx.save_for_backward(qweight, w_scale, offsets)


def _g_backward(ctx, g):
    qweight, w_scale, offsets = ctx.saved_tensors
    w = (qweight.view(torch.float8_e4m3fn).float() / w_scale[:, None, None]).to(g.dtype)  # [G, N, K]
    gx, start = [], 0
    for e, end in enumerate(offsets.tolist()):
        gx.append(g[start:end] @ w[e])
        start = end
    return (torch.cat(gx) if gx else g.new_empty((0, w.shape[2]))), None, None, None


fp8_grouped_mm_inference.register_autograd(_g_backward, setup_context=_g_setup)


class _FP8GroupedForward:
    def __init__(self, mod):
        self.mod = mod

    def __call__(self, x, offsets):
        m = self.mod
        return fp8_grouped_mm_inference(x, m.fp8_weight, m.fp8_scale, offsets)


class _FP8Forward:
    def __init__(self, mod):
        self.mod = mod

    def __call__(self, x):
        m = self.mod
        return fp8_linear_inference(x, m.fp8_weight, m.fp8_scale, m.bias)


class FP8InferenceTransform(Transform):
    """Quantizes ``nn.Linear`` weights (all, or those named in ``modules``) to e4m3 for inference."""

    def __init__(self, modules: list[str] | None = None, skip: tuple[str, ...] = ("lm_head",)):
        self.modules = modules
        self.skip = skip
        self.quantized: list[str] = []

    def transform_module(self, model) -> None:
        from ..models.llama4_moe import GroupedLinear

        for name, m in model._model.named_modules():
            if isinstance(m, GroupedLinear) and not hasattr(m, "fp8_weight"):
                if (self.modules is not None and name not in self.modules) or any(name.endswith(s) for s in self.skip):
                    continue
                q, s = quantize_experts_e4m3(m.weight)
                dev = m.weight.device
                del m.weight
                m.register_buffer("fp8_weight", q.to(dev))
                m.register_buffer("fp8_scale", s.to(dev))
                m.forward = _FP8GroupedForward(m)
                self.quantized.append(name)
                continue
            if not isinstance(m, torch.nn.Linear) or hasattr(m, "fp8_weight"):
                continue
            if self.modules is not None and name not in self.modules:
                continue
            if any(name.endswith(s) for s in self.skip):
                continue
            q, s = quantize_weight_e4m3(m.weight)
            dev = m.weight.device
            del m.weight
            m.register_buffer("fp8_weight", q.to(dev))
            m.register_buffer("fp8_scale", s.to(dev))
            m.forward = _FP8Forward(m)
            self.quantized.append(name)

    def transform_state_dict_for_submodule(self, model, submodule_name, state_dict):
        if submodule_name not in self.quantized or "weight" not in state_dict:
            return state_dict
        sd = dict(state_dict)
        w = sd.pop("weight")
        sd["fp8_weight"], sd["fp8_scale"] = quantize_experts_e4m3(w) if w.ndim == 3 else quantize_weight_e4m3(w)
        return sd


TEInference8BitTransform = FP8InferenceTransform  # API-compatible name
