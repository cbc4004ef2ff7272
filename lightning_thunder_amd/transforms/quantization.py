"""NF4 4-bit weight quantization of ``nn.Linear`` (K9).

Reference parity: ``thunder/transforms/quantization.py:19-293`` (``BitsAndBytesLinearQuant4bit``:
Linear weights -> NF4 qweight + absmax + code; ``linear`` -> ``bnb_matmul_nf4``).

MI355X design: the quantized linear is a ``torch.library`` custom op
(``lta::nf4_linear``) so it is traced like any other op (``thunder.torch.custom_op`` support)
and also runs eagerly.  On the GPU:

* decode (<= 8 activation rows): ONE fused kernel, ``lta_gemv_nf4`` (ops/csrc/nf4.hip), streams the
  4-bit weight once and decodes it in registers against the activations -- the weight is never
  materialised in bf16 and the HBM traffic is a quarter of a bf16 GEMV's;
* prefill / QLoRA training (more rows): the HIP dequant kernel writes a transient bf16 weight and
  the hand-written MFMA GEMM (``ops.gemm.linear``) consumes it.

Gradients flow to the activations (QLoRA: frozen base weights + LoRA adapters).
"""
from __future__ import annotations

import torch

from ..core.transform_common import Transform

# bitsandbytes' NF4 code book (quantiles of N(0,1) normalised to [-1, 1])
NF4_CODE = torch.tensor([
    -1.0, -0.6961928009986877, -0.5250730514526367, -0.39491748809814453, -0.28444138169288635,
    -0.18477343022823334, -0.09105003625154495, 0.0, 0.07958029955625534, 0.16093020141124725,
    0.24611230194568634, 0.33791524171829224, 0.44070982933044434, 0.5626170039176941, 0.7229568362236023, 1.0,
], dtype=torch.float32)


def quantize_nf4(w: torch.Tensor, blocksize: int = 64):
    """w (any float dtype, numel % blocksize == 0) -> (packed uint8 [n/2], absmax fp32 [n/blocksize])."""
    flat = w.detach().float().reshape(-1)
    n = flat.numel()
    if n % blocksize or n % 2:
        raise ValueError(f"NF4 needs numel divisible by the blocksize ({blocksize}), got {n}")
    blocks = flat.view(-1, blocksize)
    absmax = blocks.abs().amax(1).clamp_min(1e-12)
    normed = (blocks / absmax[:, None]).reshape(-1)
    code = NF4_CODE.to(flat.device)
    idx = (normed[:, None] - code[None, :]).abs().argmin(1).to(torch.uint8)
    packed = (idx[0::2] << 4) | idx[1::2]
    return packed.contiguous(), absmax.contiguous()


def dequantize_nf4(packed: torch.Tensor, absmax: torch.Tensor, shape, dtype=torch.bfloat16, blocksize: int = 64,
                   code: torch.Tensor | None = None) -> torch.Tensor:
    code = (NF4_CODE if code is None else code).to(packed.device)
    n = packed.numel() * 2
    if packed.is_cuda and dtype in (torch.bfloat16, torch.float16):
        from ..ops._lib import require, stream_ptr, check, register_signature, c_int, c_void_p, c_int64, DTYPE_CODE

        lib = require()
        register_signature("lta_nf4_dequant", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p])
        out = torch.empty(n, dtype=dtype, device=packed.device)
        check(lib.lta_nf4_dequant(DTYPE_CODE[dtype], packed.data_ptr(), absmax.data_ptr(), code.data_ptr(),
                                  out.data_ptr(), n, blocksize, stream_ptr(packed.device)), "lta_nf4_dequant")
        return out.view(shape)
    idx = torch.stack([(packed >> 4) & 15, packed & 15], 1).reshape(-1).long()
    vals = code[idx].view(-1, blocksize) * absmax[:, None]
    return vals.reshape(shape).to(dtype)


def gemv_nf4_supported(x: torch.Tensor, in_features: int, blocksize: int) -> bool:
    if not x.is_cuda or x.dtype not in (torch.bfloat16, torch.float16) or x.shape[-1] != in_features:
        return False
    rows = x.numel() // max(in_features, 1)
    return 1 <= rows <= 8 and in_features % 32 == 0 and blocksize % 32 == 0


def gemv_nf4(x: torch.Tensor, qweight: torch.Tensor, absmax: torch.Tensor, code: torch.Tensor, out_features: int,
             blocksize: int, bias: torch.Tensor | None = None) -> torch.Tensor:
    """Fused NF4 decode GEMV: ``x [.., K] . dequant(qweight)^T (+ bias)`` without a bf16 weight."""
    from ..ops._lib import require, stream_ptr, check, register_signature, c_int, c_void_p, DTYPE_CODE

    register_signature("lta_gemv_nf4", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                        c_int, c_int, c_int, c_int, c_int, c_void_p])
    K = x.shape[-1]
    x2 = x.reshape(-1, K)
    if x2.stride(1) != 1 or x2.stride(0) % 8 or x2.data_ptr() % 16:
        x2 = x2.contiguous()
    M = x2.shape[0]
    y = torch.empty((M, out_features), dtype=x.dtype, device=x.device)
    code = code.to(device=x.device, dtype=torch.float32).contiguous()
    b = None if bias is None else bias.to(x.dtype).contiguous()
    check(require().lta_gemv_nf4(DTYPE_CODE[x.dtype], x2.data_ptr(), qweight.data_ptr(), absmax.data_ptr(),
                                 code.data_ptr(), None if b is None else b.data_ptr(), y.data_ptr(), M, out_features,
                                 K, x2.stride(0), out_features, blocksize, stream_ptr(x.device)), "lta_gemv_nf4")
    return y.reshape(*x.shape[:-1], out_features)


@torch.library.custom_op("lta::nf4_linear", mutates_args=())
def nf4_linear(x: torch.Tensor, qweight: torch.Tensor, absmax: torch.Tensor, code: torch.Tensor, out_features: int,
               in_features: int, blocksize: int, bias: torch.Tensor | None = None) -> torch.Tensor:
    if gemv_nf4_supported(x, in_features, blocksize):
        return gemv_nf4(x, qweight, absmax, code, out_features, blocksize, bias)
    w = dequantize_nf4(qweight, absmax, (out_features, in_features), x.dtype, blocksize, code)
    if x.is_cuda and x.dtype == torch.bfloat16:
        from ..ops.gemm import linear

        return linear(x, w, bias)
    return torch.nn.functional.linear(x, w, bias)


@nf4_linear.register_fake
def _nf4_linear_fake(x, qweight, absmax, code, out_features, in_features, blocksize, bias=None):
    return x.new_empty((*x.shape[:-1], out_features))


def _nf4_setup(ctx, inputs, output):
    x, qweight, absmax, code, out_features, in_features, blocksize, bias = inputs
    ctx.save_for_backward(qweight, absmax, code)
    ctx.meta = (out_features, in_features, blocksize, x.dtype, bias is not None)


def _nf4_backward(ctx, g):
    qweight, absmax, code = ctx.saved_tensors
    out_f, in_f, bs, dt, has_bias = ctx.meta
    w = dequantize_nf4(qweight, absmax, (out_f, in_f), dt, bs, code)
    gx = g @ w
    gb = g.reshape(-1, out_f).sum(0) if has_bias else None
    return gx, None, None, None, None, None, None, gb


nf4_linear.register_autograd(_nf4_backward, setup_context=_nf4_setup)


class _NF4Forward:
    def __init__(self, mod, blocksize):
        self.mod = mod
        self.blocksize = blocksize

    def __call__(self, x):
        m = self.mod
        return nf4_linear(x, m.qweight, m.absmax, m.nf4_code, m.out_features, m.in_features, self.blocksize, m.bias)


class NF4LinearQuant4bit(Transform):
    """Quantizes every ``nn.Linear`` (or those named in ``modules``) to NF4 in ``transform_module``."""

    def __init__(self, blocksize: int = 64, modules: list[str] | None = None, skip: tuple[str, ...] = ("lm_head",)):
        self.blocksize = blocksize
        self.modules = modules
        self.skip = skip
        self.quantized: list[str] = []

    def transform_module(self, model) -> None:
        for name, m in model._model.named_modules():
            if not isinstance(m, torch.nn.Linear) or hasattr(m, "qweight"):
                continue
            if self.modules is not None and name not in self.modules:
                continue
            if any(name.endswith(s) for s in self.skip):
                continue
            if m.weight.numel() % self.blocksize:
                continue
            q, a = quantize_nf4(m.weight, self.blocksize)
            dev = m.weight.device
            del m.weight
            m.register_buffer("qweight", q.to(dev))
            m.register_buffer("absmax", a.to(dev))
            m.register_buffer("nf4_code", NF4_CODE.to(dev))
            m.forward = _NF4Forward(m, self.blocksize)
            self.quantized.append(name)

    def transform_state_dict_for_submodule(self, model, submodule_name, state_dict):
        if submodule_name not in self.quantized or "weight" not in state_dict:
            return state_dict
        sd = dict(state_dict)
        q, a = quantize_nf4(sd.pop("weight"), self.blocksize)
        sd["qweight"], sd["absmax"], sd["nf4_code"] = q, a, NF4_CODE.clone()
        return sd


BitsAndBytesLinearQuant4bit = NF4LinearQuant4bit  # API-compatible name
