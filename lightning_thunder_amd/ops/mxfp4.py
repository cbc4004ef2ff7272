"""MXFP4 (OCP microscaling, e2m1 elements, one E8M0 scale per 32 along the reduction dim) on CDNA4.

gfx950's block-scaled MFMA (``v_mfma_scale_f32_16x16x128_f8f6f4``, format 4) multiplies e2m1
operands at 4x the bf16 rate per clock with the E8M0 scales applied in hardware, so an MXFP4 GEMM
reads a quarter of the bf16 operand bytes and needs no dequantisation pass.  Storage: two
elements per byte (low nibble = even index, ``torch.float4_e2m1fn_x2`` layout), scales as uint8
(``torch.float8_e8m0fnu`` layout).  Kernels: ``csrc/fp8.hip`` ``mx4_cast_kernel`` (quantise) and
``csrc/gemm.hip`` ``gemm_nt_mxfp4_kernel`` (NT GEMM, bf16 out, optional bias).

The reference has no MXFP4 path (its fp4 support is the dtype, ``thunder/core/dtypes.py``); this
is the MI355X-native counterpart of its MXFP8 TransformerEngine recipe for 4-bit inference.
"""
from __future__ import annotations

import torch

from ._lib import require, stream_ptr, check, register_signature, c_int, c_int64, c_void_p, DTYPE_CODE

register_signature("lta_mxfp4_cast", [c_int, c_void_p, c_void_p, c_void_p, c_int64, c_void_p])
register_signature("lta_gemm_nt_mxfp4", [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                         c_int, c_int, c_int, c_int, c_void_p])
register_signature("lta_gemv_mxfp4", [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                      c_int, c_void_p])
GEMV_MAX_ROWS = 8

BLOCK = 32
E2M1_MAX = 6.0


def _e8m0_exponent(amax: torch.Tensor) -> torch.Tensor:
    """Biased E8M0 exponent per block: the smallest 2^s with amax / 2^s <= 6 (mantissa > 1.5 rounds
    the exponent up), 0 for an all-zero block (as ``mx4_exp`` in csrc/fp8.hip)."""
    m, e = torch.frexp(amax)  # amax = m * 2^e, m in [0.5, 1)
    e = e - 1  # floor(log2 amax)
    above = (m * 2) > 1.5
    s = e - 2 + above.to(e.dtype)
    be = torch.clamp(s + 127, 0, 254)
    return torch.where(amax > 0, be, torch.zeros_like(be)).to(torch.uint8)


def _e2m1_codes(v: torch.Tensor) -> torch.Tensor:
    """Round-to-nearest-even e2m1 codes (4-bit, sign in bit 3) of |v| <= 6."""
    a = v.abs()
    code = torch.zeros_like(a, dtype=torch.int32)
    # thresholds: (value, inclusive) — ties go to the even code
    for i, (t, incl) in enumerate(((0.25, False), (0.75, True), (1.25, False), (1.75, True), (2.5, False),
                                   (3.5, True), (5.0, False))):
        code += (a >= t if incl else a > t).to(torch.int32)
    neg = (v < 0) & (code != 0)
    return code | (neg.to(torch.int32) << 3)


def quantize_reference(x: torch.Tensor):
    """Pure-torch MXFP4 quantisation of ``x [..., C]`` along the last dim: (q [R, C/2] uint8,
    s [R, C/32] uint8) — the specification the HIP kernel is tested against."""
    x2 = x.reshape(-1, x.shape[-1]).float()
    R, C = x2.shape
    xb = x2.reshape(R, C // BLOCK, BLOCK)
    be = _e8m0_exponent(xb.abs().amax(-1))
    scale = torch.exp2(127.0 - be.float()).unsqueeze(-1)
    codes = _e2m1_codes(xb * scale).reshape(R, C)
    q = (codes[:, 0::2] | (codes[:, 1::2] << 4)).to(torch.uint8)
    return q, be


def _e2m1_value(c: torch.Tensor) -> torch.Tensor:
    """fp32 value of 4-bit e2m1 codes, computed elementwise (no host tensors: usable while a
    graph is being captured)."""
    c = c.to(torch.int32)
    e = (c >> 1) & 3
    m = (c & 1).to(torch.float32)
    mag = torch.where(e == 0, 0.5 * m, torch.exp2((e - 1).to(torch.float32)) * (1.0 + 0.5 * m))
    return torch.where((c & 8) != 0, -mag, mag)


def dequantize(q: torch.Tensor, s: torch.Tensor, dtype=torch.float32) -> torch.Tensor:
    """(q [R, C/2], s [R, C/32]) -> [R, C] (exact: every e2m1 value times a power of two)."""
    vals = torch.stack([_e2m1_value(q & 0xF), _e2m1_value(q >> 4)], -1).reshape(q.shape[0], -1)
    scale = torch.exp2(s.float() - 127.0).repeat_interleave(BLOCK, dim=1)
    return (vals * scale).to(dtype)


def quantize(x: torch.Tensor):
    """MXFP4-quantise ``x [..., C]`` (bf16 / fp32, C % 32 == 0) along the last dim on the GPU."""
    x2 = x.reshape(-1, x.shape[-1])
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    R, C = x2.shape
    if C % BLOCK:
        raise ValueError(f"MXFP4 needs the last dim to be a multiple of {BLOCK}, got {C}")
    if not x2.is_cuda:
        return quantize_reference(x2)
    q = torch.empty((R, C // 2), dtype=torch.uint8, device=x.device)
    s = torch.empty((R, C // BLOCK), dtype=torch.uint8, device=x.device)
    check(require().lta_mxfp4_cast(DTYPE_CODE[x2.dtype], x2.data_ptr(), q.data_ptr(), s.data_ptr(), x2.numel(),
                                   stream_ptr(x.device)), "lta_mxfp4_cast")
    return q, s


def gemm_nt(a: torch.Tensor, sa: torch.Tensor, b: torch.Tensor, sb: torch.Tensor,
            bias: torch.Tensor | None = None) -> torch.Tensor:
    """bf16 [M, N] = dequant(a) [M, K] . dequant(b) [N, K]^T (+ bias) on the block-scaled MFMA:
    a [M, K/2], b [N, K/2] packed e2m1; sa [M, K/32], sb [N, K/32] E8M0.  M, N % 256, K % 256."""
    M, K = a.shape[0], a.shape[1] * 2
    N = b.shape[0]
    if M % 256 or N % 256 or K % 256 or b.shape[1] * 2 != K:
        raise ValueError(f"gemm_nt_mxfp4: unsupported shape M={M} N={N} K={K}")
    if sa.shape != (M, K // BLOCK) or sb.shape != (N, K // BLOCK):
        raise ValueError("gemm_nt_mxfp4: scale shapes must be [M, K/32] and [N, K/32]")
    for t in (a, b, sa, sb):
        if not t.is_contiguous() or t.dtype != torch.uint8:
            raise ValueError("gemm_nt_mxfp4: operands and scales must be contiguous uint8")
    out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    if bias is not None:
        bias = bias.to(torch.bfloat16).contiguous()
    check(require().lta_gemm_nt_mxfp4(a.data_ptr(), b.data_ptr(), out.data_ptr(),
                                      None if bias is None else bias.data_ptr(), sa.data_ptr(), sb.data_ptr(), M, N,
                                      K, a.stride(0), b.stride(0), out.stride(0), stream_ptr(a.device)),
          "lta_gemm_nt_mxfp4")
    return out


def gemv(x: torch.Tensor, q: torch.Tensor, s: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """Weight-only MXFP4 decode product: bf16 [M, N] = x [M, K] (bf16, M <= 8) . dequant(q, s)^T (+ bias),
    streaming the 4-bit weight once (``csrc/mxfp4.hip``)."""
    x2 = x.reshape(-1, x.shape[-1])
    M, K = x2.shape
    N = q.shape[0]
    if M > GEMV_MAX_ROWS or q.shape[1] * 2 != K or s.shape != (N, K // BLOCK) or x2.dtype != torch.bfloat16:
        raise ValueError(f"gemv_mxfp4: unsupported operands x {tuple(x2.shape)} {x2.dtype}, q {tuple(q.shape)}")
    if x2.stride(-1) != 1 or x2.stride(0) % 8 or x2.data_ptr() % 16:
        x2 = x2.contiguous()  # the kernel reads x with 16-B vector loads
        if x2.data_ptr() % 16:
            x2 = x2.clone()
    y = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    if bias is not None:
        bias = bias.to(torch.bfloat16).contiguous()
    check(require().lta_gemv_mxfp4(x2.data_ptr(), q.data_ptr(), s.data_ptr(), None if bias is None else bias.data_ptr(),
                                   y.data_ptr(), M, N, K, x2.stride(0), y.stride(0), stream_ptr(x.device)),
          "lta_gemv_mxfp4")
    return y.reshape(*x.shape[:-1], N)
