"""Counter-based RNG (Philox4x32-10) shared by every execution path (K13).

``uniform_philox(shape, seed, offset)`` is a *pure function* of (seed, offset, element index):
element e of the output is word ``e % 4`` of ``philox(counter=(b_lo, b_hi, off_lo, off_hi),
key=(seed, 0))`` for the block b = e // 4, mapped to [0, 1) with 24 random bits — one Philox
evaluation per 4 elements (the generated kernels draw a whole block per 4 vector lanes).  hipfuse generates the same arithmetic inline in its
kernels (``hipfuse_codegen._PREAMBLE``), the torch executor evaluates it with int64 tensor ops
(below), so a dropout mask produced in a fused forward kernel is reproduced bit-exactly in the
backward — the mask is *recomputed*, never saved (reference: nvFuser's uniform_philox +
``get_and_update_rng_state``; the reference keeps ATen's Philox stream instead).

``next_seed_offset(numel)`` hands out disjoint counter ranges: the seed follows
``torch.initial_seed()`` (so ``torch.manual_seed`` makes runs reproducible) and the offset
advances by ``numel`` per call.
"""
from __future__ import annotations

import threading

import torch

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
_MASK32 = 0xFFFFFFFF

_lock = threading.Lock()
_state = {"seed": None, "offset": 0}


def next_seed_offset(numel: int) -> tuple[int, int]:
    with _lock:
        seed = torch.initial_seed() & _MASK32
        if _state["seed"] != seed:
            _state["seed"] = seed
            _state["offset"] = 0
        off = _state["offset"]
        _state["offset"] = off + int(numel)
        return seed, off


def _mulhilo(a: torch.Tensor, b: int):
    """(hi32, lo32) of a * b for a int64 tensor of uint32 values and a 32-bit constant b (exact)."""
    b_hi, b_lo = b >> 16, b & 0xFFFF
    t = a * b_lo                 # < 2^48
    hi = (a * b_hi + (t >> 16)) >> 16
    lo = ((a * b_hi) << 16) + t  # mod 2^32 below
    return hi & _MASK32, lo & _MASK32


def philox_uniform_torch(shape, seed: int, offset: int, device, dtype=torch.float32) -> torch.Tensor:
    n = 1
    for s in shape:
        n *= s
    blk = torch.arange((n + 3) // 4, device=device, dtype=torch.int64)
    c0 = blk & _MASK32
    c1 = (blk >> 32) & _MASK32
    c2 = torch.full_like(blk, offset & _MASK32)
    c3 = torch.full_like(blk, (offset >> 32) & _MASK32)
    words = philox4x32(c0, c1, c2, c3, seed & _MASK32, 0)
    w = torch.stack(words, dim=1).reshape(-1)[:n]
    u = (w >> 8).to(torch.float32) * (1.0 / 16777216.0)
    return u.reshape(tuple(shape)).to(dtype)


def philox4x32(c0, c1, c2, c3, k0: int, k1: int):
    """Philox4x32-10 block function on int64 tensors of uint32 words (Random123's philox4x32_R(10))."""
    for _ in range(10):
        hi0, lo0 = _mulhilo(c0, M0)
        hi1, lo1 = _mulhilo(c2, M1)
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & _MASK32, lo1, (hi0 ^ c3 ^ k1) & _MASK32, lo0
        k0 = (k0 + W0) & _MASK32
        k1 = (k1 + W1) & _MASK32
    return c0, c1, c2, c3


# HIP version (inlined by the fusion code generator)
PHILOX_HIP = r"""
__device__ __forceinline__ void philox4(unsigned seed, unsigned long long off, unsigned long long blk, unsigned* w) {
  unsigned c0 = (unsigned)blk, c1 = (unsigned)(blk >> 32), c2 = (unsigned)off, c3 = (unsigned)(off >> 32);
  unsigned k0 = seed, k1 = 0u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c0;
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c2;
    const unsigned n0 = (unsigned)(p1 >> 32) ^ c1 ^ k0, n2 = (unsigned)(p0 >> 32) ^ c3 ^ k1;
    c1 = (unsigned)p1; c3 = (unsigned)p0; c0 = n0; c2 = n2;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  w[0] = c0; w[1] = c1; w[2] = c2; w[3] = c3;
}
__device__ __forceinline__ float philox_u24(unsigned x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }
__device__ __forceinline__ float philox_uniform(unsigned seed, unsigned long long off, unsigned long long e) {
  unsigned w[4];
  philox4(seed, off, e >> 2, w);
  const unsigned q = (unsigned)e & 3u;
  return philox_u24(q == 0u ? w[0] : q == 1u ? w[1] : q == 2u ? w[2] : w[3]);
}
"""
