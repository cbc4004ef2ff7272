"""Counter-based RNG (Philox4x32-10) shared by every execution path (K13).

``uniform_philox(shape, seed, offset)`` is a *pure function* of (seed, offset, element index):
element e of the output is ``philox(counter=(e_lo, e_hi, off_lo, off_hi), key=(seed, 0))[0]``
mapped to [0, 1) with 24 random bits.  hipfuse generates the same arithmetic inline in its
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
    e = torch.arange(n, device=device, dtype=torch.int64)
    c0 = e & _MASK32
    c1 = (e >> 32) & _MASK32
    c2 = torch.full_like(e, offset & _MASK32)
    c3 = torch.full_like(e, (offset >> 32) & _MASK32)
    k0, k1 = seed & _MASK32, 0
    for _ in range(10):
        hi0, lo0 = _mulhilo(c0, M0)
        hi1, lo1 = _mulhilo(c2, M1)
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & _MASK32, lo1, (hi0 ^ c3 ^ k1) & _MASK32, lo0
        k0 = (k0 + W0) & _MASK32
        k1 = (k1 + W1) & _MASK32
    u = (c0 >> 8).to(torch.float32) * (1.0 / 16777216.0)
    return u.reshape(tuple(shape)).to(dtype)


# HIP version (inlined by the fusion code generator)
PHILOX_HIP = r"""
__device__ __forceinline__ float philox_uniform(unsigned seed, unsigned long long off, unsigned long long e) {
  unsigned c0 = (unsigned)e, c1 = (unsigned)(e >> 32), c2 = (unsigned)off, c3 = (unsigned)(off >> 32);
  unsigned k0 = seed, k1 = 0u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c0;
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c2;
    const unsigned n0 = (unsigned)(p1 >> 32) ^ c1 ^ k0, n2 = (unsigned)(p0 >> 32) ^ c3 ^ k1;
    c1 = (unsigned)p1; c3 = (unsigned)p0; c0 = n0; c2 = n2;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return (float)(c0 >> 8) * (1.0f / 16777216.0f);
}
"""
