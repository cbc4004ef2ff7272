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


def _restart_on_manual_seed():
    """``torch.manual_seed(s)`` restarts the counter even when ``s`` equals the current seed, so that
    re-seeding with the same value replays the same dropout masks (as ATen's generators do); the seed
    comparison in :func:`next_seed_offset` alone only catches a changed seed."""
    import functools

    orig = torch.manual_seed
    if getattr(orig, "_lta_restarts_philox", False):
        return

    @functools.wraps(orig)
    def manual_seed(seed):
        with _lock:
            _state["seed"] = None
        return orig(seed)

    manual_seed._lta_restarts_philox = True
    torch.manual_seed = manual_seed
    torch.random.manual_seed = manual_seed


_restart_on_manual_seed()


# ---------------------------------------------------------------------------------------------
# Graph-safe RNG: inside a captured hipGraph the kernels' seed / offset arguments are baked into the
# graph, so a replay would reuse the capture's dropout masks.  While a HipGraphRunner captures, every
# ``get_rng_seed_offset`` returns ``GraphRngInt`` values instead of plain ints: the seed and an offset
# RELATIVE to the region's Philox base, both carrying the region's device RNG state (int64 [seed, base]).
# The consumers (hipfuse Philox kernels, attention dropout, the torch fallback) read seed and base from
# that state, so the runner only rewrites the state (one small launch) before each replay, drawing
# ``base = next_seed_offset(total)`` for the whole region: the same counter ranges, in the same order, as
# an uncaptured run.  The backward receives the forward's GraphRngInt values and recomputes the masks from
# the same state (requirement, as for delayed scaling: each forward's backward runs before the forward's
# region replays again).  Reference counterpart: PyTorch's graph-safe Philox state (offset_extragraph).
# ---------------------------------------------------------------------------------------------
class GraphRngInt(int):
    """An RNG seed / relative offset drawn inside a graph capture (see above)."""

    def __new__(cls, value: int, state: torch.Tensor, kind: str):
        o = int.__new__(cls, value)
        o.state = state
        o.kind = kind  # "seed" | "offset"
        return o

    def __repr__(self):
        return f"GraphRngInt({int(self)}, {self.kind})"

    def __reduce__(self):  # pickles / deep copies as the plain value it stands for
        return (int, (int(self),))


class GraphRngContext:
    """The RNG draws of one region run under a hipGraph runner: ``state`` (int64 [2] on the device) and
    the running total.  ``on_first_draw(state)`` (the runner's uncaptured warm-up call) writes the live
    (seed, offset) into the state before the first consumer kernel is enqueued; the caller then
    advances the counter by ``total`` (:func:`advance_offset`)."""

    def __init__(self, state: torch.Tensor, on_first_draw=None):
        self.state = state
        self.total = 0
        self.on_first_draw = on_first_draw

    def draw(self, numel: int):
        if self.total == 0 and self.on_first_draw is not None:
            self.on_first_draw(self.state)
        with _lock:
            rel = self.total
            self.total += int(numel)
        return GraphRngInt(0, self.state, "seed"), GraphRngInt(rel, self.state, "offset")


def peek_seed_offset() -> tuple[int, int]:
    """(seed, offset) the next ``next_seed_offset`` call would return, without advancing."""
    with _lock:
        seed = torch.initial_seed() & _MASK32
        if _state["seed"] != seed:
            _state["seed"] = seed
            _state["offset"] = 0
        return seed, _state["offset"]


def advance_offset(numel: int) -> None:
    with _lock:
        _state["offset"] += int(numel)


_graph_ctx = threading.local()


def graph_context():
    return getattr(_graph_ctx, "ctx", None)


def set_graph_context(ctx) -> None:
    _graph_ctx.ctx = ctx


def seed_offset_for(numel: int):
    """``next_seed_offset`` outside a capture; GraphRngInt (seed, relative offset) inside one."""
    ctx = graph_context()
    if ctx is not None:
        return ctx.draw(numel)
    return next_seed_offset(numel)


def is_graph_rng(*vals) -> bool:
    return any(type(v) is GraphRngInt for v in vals)


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
    if is_graph_rng(seed, offset):  # seed / base from the region's device state (graph-safe RNG)
        st = (seed if type(seed) is GraphRngInt else offset).state
        off = st[1] + int(offset)
        c2 = (off & _MASK32).expand_as(blk)
        c3 = ((off >> 32) & _MASK32).expand_as(blk)
        k0 = st[0] & _MASK32
    else:
        seed, offset = int(seed), int(offset)
        c2 = torch.full_like(blk, offset & _MASK32)
        c3 = torch.full_like(blk, (offset >> 32) & _MASK32)
        k0 = seed & _MASK32
    words = philox4x32(c0, c1, c2, c3, k0, 0)
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
