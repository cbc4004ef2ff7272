"""FP8 (OCP e4m3fn / e5m2) kernels for the FP8 linear path (K8): casts, cast+transpose and the
hand-written block-scaled-MFMA GEMM (``csrc/fp8.hip``, ``csrc/gemm.hip``)."""
from __future__ import annotations

import torch

from ._lib import require, stream_ptr, check, register_signature, c_int, c_int64, c_void_p, c_float, DTYPE_CODE

E4M3_MAX = 448.0
E5M2_MAX = 57344.0

register_signature("lta_amax", [c_int, c_void_p, c_int64, c_void_p, c_void_p])
register_signature("lta_fp8_cast", [c_int, c_int, c_void_p, c_void_p, c_int64, c_void_p, c_float, c_void_p, c_void_p,
                                    c_void_p])
register_signature("lta_fp8_cast_transpose", [c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p,
                                              c_float, c_void_p, c_void_p, c_void_p])
register_signature("lta_gemm_nt_fp8", [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                       c_int, c_int, c_int, c_void_p, c_void_p, c_void_p])


def amax_into(x: torch.Tensor, out: torch.Tensor) -> None:
    """out (fp32 device scalar, zero-initialised) = max(out, max |x|) — one read of x, no temporaries."""
    check(require().lta_amax(DTYPE_CODE[x.dtype], x.data_ptr(), x.numel(), out.data_ptr(), stream_ptr(x.device)),
          "lta_amax")


def scale_for(t: torch.Tensor, fmax: float, margin: float = 0.0) -> torch.Tensor:
    """Per-tensor scale as a device scalar (reference helper; the kernels derive it on device)."""
    amax = torch.zeros((), dtype=torch.float32, device=t.device)
    amax_into(t, amax)
    return (fmax / amax.clamp_min(1e-12)) * (2.0 ** -margin)


def cast(x: torch.Tensor, amax: torch.Tensor, fmax: float, scale_out: torch.Tensor | None = None,
         e5m2: bool = False, amax_out: torch.Tensor | None = None):
    """fp8(x * fmax / amax) as uint8 storage; the scale used is written to ``scale_out``."""
    lib = require()
    y = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    check(lib.lta_fp8_cast(DTYPE_CODE[x.dtype], int(e5m2), x.data_ptr(), y.data_ptr(), x.numel(), amax.data_ptr(), fmax,
                           None if scale_out is None else scale_out.data_ptr(),
                           None if amax_out is None else amax_out.data_ptr(), stream_ptr(x.device)), "lta_fp8_cast")
    return y


def cast_transpose(x2d: torch.Tensor, amax: torch.Tensor, fmax: float, scale_out: torch.Tensor | None = None,
                   e5m2: bool = False, rowmajor: bool = True, amax_out: torch.Tensor | None = None):
    """x [R, C] -> (fp8 [R, C] or None, fp8 [C, R]) as uint8 storage."""
    lib = require()
    R, C = x2d.shape
    y = torch.empty((R, C), dtype=torch.uint8, device=x2d.device) if rowmajor else None
    yt = torch.empty((C, R), dtype=torch.uint8, device=x2d.device)
    check(lib.lta_fp8_cast_transpose(DTYPE_CODE[x2d.dtype], int(e5m2), x2d.data_ptr(),
                                     None if y is None else y.data_ptr(), yt.data_ptr(), R, C, amax.data_ptr(), fmax,
                                     None if scale_out is None else scale_out.data_ptr(),
                                     None if amax_out is None else amax_out.data_ptr(), stream_ptr(x2d.device)),
          "lta_fp8_cast_transpose")
    return y, yt


register_signature("lta_gemm4_fp8", [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                      c_int, c_int, c_int, c_void_p, c_void_p, c_void_p])


def gemm4_fp8_supported(a: torch.Tensor, b: torch.Tensor) -> bool:
    """The 4-wave fp8 kernel (csrc/gemm4_fp8.hip): M, N % 256, K % 256, 16-B aligned rows."""
    M, K = a.shape
    N = b.shape[0]
    return (M % 256 == 0 and N % 256 == 0 and K % 256 == 0 and a.stride(1) == 1 and b.stride(1) == 1
            and a.stride(0) % 16 == 0 and b.stride(0) % 16 == 0 and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0
            and M * a.stride(0) < 2**31 and N * b.stride(0) < 2**31)


register_signature("lta_gemm4_fp8_res", [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                          c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p])


def gemm_nt_fp8(a: torch.Tensor, b: torch.Tensor, sa: torch.Tensor, sb: torch.Tensor, fmt_a: int = 0, fmt_b: int = 0,
                bias: torch.Tensor | None = None, residual: torch.Tensor | None = None) -> torch.Tensor:
    """bf16 [M, N] = (a [M,K] . b[N,K]^T) / (sa * sb) (+ bias); a/b fp8 as uint8, sa/sb device scalars.
    The 4-wave pipelined kernel (gemm4_fp8) when the shape tiles, else the 8-wave one (gemm.hip)."""
    lib = require()
    M, K = a.shape
    N = b.shape[0]
    out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    if residual is not None:
        r2 = residual.reshape(M, N)
        if (gemm4_fp8_supported(a, b) and r2.dtype == torch.bfloat16 and r2.stride(1) == 1 and r2.stride(0) % 8 == 0
                and r2.data_ptr() % 16 == 0):
            check(lib.lta_gemm4_fp8_res(a.data_ptr(), b.data_ptr(), out.data_ptr(),
                                        None if bias is None else bias.data_ptr(), r2.data_ptr(), M, N, K, a.stride(0),
                                        b.stride(0), out.stride(0), r2.stride(0), fmt_a, fmt_b, sa.data_ptr(),
                                        sb.data_ptr(), stream_ptr(a.device)), "lta_gemm4_fp8_res")
            return out
        return gemm_nt_fp8(a, b, sa, sb, fmt_a, fmt_b, bias) + r2
    fn, name = ((lib.lta_gemm4_fp8, "lta_gemm4_fp8") if gemm4_fp8_supported(a, b)
                else (lib.lta_gemm_nt_fp8, "lta_gemm_nt_fp8"))
    check(fn(a.data_ptr(), b.data_ptr(), out.data_ptr(), None if bias is None else bias.data_ptr(), M, N, K,
             a.stride(0), b.stride(0), out.stride(0), fmt_a, fmt_b, sa.data_ptr(), sb.data_ptr(), stream_ptr(a.device)),
          name)
    return out


register_signature("lta_gemm4_fp8_qkv_rope", [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                              c_int, c_int, c_void_p])


def gemm_qkv_rope(qa: torch.Tensor, qb: torch.Tensor, sa: torch.Tensor, sb: torch.Tensor, out_shape, cos: torch.Tensor,
                  sin: torch.Tensor, n_head: int, n_query_groups: int, head_size: int, rope_n: int):
    """``q, k, v = qkv_split_rope(gemm(qa, qb) / (sa sb))`` for the e4m3 attention input projection:
    the RoPE split runs in the fp8 GEMM's epilogue (csrc/gemm4_fp8.hip QKV) when supported, else
    the GEMM then csrc/rope.hip.  ``out_shape`` = (B, T, N) of the unfused projection."""
    import os

    from .gemm import _rope_halves_equal
    from .fused import qkv_rope_fwd

    B, T, N = out_shape
    M, K = qa.shape
    ok = (os.environ.get("LTA_FUSED_QKV_ROPE", "1") != "0" and head_size == 128 and rope_n == 128
          and N == (n_head + 2 * n_query_groups) * 128 and tuple(qb.shape) == (N, K) and M == B * T
          and gemm4_fp8_supported(qa, qb) and cos.dtype == torch.float32 and sin.dtype == torch.float32
          and cos.dim() == 2 and sin.dim() == 2 and cos.shape[-1] == 128 and sin.shape[-1] == 128
          and cos.shape[0] >= T and sin.shape[0] >= T)
    if ok and _rope_halves_equal(cos, sin, T):
        c = cos[:T].contiguous()
        s_ = sin[:T].contiguous()
        q = torch.empty((B, n_head, T, 128), dtype=torch.bfloat16, device=qa.device)
        k = torch.empty((B, n_query_groups, T, 128), dtype=torch.bfloat16, device=qa.device)
        v = torch.empty_like(k)
        check(require().lta_gemm4_fp8_qkv_rope(qa.data_ptr(), qb.data_ptr(), sa.data_ptr(), sb.data_ptr(), c.data_ptr(),
                                               s_.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), M, K,
                                               qa.stride(0), qb.stride(0), T, n_head, n_query_groups, 0, 0,
                                               stream_ptr(qa.device)), "lta_gemm4_fp8_qkv_rope")
        return q, k, v
    return qkv_rope_fwd(gemm(qa, qb, sa, sb, 0, 0, None, out_shape), cos, sin, n_head, n_query_groups, head_size,
                        rope_n)


register_signature("lta_gemm_grouped_nt_fp8", [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                                c_int64, c_void_p, c_void_p, c_void_p])


def grouped_mm_fp8(qa: torch.Tensor, qw: torch.Tensor, sa: torch.Tensor, sw: torch.Tensor,
                   offs: torch.Tensor) -> torch.Tensor:
    """bf16 [M, N]: rows of group g of ``qa`` ([M, K] e4m3 as uint8, device scalar scale ``sa``)
    times expert g's ``qw[g]`` ([G, N, K] e4m3, scales ``sw`` [G]); ``offs`` int32 row ends."""
    lib = require()
    M, K = qa.shape
    G, N, _ = qw.shape
    out = torch.empty((M, N), dtype=torch.bfloat16, device=qa.device)
    check(lib.lta_gemm_grouped_nt_fp8(qa.data_ptr(), qw.data_ptr(), out.data_ptr(), offs.data_ptr(), G, M, N, K,
                                      qw.stride(0), sa.data_ptr(), sw.data_ptr(), stream_ptr(qa.device)),
          "lta_gemm_grouped_nt_fp8")
    return out


register_signature("lta_gemm4_fp8_layout", [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                             c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p])


def gemm_fp8_layout(a: torch.Tensor, b: torch.Tensor, sa: torch.Tensor, sb: torch.Tensor, fmt_a: int, at: bool,
                    residual: torch.Tensor | None = None) -> torch.Tensor:
    """bf16 C = (opA . opB) / (sa sb) (+ residual) reading the backward's operands where they are,
    without transposed fp8 copies: B is stored [K][N] (the weight [out][in] for the dgrad, the saved
    activation [tokens][in] for the wgrad); A is [M][K] (``at`` False: dY for the dgrad) or stored
    [K][M] (``at`` True: dY [tokens][out] for the wgrad).  fp8 as uint8, scales device scalars."""
    K, N = b.shape
    M = a.shape[1] if at else a.shape[0]
    assert (a.shape[0] if at else a.shape[1]) == K and a.stride(1) == 1 and b.stride(1) == 1
    out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    r2 = None
    if residual is not None:
        r2 = residual.reshape(M, N)
        assert not at and r2.dtype == torch.bfloat16 and r2.stride(1) == 1
    check(require().lta_gemm4_fp8_layout(a.data_ptr(), b.data_ptr(), out.data_ptr(),
                                         None if r2 is None else r2.data_ptr(), M, N, K, a.stride(0), b.stride(0),
                                         out.stride(0), 0 if r2 is None else r2.stride(0), fmt_a, 0, int(at), 1,
                                         sa.data_ptr(), sb.data_ptr(), stream_ptr(a.device)), "lta_gemm4_fp8_layout")
    return out


def quantize_rows(t: torch.Tensor, e5m2: bool = False):
    """t (any shape, last dim C) -> (q [R, C], scale): per-tensor current scaling, row-major copy only
    (the backward GEMMs read it in place through transposed LDS reads)."""
    t2 = t.reshape(-1, t.shape[-1])
    st = torch.zeros(2, dtype=torch.float32, device=t.device)  # amax, scale
    amax_into(t2, st[0])
    q = cast(t2, st[0], E5M2_MAX if e5m2 else E4M3_MAX, st[1], e5m2=e5m2)
    return q, st[1]


def fp8_linear_supported(M: int, N: int, K: int) -> bool:
    return M % 256 == 0 and N % 256 == 0 and K % 256 == 0


def fp8_linear_fwd(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None):
    """y = x @ w^T + b with e4m3 operands.  Returns (y, x^T fp8, w^T fp8, scales[sx, sw]) —
    the transposed copies are what the backward's dgrad/wgrad GEMMs read.  Per call: one amax
    pass and one cast(+transpose) pass per operand; the scales never leave the device."""
    K = x.shape[-1]
    N = w.shape[0]
    x2 = x.reshape(-1, K)
    st = torch.zeros(4, dtype=torch.float32, device=x.device)  # amax_x, amax_w, s_x, s_w
    amax_into(x2, st[0])
    amax_into(w, st[1])
    qx, qxT = cast_transpose(x2, st[0], E4M3_MAX, st[2])
    qw, qwT = cast_transpose(w, st[1], E4M3_MAX, st[3])
    scales = st[2:4]
    y = gemm_nt_fp8(qx, qw, st[2], st[3], 0, 0, bias)
    return y.reshape(*x.shape[:-1], N), qxT, qwT, scales


def fp8_linear_bwd(dy: torch.Tensor, qxT: torch.Tensor, qwT: torch.Tensor, scales: torch.Tensor, has_bias: bool,
                   x_shape):
    N = dy.shape[-1]
    dy2 = dy.reshape(-1, N)
    st = torch.zeros(4, dtype=torch.float32, device=dy.device)  # amax_dy, s_dy, (s_dy, s_w) / (s_dy, s_x) below
    amax_into(dy2, st[0])
    qdy, qdyT = cast_transpose(dy2, st[0], E5M2_MAX, st[1], e5m2=True)
    dx = gemm_nt_fp8(qdy, qwT, st[1], scales[1], 1, 0)   # [M, K]
    dw = gemm_nt_fp8(qdyT, qxT, st[1], scales[0], 1, 0)  # [N, K]
    db = dy2.sum(0) if has_bias else None
    return dx.reshape(x_shape), dw, db


def quantize(t: torch.Tensor, e5m2: bool = False):
    """t (any shape, last dim C) -> (q [R, C], q^T [C, R], scale) with per-tensor current scaling."""
    t2 = t.reshape(-1, t.shape[-1])
    st = torch.zeros(2, dtype=torch.float32, device=t.device)  # amax, scale
    amax_into(t2, st[0])
    q, qT = cast_transpose(t2, st[0], E5M2_MAX if e5m2 else E4M3_MAX, st[1], e5m2=e5m2)
    return q, qT, st[1]


def gemm(qa: torch.Tensor, qb: torch.Tensor, sa: torch.Tensor, sb: torch.Tensor, fmt_a: int, fmt_b: int,
         bias: torch.Tensor | None, out_shape, residual: torch.Tensor | None = None) -> torch.Tensor:
    return gemm_nt_fp8(qa, qb, sa, sb, fmt_a, fmt_b, bias, residual).reshape(out_shape)


# ---------------------------------------------------------------------------------------------
# Delayed scaling (TransformerEngine ``DelayedScaling`` recipe; reference
# thunder/executors/transformer_engineex_impl.py:49-515, te_fp8_amax_and_scale_update)
# ---------------------------------------------------------------------------------------------
class DelayedScaling:
    """Scale of each quantised tensor = fp8_max / max(amax history) / 2^margin.

    Every quantisation folds its tensor's amax into the current-step slot *while casting* (the cast
    kernel's amax output), so no separate amax pass runs; the history advances once per forward
    (``delayed_update``), after an all-reduce(MAX) of the current amaxes over ``process_group``
    (default: the world group when torch.distributed is initialised, ``reduce_amax=True``), so every
    data-parallel rank uses identical scales.  A slot's first use falls back to current scaling."""

    def __init__(self, amax_history_len: int = 16, margin: int = 0, reduce_amax: bool = True, process_group=None):
        self.amax_history_len = amax_history_len
        self.margin = margin
        self.reduce_amax = reduce_amax
        self.process_group = process_group

    def __repr__(self):
        return f"DelayedScaling(amax_history_len={self.amax_history_len}, margin={self.margin}, " \
               f"reduce_amax={self.reduce_amax})"


class _DelayedState:
    def __init__(self, recipe: DelayedScaling, n_slots: int):
        self.recipe = recipe
        self.hist = self.cur = self.hmax = None
        self.step_amax = None  # first-step amax of a slot (current scaling: no history yet)
        self.updates = 0
        self.resize(n_slots)

    def resize(self, n_slots: int) -> None:
        """Set the slot count (before the first quantisation; the transform knows it only after it
        has rewritten the trace)."""
        self.n = n_slots
        self.step_src = [None] * n_slots  # the amax tensor each slot is scaled from in this step
        self.seen = [False] * n_slots
        self.step_seen = [-1] * n_slots  # the step (``updates``) a slot was last quantised in

    def ensure(self, device):
        if self.hist is None:
            z = lambda *shape: torch.zeros(shape, dtype=torch.float32, device=device)  # noqa: E731
            self.hist, self.cur, self.hmax = z(self.recipe.amax_history_len, self.n), z(self.n), z(self.n)
            self.step_amax = z(self.n)
            # max |w| of each slot's fp8 weight shadow (written when the shadow is (re)cast), folded into the
            # step's amaxes by delayed_update: a forward that reads a shadow launches no cast to record it
            self.shadow_amax = z(self.n)
            self.has_shadow = False

    def group(self):
        import torch.distributed as tdist

        if not self.recipe.reduce_amax or not tdist.is_available() or not tdist.is_initialized():
            return None
        g = self.recipe.process_group
        return g if g is not None else tdist.distributed_c10d._get_default_group()


_DELAYED: dict[int, _DelayedState] = {}
_DELAYED_KEYS = iter(range(1 << 62))


def new_delayed_state(recipe: DelayedScaling, n_slots: int) -> int:
    key = next(_DELAYED_KEYS)
    _DELAYED[key] = _DelayedState(recipe, n_slots)
    return key


def release_delayed_state(key: int) -> None:
    """Drop a state no program uses (the transform registered it, then converted no linear)."""
    _DELAYED.pop(key, None)


def delayed_state(key: int) -> _DelayedState:
    return _DELAYED[key]


def delayed_update(key: int) -> None:
    """Advance the amax history by one step (device-only: graph-capturable but for the collective)."""
    st = _DELAYED[key]
    if st.hist is None:
        return
    if st.has_shadow:
        torch.maximum(st.cur, st.shadow_amax, out=st.cur)
    g = st.group()
    if g is not None and torch.distributed.get_world_size(g) > 1:
        torch.distributed.all_reduce(st.cur, op=torch.distributed.ReduceOp.MAX, group=g)
    h = st.hist
    if h.shape[0] > 1:
        h[1:] = h[:-1].clone()
    h[0] = st.cur
    torch.amax(h, 0, out=st.hmax)
    st.cur.zero_()
    st.updates += 1


def quantize_delayed(t: torch.Tensor, e5m2: bool, key: int, slot: int):
    """As :func:`quantize`, scaled from the slot's amax history; the tensor's own amax goes to the
    slot's current-step entry.  Returns (q, q^T, scale) with a private scale scalar.

    Every later quantisation of the slot within the same step — a sibling linear reading the same
    input, or the backward's recompute of an activation-checkpointed region — is scaled from the
    very amax the first one used, so the recompute reproduces the forward's fp8 values bit for bit
    (also on a slot's first step, where the forward fell back to current scaling and the history is
    still empty); its amax contribution is the same max again (reference: TE's recompute-phase
    handling, thunder/executors/transformer_engineex_impl.py:459-515).

    Requirement: each forward is followed by its own backward before the next forward (f1 b1 f2 b2).
    The scaling source is the live history max, which ``delayed_update`` advances at the start of
    every forward; with interleaved schedules (f1 f2 b2 b1: pipelining, or accumulation that runs
    several forwards first) the recompute of f1's checkpointed region inside b1 would read f2's
    scaling source and no longer reproduce f1's fp8 values bit for bit."""
    st = _DELAYED[key]
    st.ensure(t.device)
    t2 = t.reshape(-1, t.shape[-1])
    fmax = (E5M2_MAX if e5m2 else E4M3_MAX) * 2.0 ** -st.recipe.margin
    scale = torch.empty((), dtype=torch.float32, device=t.device)
    if st.step_seen[slot] != st.updates:  # first quantisation of the slot in this step
        st.step_seen[slot] = st.updates
        if st.seen[slot]:
            # the history max itself (a view: hmax only changes in delayed_update, after the step's
            # last quantisation), not a per-slot device copy of it (a 4-byte memcpy launch each)
            st.step_src[slot] = st.hmax[slot]
        else:  # first use of the slot: no history yet -> current scaling for this step
            st.seen[slot] = True
            amax_in = st.step_amax[slot]
            amax_in.zero_()
            amax_into(t2, amax_in)
            st.step_src[slot] = amax_in
    amax_in = st.step_src[slot]
    q, qT = cast_transpose(t2, amax_in, fmax, scale, e5m2=e5m2, amax_out=st.cur[slot])
    return q, qT, scale


def delayed_scaling_source(t2: torch.Tensor, e5m2: bool, key: int, slot: int):
    """(amax source tensor, fmax, fresh scale scalar, amax sink) of a delayed-scaling quantisation of
    the 2-D ``t2`` in ``slot`` -- the bookkeeping of :func:`quantize_delayed`, for kernels that cast
    as a side output of their own pass (row casts, producer-fused casts)."""
    st = _DELAYED[key]
    st.ensure(t2.device)
    fmax = (E5M2_MAX if e5m2 else E4M3_MAX) * 2.0 ** -st.recipe.margin
    scale = torch.empty((), dtype=torch.float32, device=t2.device)
    if st.step_seen[slot] != st.updates:
        st.step_seen[slot] = st.updates
        if st.seen[slot]:
            st.step_src[slot] = st.hmax[slot]
        else:
            st.seen[slot] = True
            amax_in = st.step_amax[slot]
            amax_in.zero_()
            amax_into(t2, amax_in)
            st.step_src[slot] = amax_in
    return st.step_src[slot], fmax, scale, st.cur[slot]


def quantize_delayed_rows(t: torch.Tensor, e5m2: bool, key: int, slot: int):
    """As :func:`quantize_delayed` without the transposed copy: (q [R, C], scale).

    A parameter's e4m3 copy is kept as a *weight shadow* that the fused AdamW rewrites while it
    updates the weight (``optim.AdamW``, ``csrc/adamw.hip``): the next forward reads the shadow
    instead of launching a cast of the whole weight (see :func:`weight_shadow`)."""
    t2 = t.reshape(-1, t.shape[-1])
    sh = _shadow_lookup(t) if not e5m2 else None
    if sh is not None and sh.key == key and sh.slot == slot:
        st = _DELAYED[key]
        st.ensure(t.device)
        if st.step_seen[slot] != st.updates:
            st.step_seen[slot] = st.updates
            st.step_src[slot] = st.hmax[slot]
        SHADOW_STATS["reused"] += 1
        return sh.q, sh.scale
    amax_in, fmax, scale, sink = delayed_scaling_source(t2, e5m2, key, slot)
    q = cast(t2, amax_in, fmax, scale, e5m2=e5m2, amax_out=sink)
    if not e5m2 and _shadow_candidate(t):
        # a weight's slot is its own (FP8LinearTransform: one slot per linear operand), so the step's
        # amax of the slot so far is max |w|
        st = _DELAYED[key]
        st.shadow_amax[slot].copy_(sink)
        st.has_shadow = True
        _SHADOWS[t.data_ptr()] = _WeightShadow(t, q, scale, key, slot, fmax)
        SHADOW_STATS["registered"] += 1
    return q, scale


# ---------------------------------------------------------------------------------------------
# fp8 weight shadows: the e4m3 copy of a bf16 parameter, refreshed by the optimizer's update kernel
# ---------------------------------------------------------------------------------------------
class _WeightShadow:
    """e4m3 copy ``q`` of parameter ``ref()`` cast with ``scale``, valid while the parameter's version
    counter is ``version``.  The fused AdamW writes the updated weight's cast into ``q`` / ``scale``
    (scaled from the slot's amax source of the step, max |w| folded into the slot's amax history);
    any other in-place write to the parameter bumps its version and the next forward casts again."""
    __slots__ = ("ref", "q", "scale", "key", "slot", "fmax", "version", "shape")

    def __init__(self, t, q, scale, key, slot, fmax):
        import weakref

        ptr = t.data_ptr()
        # drop the registry entry (and its e4m3 copy) with the parameter
        self.ref = weakref.ref(t, lambda _r, ptr=ptr: _SHADOWS.pop(ptr, None) if _SHADOWS.get(ptr) is self else None)
        self.q, self.scale, self.key, self.slot, self.fmax = q, scale, key, slot, fmax
        self.version = t._version
        self.shape = tuple(t.shape)


_SHADOWS: dict[int, _WeightShadow] = {}
SHADOW_STATS = {"reused": 0, "registered": 0}  # forward casts skipped / shadows (re)created


def _shadows_enabled() -> bool:
    import os

    return os.environ.get("LTA_FP8_WEIGHT_SHADOW", "1") != "0"


def _shadow_candidate(t: torch.Tensor) -> bool:
    return (_shadows_enabled() and t.is_cuda and t.dtype == torch.bfloat16 and t.is_leaf and t.requires_grad
            and t.is_contiguous() and not torch.cuda.is_current_stream_capturing())


def _shadow_lookup(t: torch.Tensor):
    if not _SHADOWS or not _shadow_candidate(t):
        return None
    sh = _SHADOWS.get(t.data_ptr())
    if sh is None:
        return None
    if sh.ref() is None:  # the parameter is gone: free its e4m3 copy
        del _SHADOWS[t.data_ptr()]
        return None
    if sh.ref() is not t or sh.version != t._version or sh.shape != tuple(t.shape):
        return None
    return sh


def weight_shadow(p: torch.Tensor):
    """The optimizer's view of ``p``'s shadow: (q, amax source, scale out, delayed state, slot, fmax)
    for the update kernel to refresh (its max |w| goes to ``state.shadow_amax[slot]``, which the
    optimizer zeroes first), or None (no shadow, or stale: the next forward re-casts)."""
    sh = _shadow_lookup(p)
    if sh is None:
        return None
    st = _DELAYED.get(sh.key)
    if st is None or st.hist is None:
        return None
    src = st.step_src[sh.slot] if st.step_src[sh.slot] is not None else st.hmax[sh.slot]
    return sh.q, src, sh.scale, st, sh.slot, sh.fmax


def invalidate_weight_shadow(p: torch.Tensor) -> None:
    """``p`` changed without its shadow being refreshed (e.g. an update overlapped with the backward)."""
    _SHADOWS.pop(p.data_ptr(), None)


# ---------------------------------------------------------------------------------------------
# MXFP8 block scaling (reference: TE ``MXFP8BlockScaling``; CDNA4 runs it natively on
# v_mfma_scale_f32_16x16x128_f8f6f4 with per-32-element E8M0 scales)
# ---------------------------------------------------------------------------------------------
register_signature("lta_mx_cast_transpose", [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                             c_int, c_void_p])
register_signature("lta_gemm_nt_mxfp8", [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                         c_int, c_int, c_int, c_int, c_int, c_int, c_void_p])
register_signature("lta_fp8_mfma_scale_probe", [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p])
register_signature("lta_fp8_mfma_probe", [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p])

MX_BLOCK = 32


class MXFP8BlockScaling:
    """OCP MX: every 32 consecutive elements along a GEMM's reduction dim share one E8M0 scale;
    e4m3 for activations / weights, e5m2 for gradients (no history, no amax all-reduce)."""

    def __repr__(self):
        return "MXFP8BlockScaling()"


class MXFP4BlockScaling:
    """4-bit training recipe on CDNA4 (the MI355X counterpart of TE's ``NVFP4BlockScaling``,
    reference ``transformer_engineex_impl.py``): the forward GEMM runs on OCP MXFP4 (e2m1
    elements, E8M0 scale per 32 along K) on the block-scaled MFMA at 2x the fp8 rate; the
    backward GEMMs (dgrad, wgrad) stay MXFP8 (e5m2 gradients, e4m3 saved operands), where
    4-bit gradients would need stochastic rounding / Hadamard transforms to train stably."""

    def __repr__(self):
        return "MXFP4BlockScaling()"


def mx_quantize(t: torch.Tensor, e5m2: bool = False):
    """t [..., C] -> (q [R, C], s [R, C/32], q^T [C, R], s^T [C, R/32]): fp8 as uint8, E8M0 scales as
    uint8; blocks along C for q, along R for q^T (each is the reduction dim of the GEMM reading it)."""
    lib = require()
    t2 = t.reshape(-1, t.shape[-1])
    R, C = t2.shape
    u8 = dict(dtype=torch.uint8, device=t.device)
    q, s, qt, st = (torch.empty((R, C), **u8), torch.empty((R, C // MX_BLOCK), **u8), torch.empty((C, R), **u8),
                    torch.empty((C, R // MX_BLOCK), **u8))
    check(lib.lta_mx_cast_transpose(DTYPE_CODE[t2.dtype], int(e5m2), t2.data_ptr(), q.data_ptr(), s.data_ptr(),
                                    qt.data_ptr(), st.data_ptr(), R, C, stream_ptr(t.device)), "lta_mx_cast_transpose")
    return q, s, qt, st


def mx_dequantize(q: torch.Tensor, s: torch.Tensor, e5m2: bool = False) -> torch.Tensor:
    """Reference dequantisation (fp32) of an MX-quantised [R, C] tensor (tests / debugging)."""
    f = (torch.float8_e5m2 if e5m2 else torch.float8_e4m3fn)
    x = q.view(f).float().reshape(q.shape[0], -1, MX_BLOCK)
    scale = torch.exp2(s.float() - 127.0).unsqueeze(-1)
    return (x * scale).reshape(q.shape)


def gemm_nt_mx(a: torch.Tensor, sa: torch.Tensor, b: torch.Tensor, sb: torch.Tensor, fmt_a: int = 0, fmt_b: int = 0,
               bias: torch.Tensor | None = None) -> torch.Tensor:
    """bf16 [M, N] = a [M,K] . b [N,K]^T with E8M0 block scales sa [M, K/32], sb [N, K/32]."""
    lib = require()
    M, K = a.shape
    N = b.shape[0]
    out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    check(lib.lta_gemm_nt_mxfp8(a.data_ptr(), b.data_ptr(), out.data_ptr(), None if bias is None else bias.data_ptr(),
                                sa.data_ptr(), sb.data_ptr(), M, N, K, a.stride(0), b.stride(0), out.stride(0), fmt_a,
                                fmt_b, stream_ptr(a.device)), "lta_gemm_nt_mxfp8")
    return out


def mfma_probe(a: torch.Tensor, b: torch.Tensor, fmt_a: int, fmt_b: int) -> torch.Tensor:
    """One unscaled v_mfma_scale_f32_16x16x128_f8f6f4 from raw per-lane operand registers (formats:
    0 e4m3, 1 e5m2, 4 e2m1): a, b [64, 32] uint8 -> [64, 4] fp32 accumulator registers."""
    assert a.shape == (64, 32) and b.shape == (64, 32) and a.dtype == b.dtype == torch.uint8
    c = torch.empty((64, 4), dtype=torch.float32, device=a.device)
    check(require().lta_fp8_mfma_probe(a.contiguous().data_ptr(), b.contiguous().data_ptr(), c.data_ptr(), fmt_a,
                                       fmt_b, stream_ptr(a.device)), "lta_fp8_mfma_probe")
    return c


def mfma_scale_probe(a: torch.Tensor, b: torch.Tensor, sa: torch.Tensor, sb: torch.Tensor) -> torch.Tensor:
    """One v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3) with per-lane operand/scale registers:
    a, b [64, 32] uint8, sa, sb [64] int32 -> [64, 4] fp32 accumulator registers."""
    c = torch.empty((64, 4), dtype=torch.float32, device=a.device)
    check(require().lta_fp8_mfma_scale_probe(a.data_ptr(), b.data_ptr(), sa.data_ptr(), sb.data_ptr(), c.data_ptr(),
                                             stream_ptr(a.device)), "lta_fp8_mfma_scale_probe")
    return c


# ---------------------------------------------------------------------------------------------
# Producer-fused input casts (delayed scaling): the RMSNorm / SwiGLU forward kernels emit the e4m3
# copy the following fp8 linear reads, instead of a bf16 activation plus a separate cast pass
# (csrc/rmsnorm.hip rmsnorm_fwd_fp8_kernel, csrc/swiglu_ce.hip swiglu_fwd_fp8_kernel).  A slot's first
# quantisation (no amax history yet: current scaling of the tensor itself) takes the unfused path.
# ---------------------------------------------------------------------------------------------
register_signature("lta_rmsnorm_fwd_fp8", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_float,
                                           c_void_p, c_float, c_void_p, c_void_p, c_void_p])
register_signature("lta_swiglu_fwd_fp8", [c_int, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_float, c_void_p,
                                          c_void_p, c_void_p])


def _first_use(key: int, slot: int, device) -> bool:
    st = _DELAYED[key]
    st.ensure(device)
    return not st.seen[slot]


def rms_norm_fwd_fp8_delayed(x: torch.Tensor, w: torch.Tensor, eps: float, key: int, slot: int):
    """(q [R, C] e4m3 as uint8, scale, rstd [R]) of rms_norm(x, w) quantised in ``slot``."""
    from .rmsnorm import rms_norm_fwd

    C = x.shape[-1]
    x2 = x.reshape(-1, C)
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    if not _first_use(key, slot, x.device):
        amax_in, fmax, scale, sink = delayed_scaling_source(x2, False, key, slot)
        q = torch.empty(x2.shape, dtype=torch.uint8, device=x.device)
        rstd = torch.empty(x2.shape[0], dtype=torch.float32, device=x.device)
        rc = require().lta_rmsnorm_fwd_fp8(DTYPE_CODE[x2.dtype], x2.data_ptr(), w.contiguous().data_ptr(), q.data_ptr(),
                                           rstd.data_ptr(), x2.shape[0], C, float(eps), amax_in.data_ptr(), fmax,
                                           scale.data_ptr(), sink.data_ptr(), stream_ptr(x.device))
        if rc == 0:
            return q, scale, rstd
        if rc != -1:
            check(rc, "lta_rmsnorm_fwd_fp8")
    y, rstd = rms_norm_fwd(x2, w, eps)
    q, scale = quantize_delayed_rows(y, False, key, slot)
    return q, scale, rstd


def swiglu_fwd_fp8_delayed(a: torch.Tensor, b: torch.Tensor, key: int, slot: int):
    """(q [R, C] e4m3 as uint8, scale) of silu(a) * b quantised in ``slot``."""
    from .fused import swiglu_fwd

    C = a.shape[-1]
    if not _first_use(key, slot, a.device) and a.is_contiguous() and b.is_contiguous():
        amax_in, fmax, scale, sink = delayed_scaling_source(a.reshape(-1, C), False, key, slot)
        q = torch.empty((a.numel() // C, C), dtype=torch.uint8, device=a.device)
        rc = require().lta_swiglu_fwd_fp8(DTYPE_CODE[a.dtype], a.data_ptr(), b.data_ptr(), q.data_ptr(), a.numel(),
                                          amax_in.data_ptr(), fmax, scale.data_ptr(), sink.data_ptr(),
                                          stream_ptr(a.device))
        if rc == 0:
            return q, scale
        if rc != -1:
            check(rc, "lta_swiglu_fwd_fp8")
    return quantize_delayed_rows(swiglu_fwd(a, b), False, key, slot)


register_signature("lta_swiglu_bwd_fp8", [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p,
                                          c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p])


def swiglu_bwd_fp8_delayed(g: torch.Tensor, a: torch.Tensor, b: torch.Tensor, key: int, slot_a: int, slot_b: int):
    """(qa, sa, qb, sb): the SwiGLU input gradients da / db as e5m2 copies quantised in their slots."""
    from .fused import swiglu_bwd

    C = a.shape[-1]
    if (not _first_use(key, slot_a, a.device) and not _first_use(key, slot_b, a.device) and g.is_contiguous()
            and a.is_contiguous() and b.is_contiguous()):
        ia, fmax, sa, ka = delayed_scaling_source(a.reshape(-1, C), True, key, slot_a)
        ib, _, sb, kb = delayed_scaling_source(a.reshape(-1, C), True, key, slot_b)
        qa = torch.empty((a.numel() // C, C), dtype=torch.uint8, device=a.device)
        qb = torch.empty_like(qa)
        rc = require().lta_swiglu_bwd_fp8(DTYPE_CODE[a.dtype], g.data_ptr(), a.data_ptr(), b.data_ptr(), qa.data_ptr(),
                                          qb.data_ptr(), a.numel(), ia.data_ptr(), ib.data_ptr(), fmax, sa.data_ptr(),
                                          sb.data_ptr(), ka.data_ptr(), kb.data_ptr(), stream_ptr(a.device))
        if rc == 0:
            return qa, sa, qb, sb
        if rc != -1:
            check(rc, "lta_swiglu_bwd_fp8")
    da, db = swiglu_bwd(g, a, b)
    qa, sa = quantize_delayed_rows(da, True, key, slot_a)
    qb, sb = quantize_delayed_rows(db, True, key, slot_b)
    return qa, sa, qb, sb


def attn_fwd_fp8_delayed(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool, scale: float, key: int,
                         slot: int):
    """(o, lse, q8 [B*T, Hq*D], scale): the flash-attention forward whose output is also the input of an
    fp8 output projection: O leaves the kernel a second time as e4m3 quantised in ``slot`` (csrc
    AttnQ8 epilogue of the v4 kernel; no separate cast re-reading O).  O keeps its [B, T, Hq, D] storage,
    so the e4m3 rows are the projection input's [B*T, Hq*D] rows."""
    from .attention import attn_fwd

    B, Hq, T, D = q.shape
    if not _first_use(key, slot, q.device) and q.dtype == torch.bfloat16:
        amax_in, fmax, sc, sink = delayed_scaling_source(q, False, key, slot)  # not the first use: q unread
        q8 = torch.empty((B * T, Hq * D), dtype=torch.uint8, device=q.device)
        o, lse, used = attn_fwd(q, k, v, causal, scale, fp8_out=(q8, amax_in, fmax, sc, sink))
        if used:
            return o, lse, q8, sc
        qq, s2 = quantize_delayed_rows(o.transpose(1, 2).reshape(B * T, Hq * D), False, key, slot)
        return o, lse, qq, s2
    o, lse = attn_fwd(q, k, v, causal, scale)
    qq, s2 = quantize_delayed_rows(o.transpose(1, 2).reshape(B * T, Hq * D), False, key, slot)
    return o, lse, qq, s2


register_signature("lta_rmsnorm_bwd_fp8",[c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_int64, c_int64, c_int, c_void_p, c_void_p, c_void_p, c_float, c_void_p,
                                           c_void_p, c_void_p])


def rms_norm_bwd_fp8_delayed(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor | None, rstd: torch.Tensor,
                             residual: torch.Tensor | None, key: int, slot: int):
    """(dx, dw, q, scale): the RMSNorm backward (+ the residual stream's gradient) whose dx is also the
    output gradient of an fp8 linear, so it leaves the kernel a second time as an e5m2 copy quantised
    in ``slot`` (csrc/rmsnorm.hip Q8: no separate cast launch re-reading dx)."""
    from .rmsnorm import rms_norm_bwd, _as_2d, _bwd_blocks
    from ._lib import ptr

    C = x.shape[-1]
    if not _first_use(key, slot, x.device) and x.dtype in (torch.bfloat16, torch.float16):
        x2, rows, _ = _as_2d(x)
        dy2 = _as_2d(dy)[0]
        r2 = None if residual is None else _as_2d(residual)[0]
        wc = None if w is None else w.contiguous()
        amax_in, fmax, scale, sink = delayed_scaling_source(x2, True, key, slot)
        dx = torch.empty_like(x2)
        q = torch.empty(x2.shape, dtype=torch.uint8, device=x.device)
        nblocks = _bwd_blocks(rows)
        dw = None if wc is None else torch.empty_like(wc)
        ws = None if wc is None else torch.empty((nblocks, C), device=x.device, dtype=torch.float32)
        rc = require().lta_rmsnorm_bwd_fp8(DTYPE_CODE[x2.dtype], ptr(dy2), ptr(x2), ptr(wc), ptr(rstd), ptr(dx), ptr(dw),
                                           ptr(ws), rows, C, nblocks, ptr(r2), q.data_ptr(), amax_in.data_ptr(), fmax,
                                           scale.data_ptr(), sink.data_ptr(), stream_ptr(x.device))
        if rc == 0:
            return dx.view(x.shape), dw, q, scale
        if rc != -1:
            check(rc, "lta_rmsnorm_bwd_fp8")
    dx, dw = rms_norm_bwd(dy, x, w, rstd, residual)
    q, scale = quantize_delayed_rows(dx, True, key, slot)
    return dx, dw, q, scale
