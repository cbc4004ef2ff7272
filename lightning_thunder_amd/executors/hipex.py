"""hipex: the hand-written CDNA4 kernel executor (replaces the reference's cuDNN / sdpa / apex / TE /
Triton-CE executors: ``thunder/executors/{cudnnex,sdpaex,apexex,triton_crossentropy,transformer_engineex}.py``).

It claims high-level ltorch ops whole (RMSNorm, SDPA, cross-entropy, RoPE/qkv-split,
SwiGLU, ...) on HIP devices and provides *grad transforms* so autodiff saves exactly
what the fused backward kernels need (e.g. RMSNorm's per-row rstd, attention's LSE).
"""
from __future__ import annotations

import math

import torch

from ..core.prims import OpTags
from ..core.proxies import TensorProxy, pyval
from ..core import dtypes
from ..core.pytree import tree_flatten
from ..extend import OperatorExecutor, register_executor, add_default_executor

ex = OperatorExecutor("hipex", version="0.1")
register_executor(ex)
add_default_executor(ex)

hipex = ex


def _gpu(*ts) -> bool:
    return all(t is None or (isinstance(t, TensorProxy) and t.device.type == "cuda") for t in ts)


_FLOAT16ISH = (torch.bfloat16, torch.float16, torch.float32)


# =========================================================================================
# K2 GEMM: linear forward (+ fused epilogues) on the hand-written MFMA kernel
# =========================================================================================
def _linear_meta(x, w, bias=None, residual=None, act=None):
    return TensorProxy(like=x, shape=tuple(x.shape[:-1]) + (w.shape[0],))


def _linear_impl(x, w, bias=None, residual=None, act=None):
    from ..ops.gemm import linear

    return linear(x, w, bias, residual, act)


hip_linear = ex.register_operator("hip_linear", meta=_linear_meta, fn=_linear_impl)


def _linear_checker(a, w, bias=None):
    if not _gpu(a, w, bias) or a.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or w.ndim != 2:
        return False
    if bias is not None and (bias.dtype != torch.bfloat16 or bias.ndim != 1):
        return False
    if a.ndim < 2:
        return False
    M = 1
    for s in a.shape[:-1]:
        M *= s
    N, K = w.shape
    if a.shape[-1] != K:
        return False
    if M <= 8:  # decode: the weight-streaming GEMV (csrc/gemv.hip)
        return K % 8 == 0
    return _hand_gemm_shape(M, N, K)


def _hand_gemm_shape(M: int, N: int, K: int) -> bool:
    """A shape some hand GEMM tiles: gemm4 (any M >= 64 and N % 8 with edge tiles, K % 128) or the
    8-wave kernel (M, N % 256, K % 64)."""
    from ..ops.gemm import GEMM4_MIN_M

    return (M >= GEMM4_MIN_M and N % 8 == 0 and K % 128 == 0) or (M % 256 == 0 and N % 256 == 0 and K % 64 == 0)


def _linear_exec(a, w, bias=None):
    return hip_linear(a, w, bias)


def _register_linear():
    from .. import torch as ltorch

    ex.register_implementation(ltorch.linear, checker=_linear_checker, execution_transform=_linear_exec)


_register_linear()


# K2 GEMM for the prim matmul: the backward's dgrad (g @ W) and wgrad (g^T @ x) read their
# transposed operands through the transposing LDS read (csrc/gemm.hip, MN-major images)
def _mm_impl(a, b, residual=None):
    from ..ops.gemm import matmul

    return matmul(a, b, residual)


def _mm_checker(a, b):
    if not _gpu(a, b) or a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or b.ndim != 2 or a.ndim < 2:
        return False
    M = 1
    for s in a.shape[:-1]:
        M *= s
    K, N = b.shape
    return a.shape[-1] == K and _hand_gemm_shape(M, N, K)


def _mm_meta(a, b, residual=None):
    return TensorProxy(like=a, shape=tuple(a.shape[:-1]) + (b.shape[1],))


hip_matmul = ex.register_operator("hip_matmul", meta=_mm_meta, fn=_mm_impl)


def _register_matmul():
    from ..core import prims as P

    ex.register_implementation(P.matmul, checker=_mm_checker, execution_transform=lambda a, b: hip_matmul(a, b))


_register_matmul()


# =========================================================================================
# K8 FP8 linear (fwd/bwd on the block-scaled MFMA GEMM)
# =========================================================================================
def _fp8_quant_meta(t, e5m2):
    C = t.shape[-1]
    R = 1
    for d in t.shape[:-1]:
        R *= d
    u8 = torch.uint8
    return (TensorProxy(like=t, shape=(R, C), dtype=u8, requires_grad=False),
            TensorProxy(like=t, shape=(C, R), dtype=u8, requires_grad=False),
            TensorProxy(like=t, shape=(), dtype=torch.float32, requires_grad=False))


def _fp8_quant_impl(t, e5m2):
    from ..ops.fp8 import quantize

    return quantize(t, e5m2)


def _fp8_gemm_meta(qa, qb, sa, sb, fmt_a, fmt_b, bias, out_shape, residual=None):
    return TensorProxy(like=qa, shape=tuple(out_shape), dtype=torch.bfloat16)


def _fp8_gemm_impl(qa, qb, sa, sb, fmt_a, fmt_b, bias, out_shape, residual=None):
    from ..ops.fp8 import gemm

    return gemm(qa, qb, sa, sb, fmt_a, fmt_b, bias, out_shape, residual)


# quantize = amax + cast(+transpose) (pure: CSE shares one quantisation of x between the sibling
# fc_1 / fc_2 linears); gemm = the block-scaled-MFMA NT kernel
hip_fp8_quantize = ex.register_operator("hip_fp8_quantize", meta=_fp8_quant_meta, fn=_fp8_quant_impl)
hip_fp8_gemm = ex.register_operator("hip_fp8_gemm", meta=_fp8_gemm_meta, fn=_fp8_gemm_impl)


def _fp8_quant_delayed_meta(t, e5m2, key, slot):
    return _fp8_quant_meta(t, e5m2)


def _fp8_quant_delayed_impl(t, e5m2, key, slot):
    from ..ops.fp8 import quantize_delayed

    return quantize_delayed(t, e5m2, key, slot)


def _fp8_update_impl(key):
    from ..ops.fp8 import delayed_update

    delayed_update(key)


# delayed scaling: quantize against the slot's amax history (its own amax recorded while casting);
# the history advances once per forward (first op of the program), after an amax all-reduce
hip_fp8_quantize_delayed = ex.register_operator("hip_fp8_quantize_delayed", meta=_fp8_quant_delayed_meta,
                                                fn=_fp8_quant_delayed_impl)
hip_fp8_delayed_update = ex.register_operator("hip_fp8_delayed_update", meta=lambda key: None, fn=_fp8_update_impl,
                                              tags=(OpTags.DONT_DCE,))
hip_fp8_delayed_update.not_capturable = True  # may all-reduce over the data-parallel group


def _fp8_cast_meta(t, e5m2, key=None, slot=None):
    C = t.shape[-1]
    R = 1
    for d in t.shape[:-1]:
        R *= d
    return (TensorProxy(like=t, shape=(R, C), dtype=torch.uint8, requires_grad=False),
            TensorProxy(like=t, shape=(), dtype=torch.float32, requires_grad=False))


def _fp8_cast_impl(t, e5m2):
    from ..ops.fp8 import quantize_rows

    return quantize_rows(t, e5m2)


def _fp8_cast_delayed_impl(t, e5m2, key, slot):
    from ..ops.fp8 import quantize_delayed_rows

    return quantize_delayed_rows(t, e5m2, key, slot)


def _fp8_gemm_layout_meta(qa, qb, sa, sb, fmt_a, at, out_shape, residual=None):
    return TensorProxy(like=qa, shape=tuple(out_shape), dtype=torch.bfloat16)


def _fp8_gemm_layout_impl(qa, qb, sa, sb, fmt_a, at, out_shape, residual=None):
    from ..ops.fp8 import gemm_fp8_layout

    return gemm_fp8_layout(qa, qb, sa, sb, fmt_a, at, residual).reshape(out_shape)


# row-major fp8 copies only: the backward GEMMs read the saved e4m3 activation / weight and the e5m2
# gradient in place (MN-major operands through ds_read_b64_tr_b8, csrc/gemm4_fp8.hip), so no
# transposed copy is ever written (LTA_FP8_TRANSPOSED=1: the cast_transpose path, A/B)
hip_fp8_cast = ex.register_operator("hip_fp8_cast", meta=_fp8_cast_meta, fn=_fp8_cast_impl)
hip_fp8_cast_delayed = ex.register_operator("hip_fp8_cast_delayed", meta=_fp8_cast_meta, fn=_fp8_cast_delayed_impl)
hip_fp8_gemm_layout = ex.register_operator("hip_fp8_gemm_layout", meta=_fp8_gemm_layout_meta,
                                           fn=_fp8_gemm_layout_impl)


def _rms_fp8_meta(x, w, eps, key, slot):
    q, sc = _fp8_cast_meta(x, False)
    return q, sc, TensorProxy(like=x, shape=(q.shape[0],), dtype=torch.float32, requires_grad=False)


def _rms_fp8_impl(x, w, eps, key, slot):
    from ..ops.fp8 import rms_norm_fwd_fp8_delayed

    return rms_norm_fwd_fp8_delayed(x, w, eps, key, slot)


def _swiglu_fp8_impl(a, b, key, slot):
    from ..ops.fp8 import swiglu_fwd_fp8_delayed

    return swiglu_fwd_fp8_delayed(a, b, key, slot)


def _swiglu_bwd_fp8_meta(g, a, b, key, slot_a, slot_b):
    qa, sa = _fp8_cast_meta(a, True)
    qb, sb = _fp8_cast_meta(b, True)
    return qa, sa, qb, sb


def _swiglu_bwd_fp8_impl(g, a, b, key, slot_a, slot_b):
    from ..ops.fp8 import swiglu_bwd_fp8_delayed

    return swiglu_bwd_fp8_delayed(g, a, b, key, slot_a, slot_b)


hip_swiglu_bwd_fp8 = ex.register_operator("hip_swiglu_bwd_fp8", meta=_swiglu_bwd_fp8_meta, fn=_swiglu_bwd_fp8_impl)

# producer-fused input casts of the fp8 linears (delayed scaling; _fuse_fp8_cast_producers)
hip_rms_norm_fwd_fp8 = ex.register_operator("hip_rms_norm_fwd_fp8", meta=_rms_fp8_meta, fn=_rms_fp8_impl)
hip_swiglu_fp8 = ex.register_operator("hip_swiglu_fp8", meta=lambda a, b, key, slot: _fp8_cast_meta(a, False),
                                      fn=_swiglu_fp8_impl)


def _fuse_fp8_cast_producers(trace):
    """``y, rstd = hip_rms_norm_fwd(x, w, eps); q, s = hip_fp8_cast_delayed(y, False, key, slot)`` ->
    ``q, s, rstd = hip_rms_norm_fwd_fp8(x, w, eps, key, slot)``, and ``y = hip_swiglu(a, b)`` + its
    cast -> ``q, s = hip_swiglu_fp8(a, b, key, slot)`` when the cast is y's only use: the activation
    leaves the producing kernel as e4m3 (no bf16 round trip, no separate cast launch).  Parity: the
    reference's TransformerEngine layers quantise inside their fused norm / activation kernels
    (thunder/executors/transformer_engineex_impl.py)."""
    import os

    from ..core.trace import from_trace, TraceProvenance

    if os.environ.get("LTA_FP8_FUSE_PRODUCERS", "1") == "0":  # A/B hook
        return trace
    bsyms = trace.bound_symbols
    uses: dict[str, int] = {}
    for b in bsyms:
        for a in b.flat_proxy_args:
            uses[a.name] = uses.get(a.name, 0) + 1
    producer = {}
    for i, b in enumerate(bsyms):
        for o in b.flat_proxy_outs:
            producer[o.name] = i
    drop: set[int] = set()
    replace: dict[int, object] = {}
    for i, b in enumerate(bsyms):
        if b.sym is not hip_fp8_cast_delayed or len(b.args) != 4 or b.args[1]:
            continue
        y, _, key, slot = b.args
        j = producer.get(y.name)
        if j is None or j in replace or j in drop or uses.get(y.name, 0) != 1:
            continue
        pb = bsyms[j]
        if pb.sym is hip_rms_norm_fwd and len(pb.args) >= 3 and pb.args[1] is not None and pb.output[0].name == y.name:
            nb = hip_rms_norm_fwd_fp8.bind(pb.args[0], pb.args[1], pb.args[2], key, slot,
                                           output=(b.output[0], b.output[1], pb.output[1]))
        elif pb.sym is hip_swiglu and len(pb.args) == 2:
            nb = hip_swiglu_fp8.bind(pb.args[0], pb.args[1], key, slot, output=b.output)
        else:
            continue
        replace[j] = ex.bind_call_ctx(nb)
        drop.add(i)
    # backward: da, db = hip_swiglu_bwd(g, a, b) whose only uses are their e5m2 casts
    casts: dict[str, int] = {}
    for i, b in enumerate(bsyms):
        if b.sym is hip_fp8_cast_delayed and len(b.args) == 4 and b.args[1] and i not in drop:
            casts[b.args[0].name] = i
    for j, pb in enumerate(bsyms):
        if pb.sym is not hip_swiglu_bwd or j in replace or len(pb.args) != 3:
            continue
        da, db = pb.output
        ia, ib = casts.get(da.name), casts.get(db.name)
        if ia is None or ib is None or uses.get(da.name, 0) != 1 or uses.get(db.name, 0) != 1:
            continue
        ca, cb = bsyms[ia], bsyms[ib]
        if ca.args[2] != cb.args[2]:
            continue
        nb = hip_swiglu_bwd_fp8.bind(*pb.args, ca.args[2], ca.args[3], cb.args[3],
                                     output=(ca.output[0], ca.output[1], cb.output[0], cb.output[1]))
        replace[j] = ex.bind_call_ctx(nb)
        drop.update((ia, ib))
    if not replace:
        return trace
    new = from_trace(trace)
    new.bound_symbols = [replace.get(i, b) for i, b in enumerate(bsyms) if i not in drop]
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance(f"hipex: {len(replace)} fp8 input cast(s) fused into their producers"))
    return new


def _fp8_transposed() -> bool:
    import os

    return os.environ.get("LTA_FP8_TRANSPOSED", "0") == "1"


def _mx_quant_meta(t, e5m2):
    C = t.shape[-1]
    R = 1
    for d in t.shape[:-1]:
        R *= d
    u8 = torch.uint8
    mk = lambda shape: TensorProxy(like=t, shape=shape, dtype=u8, requires_grad=False)  # noqa: E731
    return mk((R, C)), mk((R, C // 32)), mk((C, R)), mk((C, R // 32))


def _mx_quant_impl(t, e5m2):
    from ..ops.fp8 import mx_quantize

    return mx_quantize(t, e5m2)


def _mx_gemm_meta(qa, sa, qb, sb, fmt_a, fmt_b, bias, out_shape):
    return TensorProxy(like=qa, shape=tuple(out_shape), dtype=torch.bfloat16)


def _mx_gemm_impl(qa, sa, qb, sb, fmt_a, fmt_b, bias, out_shape):
    from ..ops.fp8 import gemm_nt_mx

    return gemm_nt_mx(qa, sa, qb, sb, fmt_a, fmt_b, bias).reshape(out_shape)


# MXFP8: one pass emits both orientations with their 32-block E8M0 scales; the GEMM feeds the scales
# to the block-scaled MFMA per lane
hip_mx_quantize = ex.register_operator("hip_mx_quantize", meta=_mx_quant_meta, fn=_mx_quant_impl)
hip_mx_gemm = ex.register_operator("hip_mx_gemm", meta=_mx_gemm_meta, fn=_mx_gemm_impl)


def _mx_vjp(x, w, bias=None):
    from .. import torch as ltorch

    qx, sx, qxT, sxT = hip_mx_quantize(x, False)
    qw, sw, qwT, swT = hip_mx_quantize(w, False)
    y = hip_mx_gemm(qx, sx, qw, sw, 0, 0, bias, tuple(x.shape[:-1]) + (w.shape[0],))

    def bwd(g):
        qg, sg, qgT, sgT = hip_mx_quantize(g, True)
        dx = hip_mx_gemm(qg, sg, qwT, swT, 1, 0, None, tuple(x.shape))
        dw = hip_mx_gemm(qgT, sgT, qxT, sxT, 1, 0, None, tuple(w.shape))
        if bias is None:
            return dx, dw
        return dx, dw, ltorch.sum(g, tuple(range(g.ndim - 1)))

    return y, bwd


def _mx4_quant_meta(t):
    C = t.shape[-1]
    R = 1
    for d in t.shape[:-1]:
        R *= d
    u8 = torch.uint8
    return (TensorProxy(like=t, shape=(R, C // 2), dtype=u8, requires_grad=False),
            TensorProxy(like=t, shape=(R, C // 32), dtype=u8, requires_grad=False))


def _mx4_quant_impl(t):
    from ..ops.mxfp4 import quantize

    return quantize(t)


def _mx4_gemm_impl(qa, sa, qb, sb, bias, out_shape):
    from ..ops.mxfp4 import gemm_nt

    return gemm_nt(qa, sa, qb, sb, bias).reshape(out_shape)


# MXFP4 recipe: packed e2m1 + E8M0/32 operands of the forward GEMM (csrc/fp8.hip mx4 cast,
# csrc/gemm.hip gemm_nt_mxfp4_kernel)
hip_mx4_quantize = ex.register_operator("hip_mx4_quantize", meta=_mx4_quant_meta, fn=_mx4_quant_impl)
hip_mx4_gemm = ex.register_operator(
    "hip_mx4_gemm", meta=lambda qa, sa, qb, sb, bias, out_shape: TensorProxy(like=qa, shape=tuple(out_shape),
                                                                            dtype=torch.bfloat16),
    fn=_mx4_gemm_impl)


def _mx4_fwd(x, w, bias):
    qx4, sx4 = hip_mx4_quantize(x)
    qw4, sw4 = hip_mx4_quantize(w)
    return hip_mx4_gemm(qx4, sx4, qw4, sw4, bias, tuple(x.shape[:-1]) + (w.shape[0],))


def _mx4_vjp(x, w, bias=None):
    """MXFP4 forward, MXFP8 backward: the backward reads e4m3 MX copies of x^T and w^T."""
    from .. import torch as ltorch

    y = _mx4_fwd(x, w, bias)
    _, _, qxT, sxT = hip_mx_quantize(x, False)
    _, _, qwT, swT = hip_mx_quantize(w, False)

    def bwd(g):
        qg, sg, qgT, sgT = hip_mx_quantize(g, True)
        dx = hip_mx_gemm(qg, sg, qwT, swT, 1, 0, None, tuple(x.shape))
        dw = hip_mx_gemm(qgT, sgT, qxT, sxT, 1, 0, None, tuple(w.shape))
        if bias is None:
            return dx, dw
        return dx, dw, ltorch.sum(g, tuple(range(g.ndim - 1)))

    return y, bwd


def _quant(t, e5m2, key, slot):
    if key is None:
        return hip_fp8_quantize(t, e5m2)
    return hip_fp8_quantize_delayed(t, e5m2, key, slot)


def _cast(t, e5m2, key, slot):
    if key is None:
        return hip_fp8_cast(t, e5m2)
    return hip_fp8_cast_delayed(t, e5m2, key, slot)


def _fp8_vjp(x, w, bias=None, key=None, slots=None):
    from .. import torch as ltorch

    if key == "mxfp8":
        return _mx_vjp(x, w, bias)
    if key == "mxfp4":
        return _mx4_vjp(x, w, bias)
    sl = slots or (None, None, None)
    out_shape = tuple(x.shape[:-1]) + (w.shape[0],)
    if not _fp8_transposed():
        qx, sx = _cast(x, False, key, sl[0])
        qw, sw = _cast(w, False, key, sl[1])
        y = hip_fp8_gemm(qx, qw, sx, sw, 0, 0, bias, out_shape)

        def bwd_rows(g):
            qg, sg = _cast(g, True, key, sl[2])
            dx = hip_fp8_gemm_layout(qg, qw, sg, sw, 1, False, tuple(x.shape))  # dY [M, out] . W [out][in]
            dw = hip_fp8_gemm_layout(qg, qx, sg, sx, 1, True, tuple(w.shape))   # dY^T . X, both [tokens][.]
            if bias is None:
                return dx, dw
            return dx, dw, ltorch.sum(g, tuple(range(g.ndim - 1)))

        return y, bwd_rows
    qx, qxT, sx = _quant(x, False, key, sl[0])
    qw, qwT, sw = _quant(w, False, key, sl[1])
    y = hip_fp8_gemm(qx, qw, sx, sw, 0, 0, bias, out_shape)

    def bwd(g):
        qg, qgT, sg = _quant(g, True, key, sl[2])
        dx = hip_fp8_gemm(qg, qwT, sg, sw, 1, 0, None, tuple(x.shape))
        dw = hip_fp8_gemm(qgT, qxT, sg, sx, 1, 0, None, tuple(w.shape))
        if bias is None:
            return dx, dw
        db = ltorch.sum(g, tuple(range(g.ndim - 1)))
        return dx, dw, db

    return y, bwd


def _fp8_exec(x, w, bias=None, key=None, slots=None):
    if key == "mxfp8":
        qx, sx, _, _ = hip_mx_quantize(x, False)
        qw, sw, _, _ = hip_mx_quantize(w, False)
        return hip_mx_gemm(qx, sx, qw, sw, 0, 0, bias, tuple(x.shape[:-1]) + (w.shape[0],))
    if key == "mxfp4":
        return _mx4_fwd(x, w, bias)
    sl = slots or (None, None, None)
    qx, sx = _cast(x, False, key, sl[0])
    qw, sw = _cast(w, False, key, sl[1])
    return hip_fp8_gemm(qx, qw, sx, sw, 0, 0, bias, tuple(x.shape[:-1]) + (w.shape[0],))


def _register_fp8():
    from ..transforms.fp8 import fp8_linear, fp8_delayed_update, eligible
    from ..core.transforms import register_vjp

    ex.register_implementation(fp8_linear, checker=eligible, execution_transform=_fp8_exec)
    register_vjp(fp8_linear)(_fp8_vjp)
    ex.register_implementation(fp8_delayed_update, hip_fp8_delayed_update)


_register_fp8()


def _fuse_linear_epilogues(trace):
    """``y = hip_linear(x, w, b); z = y + r`` (y used nowhere else) -> ``z = hip_linear(x, w, b, r)``:
    the residual add runs in the GEMM's epilogue (one HBM round trip of y saved)."""
    from ..core.trace import from_trace, TraceProvenance

    bsyms = trace.bound_symbols
    uses: dict[str, int] = {}
    for b in bsyms:
        for a in b.flat_proxy_args:
            uses[a.name] = uses.get(a.name, 0) + 1
    producer = {}
    for i, b in enumerate(bsyms):
        for o in b.flat_proxy_outs:
            producer[o.name] = i
    drop: set[int] = set()
    replace: dict[int, object] = {}
    for i, b in enumerate(bsyms):
        if b.sym.name not in ("torch_add", "add") or b.kwargs.get("alpha") not in (None, 1):
            continue
        if len(b.args) < 2 or not all(isinstance(a, TensorProxy) for a in b.args[:2]):
            continue
        for pos in (0, 1):
            y, r = b.args[pos], b.args[1 - pos]
            j = producer.get(y.name)
            if (j is None or j in drop or bsyms[j].sym not in (hip_linear, hip_matmul, hip_fp8_gemm, hip_fp8_gemm_layout)
                    or uses.get(y.name, 0) != 1):
                continue
            lb = bsyms[j]
            if tuple(r.shape) != tuple(y.shape) or r.dtype != y.dtype or tuple(b.output.shape) != tuple(y.shape):
                continue
            if lb.sym is hip_fp8_gemm_layout:
                if lb.args[5] or (len(lb.args) > 7 and lb.args[7] is not None) or "residual" in lb.kwargs:
                    continue  # the residual epilogue exists for the dgrad layout (A [M][K]) only
                if producer.get(r.name, -1) > i or j in replace:
                    continue
                replace[i] = ex.bind_call_ctx(hip_fp8_gemm_layout.bind(*lb.args[:7], r, output=b.output))
                drop.add(j)
                break
            if lb.sym is hip_fp8_gemm:
                if len(lb.args) > 8 and lb.args[8] is not None or "residual" in lb.kwargs:
                    continue
                if producer.get(r.name, -1) > i or j in replace:
                    continue
                # computed where the add was (every input of the GEMM exists there)
                nb = ex.bind_call_ctx(hip_fp8_gemm.bind(*lb.args[:8], r, output=b.output))
                replace[i] = nb
                drop.add(j)
                break
            if producer.get(r.name, -1) > j:
                continue  # the residual is produced after the GEMM: the fused op could not see it
            if lb.sym is hip_matmul:
                if len(lb.args) > 2 and lb.args[2] is not None:
                    continue
                nb = hip_matmul.bind(lb.args[0], lb.args[1], r, output=b.output)
                nb = ex.bind_call_ctx(nb)
                replace[j] = nb  # computed where the GEMM was (the add's consumers come later)
                drop.add(i)
                break
            if len(lb.args) > 3 and lb.args[3] is not None:
                continue
            bias = lb.args[2] if len(lb.args) > 2 else lb.kwargs.get("bias")
            nb = hip_linear.bind(lb.args[0], lb.args[1], bias, r, output=b.output)
            nb = ex.bind_call_ctx(nb)
            replace[i] = nb
            drop.add(j)
            break
    if not replace:
        return trace
    new = from_trace(trace)
    new.bound_symbols = [replace.get(i, b) for i, b in enumerate(bsyms) if i not in drop]
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance(f"hipex: {len(replace)} residual add(s) fused into GEMM epilogues"))
    return new


# =========================================================================================
# K2b decode GEMV with fused prologues (rmsnorm) / gated epilogues (SwiGLU up-projection pair)
# =========================================================================================
def _decode_linear_meta(x, w, bias=None, residual=None, act=None, gate_weight=None, norm=False, norm_weight=None,
                        eps=1e-5):
    return TensorProxy(like=x, shape=tuple(x.shape[:-1]) + (w.shape[0],))


def _decode_linear_impl(x, w, bias=None, residual=None, act=None, gate_weight=None, norm=False, norm_weight=None,
                        eps=1e-5):
    from ..ops.gemm import gemv_nt, gemv_supported, _torch_linear

    K, N = x.shape[-1], w.shape[0]
    x2 = x.reshape(-1, K)
    r2 = None if residual is None else residual.reshape(-1, N)
    ok = gemv_supported(x2, w, bias, r2) and (gate_weight is None or gate_weight.stride() == w.stride())
    if ok and norm_weight is not None:
        ok = norm_weight.is_contiguous() and norm_weight.dtype == x.dtype
    if ok:
        y = gemv_nt(x2, w, bias=bias, residual=r2, act=act, gate_weight=gate_weight, norm=norm,
                    norm_weight=norm_weight, eps=eps)
        return y.reshape(*x.shape[:-1], N)
    if norm:  # unaligned operands: the same math on the library path
        from ..ops.rmsnorm import rms_norm_fwd

        x2, _ = rms_norm_fwd(x2, norm_weight, eps)
    if gate_weight is not None:
        y = _torch_linear(x2, w, None, None, act) * torch.nn.functional.linear(x2, gate_weight)
    else:
        y = _torch_linear(x2, w, bias, r2, act)
    return y.reshape(*x.shape[:-1], N)


hip_decode_linear = ex.register_operator("hip_decode_linear", meta=_decode_linear_meta, fn=_decode_linear_impl)
_GEMV_MAX_ROWS = 8


def _rows(t) -> int:
    r = 1
    for d in t.shape[:-1]:
        r *= d
    return r


def _linear_parts(b):
    names = ("x", "w", "bias", "residual", "act")
    d = dict(zip(names, b.args))
    d.update({k: v for k, v in b.kwargs.items() if k in names})
    return d


def _fuse_decode_gemv(trace):
    """Decode-shaped (<= 8 rows) chains around the weight-streaming GEMV, one launch each:

    * ``a = hip_linear(x, w1); b = hip_linear(x, w2); y = hip_swiglu(a, b)`` ->
      ``y = hip_decode_linear(x, w1, act="silu", gate_weight=w2)`` (LLaMA MLP up-projections + gate);
    * ``y, rstd = hip_rms_norm_fwd(x, g, eps)`` whose ``y`` only feeds decode linears (and ``rstd``
      nothing) -> the norm runs in those GEMVs' prologue (``norm=True``).
    Every launch removed is ~5 us of a ~1 ms decode step on MI355X (kernel floor + boundary)."""
    from ..core.trace import from_trace, TraceProvenance

    bsyms = list(trace.bound_symbols)

    def count_uses(skip):
        u: dict[str, int] = {}
        for k, b in enumerate(bsyms):
            if k not in skip:
                for a in b.flat_proxy_args:
                    u[a.name] = u.get(a.name, 0) + 1
        for o in tree_flatten(trace.output)[0] if trace.output is not None else ():
            if isinstance(o, TensorProxy):
                u[o.name] = u.get(o.name, 0) + 1
        return u

    uses = count_uses(())
    producer = {}
    for i, b in enumerate(bsyms):
        for o in b.flat_proxy_outs:
            producer[o.name] = i
    drop: set[int] = set()
    n_gated = n_norm = 0

    def bind(i, *args, output, **kwargs):
        bsyms[i] = ex.bind_call_ctx(hip_decode_linear.bind(*args, output=output, **kwargs))

    # SwiGLU up-projection pairs
    for i, b in enumerate(bsyms):
        if b.sym is not hip_swiglu or len(b.args) != 2:
            continue
        a, g = b.args
        ja, jg = producer.get(a.name), producer.get(g.name)
        if ja is None or jg is None or ja in drop or jg in drop or ja == jg:
            continue
        la, lg = bsyms[ja], bsyms[jg]
        if la.sym is not hip_linear or lg.sym is not hip_linear or uses.get(a.name) != 1 or uses.get(g.name) != 1:
            continue
        pa, pg = _linear_parts(la), _linear_parts(lg)
        if pa["x"].name != pg["x"].name or any(p.get(k) is not None for p in (pa, pg) for k in ("bias", "residual", "act")):
            continue
        if _rows(pa["x"]) > _GEMV_MAX_ROWS or tuple(pa["w"].shape) != tuple(pg["w"].shape):
            continue
        bind(i, pa["x"], pa["w"], None, None, "silu", pg["w"], False, None, 1e-5, output=b.output)
        drop.update((ja, jg))
        n_gated += 1

    # the same pair written out (HF LlamaMLP): y = mul(silu(a), b)
    for i, b in enumerate(bsyms):
        if i in drop or b.sym.name != "mul" or len(b.args) != 2 or not all(isinstance(a, TensorProxy) for a in b.args):
            continue
        for s_arg, g_arg in (b.args, b.args[::-1]):
            js = producer.get(s_arg.name)
            if js is None or js in drop or bsyms[js].sym.name != "silu" or uses.get(s_arg.name) != 1:
                continue
            sb = bsyms[js]
            a = sb.args[0] if sb.args else None
            if len(sb.args) > 1 and sb.args[1] not in (False, None):
                continue
            ja, jg = producer.get(getattr(a, "name", None)), producer.get(g_arg.name)
            if ja is None or jg is None or ja in drop or jg in drop or ja == jg:
                continue
            la, lg = bsyms[ja], bsyms[jg]
            if la.sym is not hip_linear or lg.sym is not hip_linear or uses.get(a.name) != 1 or uses.get(g_arg.name) != 1:
                continue
            pa, pg = _linear_parts(la), _linear_parts(lg)
            if pa["x"].name != pg["x"].name or any(p.get(k) is not None for p in (pa, pg) for k in ("bias", "residual", "act")):
                continue
            if _rows(pa["x"]) > _GEMV_MAX_ROWS or tuple(pa["w"].shape) != tuple(pg["w"].shape) or b.output.dtype != a.dtype:
                continue
            bind(i, pa["x"], pa["w"], None, None, "silu", pg["w"], False, None, 1e-5, output=b.output)
            drop.update((ja, jg, js))
            n_gated += 1
            break

    # RMSNorm prologues
    uses = count_uses(drop)
    for i, b in enumerate(bsyms):
        if i in drop or b.sym is not hip_rms_norm_fwd:
            continue
        y, rstd = b.output
        x, g, eps = b.args[0], b.args[1], b.args[2]
        if uses.get(rstd.name, 0) or _rows(x) > _GEMV_MAX_ROWS or not isinstance(eps, (int, float)):
            continue
        consumers = [j for j, c in enumerate(bsyms) if j not in drop and any(a.name == y.name for a in c.flat_proxy_args)]
        ok = bool(consumers)
        for j in consumers:
            c = bsyms[j]
            if c.sym is hip_linear:
                p = _linear_parts(c)
                ok = ok and p["x"] is not None and p["x"].name == y.name and p["w"].name != y.name
            elif c.sym is hip_decode_linear:
                ok = ok and c.args[0].name == y.name and not c.args[6] and all(
                    getattr(a, "name", None) != y.name for a in c.args[1:])
            else:
                ok = False
        if not ok or sum(1 for j in consumers) != uses.get(y.name, 0):
            continue
        for j in consumers:
            c = bsyms[j]
            if c.sym is hip_linear:
                p = _linear_parts(c)
                bind(j, x, p["w"], p.get("bias"), p.get("residual"), p.get("act"), None, True, g, float(eps),
                     output=c.output)
            else:
                a = list(c.args)
                bind(j, x, a[1], a[2], a[3], a[4], a[5], True, g, float(eps), output=c.output)
        drop.add(i)
        n_norm += 1

    if not drop:
        return trace
    new = from_trace(trace)
    new.bound_symbols = [b for i, b in enumerate(bsyms) if i not in drop]
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance(f"hipex: decode GEMV fusion ({n_gated} gated pair(s), {n_norm} norm prologue(s))"))
    return new


def _decode_group_meta(x, weights, norm=False, norm_weight=None, eps=1e-5, packed=False):
    if packed:
        return TensorProxy(like=x, shape=tuple(x.shape[:-1]) + (sum(w.shape[0] for w in weights),))
    return tuple(TensorProxy(like=x, shape=tuple(x.shape[:-1]) + (w.shape[0],)) for w in weights)


def _decode_group_impl(x, weights, norm=False, norm_weight=None, eps=1e-5, packed=False):
    from ..ops.gemm import gemv_group, gemv_supported

    K = x.shape[-1]
    x2 = x.reshape(-1, K)
    ok = all(gemv_supported(x2, w) for w in weights)
    if ok and norm_weight is not None:
        ok = norm_weight.is_contiguous() and norm_weight.dtype == x.dtype
    if ok:
        outs = gemv_group(x2, list(weights), norm=norm, norm_weight=norm_weight, eps=eps, packed=packed)
    else:
        if norm:
            from ..ops.rmsnorm import rms_norm_fwd

            x2, _ = rms_norm_fwd(x2, norm_weight, eps)
        outs = [torch.nn.functional.linear(x2, w) for w in weights]
        if packed:
            outs = torch.cat(outs, -1)
    if packed:
        return outs.reshape(*x.shape[:-1], outs.shape[-1])
    return tuple(o.reshape(*x.shape[:-1], o.shape[-1]) for o in outs)


hip_decode_linear_group = ex.register_operator("hip_decode_linear_group", meta=_decode_group_meta,
                                               fn=_decode_group_impl)


def _group_decode_projections(trace):
    """Sibling decode projections of one input (HF attention's q / k / v: ``hip_decode_linear`` or
    ``hip_linear`` with <= 8 rows, same x and norm prologue, no bias / residual / activation / gate)
    -> one ``hip_decode_linear_group`` launch streaming all their weights (up to 3 per launch)."""
    from ..core.trace import from_trace, TraceProvenance

    bsyms = list(trace.bound_symbols)
    groups: dict = {}
    for i, b in enumerate(bsyms):
        if b.sym is hip_decode_linear:
            a = list(b.args) + [None] * (9 - len(b.args))
            x, w, bias, res, act, gate, norm, g, eps = a[:9]
            if any(v is not None for v in (bias, res, act, gate)):
                continue
        elif b.sym is hip_linear:
            p = _linear_parts(b)
            x, w = p["x"], p["w"]
            if any(p.get(k) is not None for k in ("bias", "residual", "act")):
                continue
            norm, g, eps = False, None, 1e-5
        else:
            continue
        if not isinstance(x, TensorProxy) or _rows(x) > _GEMV_MAX_ROWS or w.ndim != 2:
            continue
        key = (x.name, bool(norm), getattr(g, "name", None), float(eps) if isinstance(eps, (int, float)) else eps)
        groups.setdefault(key, []).append(i)
    replace: dict[int, object] = {}
    drop: set[int] = set()
    n = 0
    # cat(p0, p1, p2, dim=-1) of sibling projections used only by the cat -> one packed launch
    uses: dict[str, int] = {}
    for b in bsyms:
        for a in b.flat_proxy_args:
            uses[a.name] = uses.get(a.name, 0) + 1
    producer = {o.name: i for i, b in enumerate(bsyms) for o in b.flat_proxy_outs}
    member = {i: key for key, idxs in groups.items() for i in idxs}
    for ci, cb in enumerate(bsyms):
        if cb.sym.name not in ("cat", "torch_cat", "cat_prim") or not cb.args or not isinstance(cb.args[0], (list, tuple)):
            continue
        parts = cb.args[0]
        dim = cb.args[1] if len(cb.args) > 1 else cb.kwargs.get("dim", 0)
        if not 2 <= len(parts) <= 3 or not all(isinstance(p, TensorProxy) for p in parts) or dim not in (-1, parts[0].ndim - 1):
            continue
        js = [producer.get(p.name) for p in parts]
        if any(j is None or j in drop or j in replace or uses.get(p.name) != 1 for j, p in zip(js, parts)):
            continue
        keys = {member.get(j) for j in js}
        if len(keys) != 1 or None in keys:
            continue
        (xname, norm, gname, eps), = keys
        first = bsyms[js[0]]
        g = (first.args[7] if len(first.args) > 7 else first.kwargs.get("norm_weight")) if norm else None
        ws = tuple(bsyms[j].args[1] for j in js)
        replace[ci] = ex.bind_call_ctx(hip_decode_linear_group.bind(first.args[0], ws, norm, g, eps, True,
                                                                    output=cb.output))
        drop.update(js)
        for key_idxs in groups.values():
            for j in js:
                if j in key_idxs:
                    key_idxs.remove(j)
        n += 1
    for (xname, norm, gname, eps), idxs in groups.items():
        for c0 in range(0, len(idxs) - 1, 3):
            chunk = idxs[c0:c0 + 3]
            if len(chunk) < 2:
                continue
            first = bsyms[chunk[0]]
            x = first.args[0]
            g = None
            if norm:
                g = first.args[7] if len(first.args) > 7 else first.kwargs.get("norm_weight")
            ws = tuple(bsyms[j].args[1] for j in chunk)
            outs = tuple(bsyms[j].output for j in chunk)
            replace[chunk[0]] = ex.bind_call_ctx(hip_decode_linear_group.bind(x, ws, norm, g, eps, output=outs))
            drop.update(chunk[1:])
            n += 1
    if not n:
        return trace
    new = from_trace(trace)
    new.bound_symbols = [replace.get(i, b) for i, b in enumerate(bsyms) if i not in drop]
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance(f"hipex: {n} grouped decode projection launch(es)"))
    return new


def _qkv_rope_cache_meta(qkv, cos, sin, n_head, n_query_groups, head_size, rope_n, kc, vc, pos):
    B, T, _ = qkv.shape
    return TensorProxy(like=qkv, shape=(B, n_head, T, head_size)), TensorProxy(like=kc), TensorProxy(like=vc)


def _qkv_rope_cache_impl(qkv, cos, sin, n_head, n_query_groups, head_size, rope_n, kc, vc, pos):
    from ..ops.fused import qkv_rope_cache_fwd, qkv_rope_cache_supported, qkv_rope_fwd

    if qkv_rope_cache_supported(qkv, kc, vc, pos, n_query_groups, head_size):
        return qkv_rope_cache_fwd(qkv, cos, sin, n_head, n_query_groups, head_size, rope_n, kc, vc, pos)
    q, k, v = qkv_rope_fwd(qkv, cos, sin, n_head, n_query_groups, head_size, rope_n)
    return q, kc.index_copy_(2, pos, k), vc.index_copy_(2, pos, v)


hip_qkv_rope_cache = ex.register_operator("hip_qkv_rope_cache", meta=_qkv_rope_cache_meta, fn=_qkv_rope_cache_impl,
                                          tags=(OpTags.DONT_DCE, OpTags.IN_PLACE))
hip_qkv_rope_cache.written_args = (7, 8)  # kc, vc; qkv/cos/sin/pos are only read


def _fuse_kv_cache_writes(trace):
    """``q, k, v = hip_qkv_rope(...); kc = index_copy_inplace(cache_k, 2, pos, k);
    vc = index_copy_inplace(cache_v, 2, pos, v)`` (k, v used nowhere else) ->
    ``q, kc, vc = hip_qkv_rope_cache(..., cache_k, cache_v, pos)``: the rotated keys and the values
    are stored straight into the static caches by the RoPE kernel (two launches fewer per layer)."""
    from ..core.trace import from_trace, TraceProvenance

    bsyms = list(trace.bound_symbols)
    uses: dict[str, list[int]] = {}
    for i, b in enumerate(bsyms):
        for a in b.flat_proxy_args:
            uses.setdefault(a.name, []).append(i)
    out_names = {o.name for o in tree_flatten(trace.output)[0] if isinstance(o, TensorProxy)} \
        if trace.output is not None else set()
    replace, drop = {}, set()
    for i, b in enumerate(bsyms):
        if b.sym is not hip_qkv_rope:
            continue
        q, k, v = b.output
        uk, uv = uses.get(k.name, []), uses.get(v.name, [])
        if len(uk) != 1 or len(uv) != 1 or k.name in out_names or v.name in out_names:
            continue
        ck, cv = bsyms[uk[0]], bsyms[uv[0]]
        if ck.sym.name != "index_copy_inplace" or cv.sym.name != "index_copy_inplace":
            continue
        (bk, dk, pk, sk), (bv, dv, pv, sv) = ck.args[:4], cv.args[:4]
        if dk != 2 or dv != 2 or sk is not k or sv is not v or getattr(pk, "name", None) != getattr(pv, "name", 1):
            continue
        if pk.dtype != torch.int64 or bk.dtype != k.dtype or bv.dtype != v.dtype:
            continue
        nb = ex.bind_call_ctx(hip_qkv_rope_cache.bind(*b.args, bk, bv, pk, output=(q, ck.output, cv.output)))
        # the fused op needs the caches and positions: emit it where the RoPE was when they exist
        # there (LitGPT), else at the later cache write (HF computes the positions after the RoPE),
        # provided nothing reads q in between
        producer_pos = {o.name: j for j, bb in enumerate(bsyms) for o in bb.flat_proxy_outs}
        ready = max([producer_pos.get(x.name, -1) for x in (bk, bv, pk)] + [-1])
        if ready < i:
            at = i
        else:
            at = max(uk[0], uv[0])
            if any(i < j < at for j in uses.get(q.name, [])) or ready >= at:
                continue
            # moving the first cache write later: nothing in between may read its result or the
            # cache it writes
            lo = min(uk[0], uv[0])
            watch = {ck.output.name, cv.output.name, bk.name, bv.name}
            if any(lo < j < at for w in watch for j in uses.get(w, [])):
                continue
        replace[at] = nb
        drop.update({i, uk[0], uv[0]} - {at})
    if not replace:
        return trace
    new = from_trace(trace)
    new.bound_symbols = [replace.get(i, b) for i, b in enumerate(bsyms) if i not in drop]
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance(f"hipex: {len(replace)} KV-cache write pair(s) fused into RoPE"))
    return new


def _fuse_rms_bwd_residual(trace):
    """``(dx, dw) = hip_rms_norm_bwd(g, x, w, rstd); z = dx + r`` (dx used nowhere else) ->
    ``(z, dw) = hip_rms_norm_bwd(g, x, w, rstd, r)``: the residual stream's gradient is added in the
    normalisation backward's store pass instead of a separate elementwise launch.  The same for
    ``hip_layer_norm_bwd`` (GPT-2 / NeoX blocks)."""
    from ..core.trace import from_trace, TraceProvenance

    bsyms = trace.bound_symbols
    uses: dict[str, int] = {}
    for b in bsyms:
        for a in b.flat_proxy_args:
            uses[a.name] = uses.get(a.name, 0) + 1
    producer = {}
    for i, b in enumerate(bsyms):
        for o in b.flat_proxy_outs:
            producer[o.name] = i
    drop: set[int] = set()
    replace: dict[int, object] = {}
    for i, b in enumerate(bsyms):
        if b.sym.name not in ("torch_add", "add") or b.kwargs.get("alpha") not in (None, 1):
            continue
        if len(b.args) < 2 or not all(isinstance(a, TensorProxy) for a in b.args[:2]):
            continue
        for pos in (0, 1):
            y, r = b.args[pos], b.args[1 - pos]
            j = producer.get(y.name)
            if j is None or j in drop or j in replace or uses.get(y.name, 0) != 1:
                continue
            rb = bsyms[j]
            if rb.sym is hip_rms_norm_bwd:
                nargs = 4  # (dy, x, weight, rstd[, residual])
            elif rb.sym is hip_layer_norm_bwd:
                nargs = 6  # (dy, x, weight, mean, rstd, has_bias[, residual])
            else:
                continue
            if len(rb.args) > nargs and rb.args[nargs] is not None:
                continue
            outs = rb.output
            if outs[0] is not y or tuple(r.shape) != tuple(y.shape) or r.dtype != y.dtype:
                continue
            if tuple(b.output.shape) != tuple(y.shape) or b.output.dtype != y.dtype or producer.get(r.name, -1) > j:
                continue
            nb = ex.bind_call_ctx(rb.sym.bind(*rb.args[:nargs], r, output=(b.output, *outs[1:])))
            replace[j] = nb
            drop.add(i)
            break
    if not replace:
        return trace
    new = from_trace(trace)
    new.bound_symbols = [replace.get(i, b) for i, b in enumerate(bsyms) if i not in drop]
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance(f"hipex: {len(replace)} residual-gradient add(s) fused into a normalisation backward"))
    return new


# ---- fused SwiGLU GEMMs (csrc/gemm4.hip EPI 1 / 2) ---------------------------------------
def _gate_up_meta(x, w1, w2):
    shp = tuple(x.shape[:-1]) + (w1.shape[0],)
    return TensorProxy(like=x, shape=shp), TensorProxy(like=x, shape=shp), TensorProxy(like=x, shape=shp)


def _gate_up_impl(x, w1, w2):
    from ..ops.gemm import gate_up_swiglu

    return gate_up_swiglu(x, w1, w2, need_ab=True)


def _gate_up_y_impl(x, w1, w2):
    from ..ops.gemm import gate_up_swiglu

    return gate_up_swiglu(x, w1, w2, need_ab=False)[2]


hip_gate_up = ex.register_operator("hip_gate_up", meta=_gate_up_meta, fn=_gate_up_impl)
hip_gate_up_y = ex.register_operator("hip_gate_up_y", meta=lambda x, w1, w2: _gate_up_meta(x, w1, w2)[2],
                                     fn=_gate_up_y_impl)


def _mm_swiglu_bwd_impl(dy, w, a, b):
    from ..ops.gemm import matmul_swiglu_bwd

    return matmul_swiglu_bwd(dy, w, a, b)


hip_matmul_swiglu_bwd = ex.register_operator(
    "hip_matmul_swiglu_bwd", meta=lambda dy, w, a, b: (TensorProxy(like=a), TensorProxy(like=b)), fn=_mm_swiglu_bwd_impl)


def _fuse_swiglu_gemms(trace):
    """LLaMA-MLP SwiGLU chains onto the GEMM epilogues (prefill / training shapes; decode rows go to
    the gated GEMV of :func:`_fuse_decode_gemv`):

    * forward: ``a = hip_linear(x, w1); b = hip_linear(x, w2); y = hip_swiglu(a, b)`` ->
      ``a, b, y = hip_gate_up(x, w1, w2)`` (one launch; ``hip_gate_up_y`` when nothing else reads
      a / b, e.g. inference);
    * backward: ``g = hip_matmul(dy, w); da, db = hip_swiglu_bwd(g, a, b)`` (g read nowhere else) ->
      ``da, db = hip_matmul_swiglu_bwd(dy, w, a, b)``.
    Reference counterpart: nvFuser fusing the pointwise SwiGLU into its matmul segments
    (thunder/executors/nvfuserex_impl.py:2437-2488)."""
    from ..core.trace import from_trace, TraceProvenance
    from ..ops.gemm import _fused_swiglu_on

    if not _fused_swiglu_on():
        return trace
    bsyms = list(trace.bound_symbols)
    uses: dict[str, list] = {}
    for k, b in enumerate(bsyms):
        for a in b.flat_proxy_args:
            uses.setdefault(a.name, []).append(k)
    outs = {o.name for o in tree_flatten(trace.output)[0] if isinstance(o, TensorProxy)} if trace.output is not None else set()
    producer = {}
    for i, b in enumerate(bsyms):
        for o in b.flat_proxy_outs:
            producer[o.name] = i
    drop: set[int] = set()
    replace: dict[int, object] = {}
    n_fwd = n_bwd = 0
    for i, b in enumerate(bsyms):
        if b.sym is hip_swiglu and len(b.args) == 2:
            a, g = b.args
            ja, jg = producer.get(a.name), producer.get(g.name)
            if ja is None or jg is None or ja == jg or {ja, jg} & (drop | set(replace)):
                continue
            la, lg = bsyms[ja], bsyms[jg]
            if la.sym is not hip_linear or lg.sym is not hip_linear:
                continue
            pa, pg = _linear_parts(la), _linear_parts(lg)
            if pa["x"].name != pg["x"].name or any(p.get(k) is not None for p in (pa, pg) for k in ("bias", "residual", "act")):
                continue
            x, w1, w2 = pa["x"], pa["w"], pg["w"]
            if tuple(w1.shape) != tuple(w2.shape) or _rows(x) <= _GEMV_MAX_ROWS or x.dtype != torch.bfloat16:
                continue
            at = max(ja, jg)
            # every other reader of a / b must come after the fused op's position
            others = [k for k in uses.get(a.name, []) + uses.get(g.name, []) if k != i]
            if any(k <= at for k in others):
                continue
            if others or a.name in outs or g.name in outs:
                nb = ex.bind_call_ctx(hip_gate_up.bind(x, w1, w2, output=(a, g, b.output)))
            else:
                nb = ex.bind_call_ctx(hip_gate_up_y.bind(x, w1, w2, output=b.output))
            replace[at] = nb
            drop.update((min(ja, jg), i))
            n_fwd += 1
        elif b.sym is hip_swiglu_bwd and len(b.args) == 3:
            g, a, bb = b.args
            j = producer.get(g.name)
            if j is None or j in drop or j in replace or bsyms[j].sym is not hip_matmul:
                continue
            mb = bsyms[j]
            if (len(mb.args) > 2 and mb.args[2] is not None) or uses.get(g.name, []) != [i] or g.name in outs:
                continue
            dy, w = mb.args[0], mb.args[1]
            if w.ndim != 2 or tuple(a.shape) != tuple(g.shape) or tuple(bb.shape) != tuple(g.shape):
                continue
            replace[i] = ex.bind_call_ctx(hip_matmul_swiglu_bwd.bind(dy, w, a, bb, output=b.output))
            drop.add(j)
            n_bwd += 1
    if not replace:
        return trace
    new = from_trace(trace)
    new.bound_symbols = [replace.get(i, b) for i, b in enumerate(bsyms) if i not in drop]
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance(f"hipex: {n_fwd} gate-up SwiGLU GEMM(s), {n_bwd} SwiGLU-backward GEMM epilogue(s)"))
    return new


def _linear_qkv_rope_impl(x, w, cos, sin, n_head, n_query_groups, head_size, rope_n):
    from ..ops.gemm import linear_qkv_rope

    return linear_qkv_rope(x, w, cos, sin, n_head, n_query_groups, head_size, rope_n)


def _linear_qkv_rope_meta(x, w, cos, sin, n_head, n_query_groups, head_size, rope_n):
    B, T = x.shape[0], x.shape[1]
    return (TensorProxy(like=x, shape=(B, n_head, T, head_size)),
            TensorProxy(like=x, shape=(B, n_query_groups, T, head_size)),
            TensorProxy(like=x, shape=(B, n_query_groups, T, head_size)))


hip_linear_qkv_rope = ex.register_operator("hip_linear_qkv_rope", meta=_linear_qkv_rope_meta, fn=_linear_qkv_rope_impl)


def _fuse_qkv_rope_gemm(trace):
    """``qkv = hip_linear(x, w); q, k, v = hip_qkv_rope(qkv, cos, sin, ...)`` (qkv read nowhere else,
    prefill / training rows) -> ``q, k, v = hip_linear_qkv_rope(x, w, cos, sin, ...)``: the attention
    input projection stores the RoPE'd head layouts from its epilogue (csrc/gemm4.hip EPI 3), so the
    [B, T, (nh + 2 ng) D] projection output never goes to HBM.  Reference counterpart: the
    torch.compile / nvFuser cat+RoPE fusion of thunder/executors/torch_compile.py (rope) — here it
    lands in the GEMM itself."""
    from ..core.trace import from_trace, TraceProvenance

    bsyms = list(trace.bound_symbols)
    uses: dict[str, list] = {}
    for k, b in enumerate(bsyms):
        for a in b.flat_proxy_args:
            uses.setdefault(a.name, []).append(k)
    outs = {o.name for o in tree_flatten(trace.output)[0] if isinstance(o, TensorProxy)} if trace.output is not None else set()
    producer = {}
    for i, b in enumerate(bsyms):
        for o in b.flat_proxy_outs:
            producer[o.name] = i
    drop: set[int] = set()
    replace: dict[int, object] = {}
    for i, b in enumerate(bsyms):
        if b.sym is not hip_qkv_rope or len(b.args) != 7:
            continue
        qkv, cos, sin, nh, ng, hs, rn = b.args
        j = producer.get(getattr(qkv, "name", None))
        if j is None or j in drop or bsyms[j].sym is not hip_linear or uses.get(qkv.name, []) != [i] or qkv.name in outs:
            continue
        p = _linear_parts(bsyms[j])
        if any(p.get(k) is not None for k in ("bias", "residual", "act")) or p["x"].ndim != 3 or _rows(p["x"]) <= _GEMV_MAX_ROWS:
            continue
        if not all(isinstance(v, int) for v in (nh, ng, hs, rn)):
            continue
        if producer.get(getattr(cos, "name", None), -1) > j or producer.get(getattr(sin, "name", None), -1) > j:
            continue  # cos / sin must exist where the GEMM runs
        replace[j] = ex.bind_call_ctx(hip_linear_qkv_rope.bind(p["x"], p["w"], cos, sin, nh, ng, hs, rn, output=b.output))
        drop.add(i)
    if not replace:
        return trace
    new = from_trace(trace)
    new.bound_symbols = [replace.get(i, b) for i, b in enumerate(bsyms) if i not in drop]
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance(f"hipex: {len(replace)} qkv projection(s) with the RoPE split in the GEMM epilogue"))
    return new


def _fp8_gemm_qkv_rope_impl(qa, qb, sa, sb, out_shape, cos, sin, n_head, n_query_groups, head_size, rope_n):
    from ..ops.fp8 import gemm_qkv_rope

    return gemm_qkv_rope(qa, qb, sa, sb, out_shape, cos, sin, n_head, n_query_groups, head_size, rope_n)


def _fp8_gemm_qkv_rope_meta(qa, qb, sa, sb, out_shape, cos, sin, n_head, n_query_groups, head_size, rope_n):
    B, T = out_shape[0], out_shape[1]
    mk = lambda h: TensorProxy(like=sa, shape=(B, h, T, head_size), dtype=torch.bfloat16)  # noqa: E731
    return mk(n_head), mk(n_query_groups), mk(n_query_groups)


hip_fp8_gemm_qkv_rope = ex.register_operator("hip_fp8_gemm_qkv_rope", meta=_fp8_gemm_qkv_rope_meta,
                                             fn=_fp8_gemm_qkv_rope_impl)


def _fuse_fp8_qkv_rope_gemm(trace):
    """``qkv = hip_fp8_gemm(qx, qw, sx, sw, 0, 0, None, shape); q, k, v = hip_qkv_rope(qkv, ...)`` (qkv
    read nowhere else) -> ``q, k, v = hip_fp8_gemm_qkv_rope(...)``: the FP8 path's counterpart of
    :func:`_fuse_qkv_rope_gemm` (csrc/gemm4_fp8.hip QKV epilogue; reference: TransformerEngine's fused
    attention input projection, thunder/executors/transformer_engineex_impl.py)."""
    from ..core.trace import from_trace, TraceProvenance

    bsyms = list(trace.bound_symbols)
    uses: dict[str, list] = {}
    for k, b in enumerate(bsyms):
        for a in b.flat_proxy_args:
            uses.setdefault(a.name, []).append(k)
    outs = {o.name for o in tree_flatten(trace.output)[0] if isinstance(o, TensorProxy)} if trace.output is not None else set()
    producer = {}
    for i, b in enumerate(bsyms):
        for o in b.flat_proxy_outs:
            producer[o.name] = i
    drop: set[int] = set()
    replace: dict[int, object] = {}
    for i, b in enumerate(bsyms):
        if b.sym is not hip_qkv_rope or len(b.args) != 7:
            continue
        qkv, cos, sin, nh, ng, hs, rn = b.args
        j = producer.get(getattr(qkv, "name", None))
        if j is None or j in drop or j in replace or bsyms[j].sym is not hip_fp8_gemm or uses.get(qkv.name, []) != [i] \
                or qkv.name in outs:
            continue
        ga = bsyms[j].args
        if len(ga) < 8 or (len(ga) > 8 and ga[8] is not None) or ga[4] != 0 or ga[5] != 0 or ga[6] is not None:
            continue
        out_shape = tuple(ga[7])
        if len(out_shape) != 3 or not all(isinstance(v, int) for v in (nh, ng, hs, rn) + out_shape):
            continue
        if producer.get(getattr(cos, "name", None), -1) > j or producer.get(getattr(sin, "name", None), -1) > j:
            continue
        replace[j] = ex.bind_call_ctx(hip_fp8_gemm_qkv_rope.bind(ga[0], ga[1], ga[2], ga[3], out_shape, cos, sin, nh, ng,
                                                                 hs, rn, output=b.output))
        drop.add(i)
    if not replace:
        return trace
    new = from_trace(trace)
    new.bound_symbols = [replace.get(i, b) for i, b in enumerate(bsyms) if i not in drop]
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance(f"hipex: {len(replace)} fp8 qkv projection(s) with the RoPE split in the GEMM epilogue"))
    return new


def _attn_bwd_rope_meta(g, q, k, v, o, lse, causal, scale, cos, sin, n_head, n_query_groups):
    B, _, T, D = q.shape
    return TensorProxy(like=g, shape=(B, T, (n_head + 2 * n_query_groups) * D))


def _attn_bwd_rope_impl(g, q, k, v, o, lse, causal, scale, cos, sin, n_head, n_query_groups):
    from ..ops.attention import attn_bwd_rope

    return attn_bwd_rope(g, q, k, v, o, lse, causal, scale, cos, sin, n_head, n_query_groups)


hip_attn_bwd_rope = ex.register_operator("hip_flash_attn_bwd_rope", meta=_attn_bwd_rope_meta, fn=_attn_bwd_rope_impl)


def _fuse_attn_bwd_rope(trace):
    """``dq, dk, dv = hip_flash_attn_bwd(...); dqkv = hip_qkv_rope_bwd(dq, dk, dv, cos, sin, ...)``
    (dq / dk / dv read nowhere else, full-width rotate-half RoPE on 128-wide heads) ->
    ``dqkv = hip_flash_attn_bwd_rope(..., cos, sin, n_head, n_query_groups)``: the RoPE backward
    runs in the attention backward's dQ / dK epilogues and the three gradients are stored straight
    into the fused projection's gradient (the mirror of the qkv-RoPE GEMM epilogue of the forward)."""
    from ..core.trace import from_trace, TraceProvenance

    bsyms = trace.bound_symbols
    uses: dict[str, int] = {}
    for b in bsyms:
        for a in b.flat_proxy_args:
            uses[a.name] = uses.get(a.name, 0) + 1
    producer = {}
    for i, b in enumerate(bsyms):
        for o in b.flat_proxy_outs:
            producer[o.name] = i
    drop: set[int] = set()
    replace: dict[int, object] = {}
    for i, b in enumerate(bsyms):
        if b.sym is not hip_qkv_rope_bwd or len(b.args) != 9:
            continue
        gq, gk, gv, cos, sin, nh, ng, hs, rn = b.args
        if not all(isinstance(t, TensorProxy) for t in (gq, gk, gv, cos, sin)) or hs != 128 or rn != hs:
            continue
        j = producer.get(gq.name)
        if j is None or j in drop or bsyms[j].sym is not hip_attn_bwd:
            continue
        ab = bsyms[j]
        if tuple(o.name for o in ab.flat_proxy_outs) != (gq.name, gk.name, gv.name):
            continue
        if any(uses.get(t.name, 0) != 1 for t in (gq, gk, gv)):
            continue
        g, q, k, v, o, lse, causal, scale = ab.args
        if q.shape[1] != nh or k.shape[1] != ng or q.shape[2] != k.shape[2]:
            continue
        replace[i] = ex.bind_call_ctx(hip_attn_bwd_rope.bind(g, q, k, v, o, lse, causal, scale, cos, sin, nh, ng,
                                                             output=b.output))
        drop.add(j)
    if not replace:
        return trace
    new = from_trace(trace)
    new.bound_symbols = [replace.get(i, b) for i, b in enumerate(bsyms) if i not in drop]
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance(f"hipex: {len(replace)} RoPE backward(s) fused into the attention backward"))
    return new


def _rms_bwd_fp8_meta(dy, x, weight, rstd, residual, key, slot):
    q, sc = _fp8_cast_meta(x, True)
    return TensorProxy(like=x), (None if weight is None else TensorProxy(like=weight)), q, sc


def _rms_bwd_fp8_impl(dy, x, weight, rstd, residual, key, slot):
    from ..ops.fp8 import rms_norm_bwd_fp8_delayed

    return rms_norm_bwd_fp8_delayed(dy, x, weight, rstd, residual, key, slot)


hip_rms_norm_bwd_fp8 = ex.register_operator("hip_rms_norm_bwd_fp8", meta=_rms_bwd_fp8_meta, fn=_rms_bwd_fp8_impl)


def _fuse_fp8_rms_bwd_casts(trace):
    """``dx, dw = hip_rms_norm_bwd(g, x, w, rstd[, r]); q, s = hip_fp8_cast_delayed(dx, True, key, slot)``
    -> ``dx, dw, q, s = hip_rms_norm_bwd_fp8(g, x, w, rstd, r, key, slot)``: a LLaMA block's residual-
    stream gradient is the output gradient of the preceding fp8 linear (the attention projection after
    norm_2's backward, the previous block's MLP projection after norm_1's), so its e5m2 copy leaves the
    norm backward's store pass (dx keeps its other uses; the cast launch re-reading dx disappears).
    Runs after :func:`_fuse_rms_bwd_residual`, so the residual add is already in the norm backward."""
    import os

    from ..core.trace import from_trace, TraceProvenance

    if os.environ.get("LTA_FP8_FUSE_PRODUCERS", "1") == "0":  # A/B hook (with the forward producers)
        return trace
    bsyms = trace.bound_symbols
    producer = {}
    for i, b in enumerate(bsyms):
        for o in b.flat_proxy_outs:
            producer[o.name] = i
    drop: set[int] = set()
    replace: dict[int, object] = {}
    for i, b in enumerate(bsyms):
        if b.sym is not hip_fp8_cast_delayed or len(b.args) != 4 or not b.args[1]:
            continue
        y, _, key, slot = b.args
        j = producer.get(y.name)
        if j is None or j in replace:
            continue
        pb = bsyms[j]
        if pb.sym is not hip_rms_norm_bwd or pb.output[0].name != y.name:
            continue
        res = pb.args[4] if len(pb.args) > 4 else None
        nb = hip_rms_norm_bwd_fp8.bind(*pb.args[:4], res, key, slot,
                                       output=(pb.output[0], pb.output[1], b.output[0], b.output[1]))
        replace[j] = ex.bind_call_ctx(nb)
        drop.add(i)
    if not replace:
        return trace
    new = from_trace(trace)
    new.bound_symbols = [replace.get(i, b) for i, b in enumerate(bsyms) if i not in drop]
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance(f"hipex: {len(replace)} e5m2 gradient cast(s) fused into RMSNorm backwards"))
    return new


def _attn_fwd_fp8_meta(q, k, v, causal, scale, key, slot):
    B, H, L, E = q.shape
    return (TensorProxy(like=q), TensorProxy(like=q, shape=(B, H, L), dtype=torch.float32, requires_grad=False),
            TensorProxy(like=q, shape=(B * L, H * E), dtype=torch.uint8, requires_grad=False),
            TensorProxy(like=q, shape=(), dtype=torch.float32, requires_grad=False))


def _attn_fwd_fp8_impl(q, k, v, causal, scale, key, slot):
    from ..ops.fp8 import attn_fwd_fp8_delayed

    return attn_fwd_fp8_delayed(q, k, v, causal, scale, key, slot)


hip_attn_fwd_fp8 = ex.register_operator("hip_flash_attn_fwd_fp8", meta=_attn_fwd_fp8_meta, fn=_attn_fwd_fp8_impl)

# the view ops of o.transpose(1, 2).reshape(B, T, H D) at every level a trace can hold them (ltorch symbols
# before flattening, their torch-executor operators, the prims)
_HEAD_MERGE_VIEWS = {"transpose", "permute", "reshape", "view", "torch_transpose", "torch_permute", "torch_reshape",
                     "torch_view", "transpose_prim", "reshape_prim"}


def _merges_heads(chain, out) -> bool:
    """``chain`` (producer order) turns the attention output [B, H, T, D] into its [B, T, H D] (or
    [B T, H D]) rows: one (1, 2) transpose / permute, then reshapes only."""
    B, H, T, D = out.shape
    swapped = False
    for b in chain:
        n = b.sym.name
        if n in ("transpose", "torch_transpose"):
            dims = {int(pyval(d)) % 4 for d in b.args[1:3]}
            if swapped or dims != {1, 2}:
                return False
            swapped = True
        elif n in ("permute", "torch_permute", "transpose_prim"):
            perm = (b.args[1] if len(b.args) == 2 else b.args[1:]) if len(b.args) > 1 else \
                b.kwargs.get("permutation", b.kwargs.get("dims"))
            try:
                perm = tuple(int(pyval(d)) % 4 for d in perm)
            except TypeError:
                return False
            if swapped or perm != (0, 2, 1, 3):
                return False
            swapped = True
        elif not swapped:
            return False
    y = chain[-1].output
    return swapped and tuple(y.shape) in ((B, T, H * D), (B * T, H * D))


def _fuse_fp8_attn_out_casts(trace):
    """``o, lse = hip_flash_attn_fwd(q, k, v, ...); y = o.transpose(1, 2).reshape(B, T, H D);
    qy, sy = hip_fp8_cast_delayed(y, False, key, slot)`` -> ``o, lse, qy, sy = hip_flash_attn_fwd_fp8(q, k,
    v, ..., key, slot)``: the e4m3 input of the FP8 output projection leaves the attention epilogue
    (O is stored [B, T, H, D], so its rows are the projection's rows); O itself is still written for the
    backward.  The view chain stays for its other readers."""
    import os

    from ..core.trace import from_trace, TraceProvenance

    if os.environ.get("LTA_FP8_FUSE_PRODUCERS", "1") == "0":
        return trace
    bsyms = trace.bound_symbols
    producer = {}
    for i, b in enumerate(bsyms):
        for o in b.flat_proxy_outs:
            producer[o.name] = i
    drop: set[int] = set()
    replace: dict[int, object] = {}
    for i, b in enumerate(bsyms):
        if b.sym is not hip_fp8_cast_delayed or len(b.args) != 4 or b.args[1]:
            continue
        y, _, key, slot = b.args
        chain, cur = [], y
        j = producer.get(cur.name)
        while j is not None and bsyms[j].sym.name in _HEAD_MERGE_VIEWS and len(chain) < 4:
            chain.append(bsyms[j])
            cur = bsyms[j].args[0]
            if not isinstance(cur, TensorProxy):
                break
            j = producer.get(cur.name)
        if j is None or j in replace or not chain or bsyms[j].sym is not hip_attn_fwd:
            continue
        ab = bsyms[j]
        out = ab.output[0]
        if cur.name != out.name or out.dtype != torch.bfloat16 or out.shape[-1] != 128:
            continue
        if not _merges_heads(chain[::-1], out):
            continue
        nb = hip_attn_fwd_fp8.bind(*ab.args[:5], key, slot, output=(ab.output[0], ab.output[1], b.output[0], b.output[1]))
        replace[j] = ex.bind_call_ctx(nb)
        drop.add(i)
    if not replace:
        return trace
    new = from_trace(trace)
    new.bound_symbols = [replace.get(i, b) for i, b in enumerate(bsyms) if i not in drop]
    new.scopes = [new.bound_symbols]
    new.set_provenance(TraceProvenance(f"hipex: {len(replace)} e4m3 attention-output cast(s) fused into the attention epilogue"))
    return new


def _post_claim(trace):
    return _fuse_attn_bwd_rope(_fuse_fp8_qkv_rope_gemm(_fuse_qkv_rope_gemm(_group_decode_projections(_fuse_kv_cache_writes(_fuse_swiglu_gemms(
        _fuse_decode_gemv(_fuse_fp8_rms_bwd_casts(_fuse_rms_bwd_residual(_fuse_linear_epilogues(
            _fuse_fp8_attn_out_casts(_fuse_fp8_cast_producers(trace))))))))))))


ex.post_claim_pass = _post_claim


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


def _rms_bwd_meta(dy, x, weight, rstd, residual=None):
    return TensorProxy(like=x), (None if weight is None else TensorProxy(like=weight))


def _rms_bwd_impl(dy, x, weight, rstd, residual=None):
    from ..ops.rmsnorm import rms_norm_bwd

    return rms_norm_bwd(dy, x, weight, rstd, residual)


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


# =========================================================================================
# K10 grouped GEMM (MoE experts)
# =========================================================================================
def _gmm_meta(a, b, offs):
    if a.ndim == 2 and b.ndim == 2:  # the wgrad form: [G, K, N]
        return TensorProxy(like=a, shape=(offs.shape[0], a.shape[0], b.shape[1]))
    return TensorProxy(like=a, shape=(a.shape[0], b.shape[2]))


def _gmm_impl(a, b, offs):
    from ..ops.gemm import grouped_mm

    return grouped_mm(a, b, offs)


hip_grouped_mm = ex.register_operator("hip_grouped_mm", meta=_gmm_meta, fn=_gmm_impl)


def _gmm_checker(a, b, offs=None, bias=None, out_dtype=None):
    """Forward / dgrad (2-D x 3-D) and wgrad (2-D x 2-D, reduction over each group's rows) forms:
    the VJP of _grouped_mm (transforms/autodiff.py) emits all three, so MoE training runs every
    expert GEMM on the hand kernels (csrc/gemm4.hip grouped modes)."""
    return (_gpu(a, b, offs) and offs is not None and bias is None and out_dtype is None and a.ndim == 2
            and b.ndim in (2, 3) and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16)


def _gmm_exec(a, b, offs=None, bias=None, out_dtype=None):
    return hip_grouped_mm(a, b, offs)


# =========================================================================================
# K5 LayerNorm
# =========================================================================================
def _ln_fwd_meta(x, weight, bias, eps):
    rows = 1
    for d in x.shape[:-1]:
        rows *= d
    st = TensorProxy(like=x, shape=(rows,), dtype=torch.float32, requires_grad=False)
    return TensorProxy(like=x), st, TensorProxy(like=st)


def _ln_fwd_impl(x, weight, bias, eps):
    from ..ops.rmsnorm import layer_norm_fwd

    return layer_norm_fwd(x, weight, bias, eps)


def _ln_bwd_meta(dy, x, weight, mean, rstd, has_bias, residual=None):
    return (TensorProxy(like=x), None if weight is None else TensorProxy(like=weight),
            TensorProxy(like=x, shape=(x.shape[-1],)) if has_bias else None)


def _ln_bwd_impl(dy, x, weight, mean, rstd, has_bias, residual=None):
    from ..ops.rmsnorm import layer_norm_bwd

    return layer_norm_bwd(dy, x, weight, mean, rstd, has_bias, residual)


hip_layer_norm_fwd = ex.register_operator("hip_layer_norm_fwd", meta=_ln_fwd_meta, fn=_ln_fwd_impl)
hip_layer_norm_bwd = ex.register_operator("hip_layer_norm_bwd", meta=_ln_bwd_meta, fn=_ln_bwd_impl)


def _ln_checker(a, normalized_shape, weight=None, bias=None, eps=1e-5):
    if not _gpu(a, weight, bias) or a.dtype not in _FLOAT16ISH:
        return False
    if len(normalized_shape) != 1 or normalized_shape[0] != a.shape[-1]:
        return False
    for t in (weight, bias):
        if t is not None and (t.dtype != a.dtype or tuple(t.shape) != (a.shape[-1],)):
            return False
    return True


def _ln_exec(a, normalized_shape, weight=None, bias=None, eps=1e-5):
    y, _, _ = hip_layer_norm_fwd(a, weight, bias, eps)
    return y


def _ln_grad(a, normalized_shape, weight=None, bias=None, eps=1e-5):
    y, mean, rstd = hip_layer_norm_fwd(a, weight, bias, eps)

    def bwd(g):
        dx, dw, db = hip_layer_norm_bwd(g, a, weight, mean, rstd, bias is not None)
        return dx, None, dw, db

    return y, bwd


# =========================================================================================
# K6 fused qkv split + RoPE (lookaside for the LitGPT helper `qkv_split_rope`)
# =========================================================================================
def _qkv_rope_meta(qkv, cos, sin, n_head, n_query_groups, head_size, rope_n):
    B, T, _ = qkv.shape
    q = TensorProxy(like=qkv, shape=(B, n_head, T, head_size))
    k = TensorProxy(like=qkv, shape=(B, n_query_groups, T, head_size))
    v = TensorProxy(like=qkv, shape=(B, n_query_groups, T, head_size))
    return q, k, v


def _qkv_rope_impl(qkv, cos, sin, n_head, n_query_groups, head_size, rope_n):
    from ..ops.fused import qkv_rope_fwd

    return qkv_rope_fwd(qkv, cos, sin, n_head, n_query_groups, head_size, rope_n)


def _qkv_rope_bwd_meta(dq, dk, dv, cos, sin, n_head, n_query_groups, head_size, rope_n):
    B, _, T, _ = dq.shape
    return TensorProxy(like=dq, shape=(B, T, (n_head + 2 * n_query_groups) * head_size))


def _qkv_rope_bwd_impl(dq, dk, dv, cos, sin, n_head, n_query_groups, head_size, rope_n):
    from ..ops.fused import qkv_rope_bwd

    return qkv_rope_bwd(dq, dk, dv, cos, sin, n_head, n_query_groups, head_size, rope_n)


hip_qkv_rope = ex.register_operator("hip_qkv_rope", meta=_qkv_rope_meta, fn=_qkv_rope_impl)
hip_qkv_rope_bwd = ex.register_operator("hip_qkv_rope_bwd", meta=_qkv_rope_bwd_meta, fn=_qkv_rope_bwd_impl)


def _qkv_rope_vjp(qkv, cos, sin, n_head, n_query_groups, head_size, rope_n):
    q, k, v = hip_qkv_rope(qkv, cos, sin, n_head, n_query_groups, head_size, rope_n)

    def bwd(gq, gk, gv):
        return (hip_qkv_rope_bwd(gq, gk, gv, cos, sin, n_head, n_query_groups, head_size, rope_n),)

    return (q, k, v), bwd


def qkv_split_rope_lookaside(qkv, cos, sin, n_head, n_query_groups, head_size, rope_n_elem):
    ok = (
        _gpu(qkv, cos, sin)
        and qkv.dtype in _FLOAT16ISH
        and qkv.ndim == 3
        and head_size % 8 == 0
        and rope_n_elem % 16 == 0
        and rope_n_elem <= head_size
        and cos.ndim == 2
        and cos.shape[0] >= qkv.shape[1]
        and cos.shape[1] == rope_n_elem
        and cos.dtype in (torch.float32, qkv.dtype)
    )
    if not ok:
        return qkv_split_rope_lookaside.__wrapped_original__(qkv, cos, sin, n_head, n_query_groups, head_size, rope_n_elem)
    return hip_qkv_rope(qkv, cos, sin, n_head, n_query_groups, head_size, rope_n_elem)


# =========================================================================================
# SwiGLU (lookaside for the LitGPT helper `swiglu`)
# =========================================================================================
hip_swiglu = ex.register_operator("hip_swiglu", meta=lambda a, b: TensorProxy(like=a),
                                  fn=lambda a, b: __import__("lightning_thunder_amd.ops.fused", fromlist=["x"]).swiglu_fwd(a, b))
hip_swiglu_bwd = ex.register_operator(
    "hip_swiglu_bwd", meta=lambda g, a, b: (TensorProxy(like=a), TensorProxy(like=b)),
    fn=lambda g, a, b: __import__("lightning_thunder_amd.ops.fused", fromlist=["x"]).swiglu_bwd(g, a, b),
)


def _swiglu_vjp(a, b):
    y = hip_swiglu(a, b)

    def bwd(g):
        da, db = hip_swiglu_bwd(g, a, b)
        return da, db

    return y, bwd


def swiglu_lookaside(a, b):
    if _gpu(a, b) and a.dtype in _FLOAT16ISH and a.dtype == b.dtype and tuple(a.shape) == tuple(b.shape):
        return hip_swiglu(a, b)
    return swiglu_lookaside.__wrapped_original__(a, b)


# =========================================================================================
# K7 softmax cross-entropy
# =========================================================================================
def _ce_fwd_meta(logits, target, ignore_index, reduction, label_smoothing, weight=None):
    rows = logits.shape[0]
    loss = TensorProxy(like=logits, shape=(rows,) if reduction == "none" else ())
    lse = TensorProxy(like=logits, shape=(rows,), dtype=torch.float32, requires_grad=False)
    stats = TensorProxy(like=logits, shape=(2,), dtype=torch.float32, requires_grad=False)
    return loss, lse, stats


def _ce_fwd_impl(logits, target, ignore_index, reduction, label_smoothing, weight=None):
    from ..ops.fused import cross_entropy_fwd

    return cross_entropy_fwd(logits, target, ignore_index, reduction, label_smoothing, weight)


def _ce_bwd_impl(g, logits, target, lse, stats, ignore_index, reduction, label_smoothing, weight=None):
    from ..ops.fused import cross_entropy_bwd

    return cross_entropy_bwd(g, logits, target, lse, stats, ignore_index, reduction, label_smoothing, weight)


hip_cross_entropy_fwd = ex.register_operator("hip_cross_entropy_fwd", meta=_ce_fwd_meta, fn=_ce_fwd_impl)
hip_cross_entropy_bwd = ex.register_operator(
    "hip_cross_entropy_bwd", meta=lambda g, logits, *a, **k: TensorProxy(like=logits), fn=_ce_bwd_impl
)


def _ce_checker(a, target, weight=None, size_average=None, ignore_index=-100, reduce=None, reduction="mean", label_smoothing=0.0):
    return (
        _gpu(a, target, weight)
        and a.ndim == 2
        and target.ndim == 1
        and (weight is None or (weight.ndim == 1 and weight.shape[0] == a.shape[1]
                                and weight.dtype in (torch.float32, torch.bfloat16, torch.float16)))
        and size_average is None
        and reduce is None
        and reduction in ("mean", "sum", "none")
        and a.dtype in _FLOAT16ISH
        and target.dtype in (torch.int64, torch.int32)
    )


def _ce_exec(a, target, weight=None, size_average=None, ignore_index=-100, reduce=None, reduction="mean", label_smoothing=0.0):
    if weight is None:
        loss, _, _ = hip_cross_entropy_fwd(a, target, ignore_index, reduction, label_smoothing)
    else:
        loss, _, _ = hip_cross_entropy_fwd(a, target, ignore_index, reduction, label_smoothing, weight)
    return loss


def _ce_grad(a, target, weight=None, size_average=None, ignore_index=-100, reduce=None, reduction="mean", label_smoothing=0.0):
    # class weights (reference: triton_crossentropy_impl.py:49-151) are a constant of the loss: no grad
    extra = () if weight is None else (weight,)
    loss, lse, stats = hip_cross_entropy_fwd(a, target, ignore_index, reduction, label_smoothing, *extra)

    def bwd(g):
        return (hip_cross_entropy_bwd(g, a, target, lse, stats, ignore_index, reduction, label_smoothing, *extra),)

    return loss, bwd


# =========================================================================================
# K3 flash attention (claims ltorch.scaled_dot_product_attention; saves O and LSE for backward)
# =========================================================================================
def _attn_fwd_meta(q, k, v, causal, scale):
    B, H, L, E = q.shape
    return TensorProxy(like=q), TensorProxy(like=q, shape=(B, H, L), dtype=torch.float32, requires_grad=False)


def _attn_fwd_impl(q, k, v, causal, scale):
    from ..ops.attention import attn_fwd

    return attn_fwd(q, k, v, causal, scale)


def _attn_bwd_impl(g, q, k, v, o, lse, causal, scale):
    from ..ops.attention import attn_bwd

    return attn_bwd(g, q, k, v, o, lse, causal, scale)


hip_attn_fwd = ex.register_operator("hip_flash_attn_fwd", meta=_attn_fwd_meta, fn=_attn_fwd_impl)
hip_attn_bwd = ex.register_operator(
    "hip_flash_attn_bwd",
    meta=lambda g, q, k, v, o, lse, causal, scale: (TensorProxy(like=q), TensorProxy(like=k), TensorProxy(like=v)),
    fn=_attn_bwd_impl,
)


# masked / dropout variant (additive or boolean mask, counter-based dropout of P, optional mask
# gradient): the same kernels with the extra terms compiled in (ops/attention.py: lta_attn_*_ex)
def _attn_fwd_ex_meta(q, k, v, mask, causal, scale, dropout_p, seed, offset):
    B, H, L, E = q.shape
    return TensorProxy(like=q), TensorProxy(like=q, shape=(B, H, L), dtype=torch.float32, requires_grad=False)


def _attn_fwd_ex_impl(q, k, v, mask, causal, scale, dropout_p, seed, offset):
    from ..ops.attention import attn_fwd

    return attn_fwd(q, k, v, causal, scale, mask=mask, dropout_p=dropout_p, seed=seed, offset=offset)


def _attn_bwd_ex_meta(g, q, k, v, o, lse, mask, causal, scale, dropout_p, seed, offset, mask_grad):
    outs = (TensorProxy(like=q), TensorProxy(like=k), TensorProxy(like=v))
    return outs + ((TensorProxy(like=mask),) if mask_grad else ())


def _attn_bwd_ex_impl(g, q, k, v, o, lse, mask, causal, scale, dropout_p, seed, offset, mask_grad):
    from ..ops.attention import attn_bwd

    return attn_bwd(g, q, k, v, o, lse, causal, scale, mask=mask, dropout_p=dropout_p, seed=seed, offset=offset,
                    mask_grad=mask_grad)


hip_attn_fwd_ex = ex.register_operator("hip_flash_attn_fwd_ex", meta=_attn_fwd_ex_meta, fn=_attn_fwd_ex_impl)
hip_attn_bwd_ex = ex.register_operator("hip_flash_attn_bwd_ex", meta=_attn_bwd_ex_meta, fn=_attn_bwd_ex_impl)


def _decode_attn_meta(q, k, v, mask, causal, scale):
    return TensorProxy(like=q)


def _decode_attn_impl(q, k, v, mask, causal, scale):
    from ..ops.attention import decode_attn

    return decode_attn(q, k, v, mask, causal, scale)


hip_decode_attn = ex.register_operator("hip_decode_attn", meta=_decode_attn_meta, fn=_decode_attn_impl)


def _broadcastable(shape, target) -> bool:
    if len(shape) > len(target):
        return False
    for a, b in zip(reversed(shape), reversed(target)):
        if a != 1 and a != b:
            return False
    return True


def _is_decode_shape(query, key, attn_mask) -> bool:
    from ..ops.attention import DECODE_MAX_QUERIES

    if attn_mask is None or not isinstance(attn_mask, TensorProxy) or attn_mask.dtype != torch.bool:
        return False
    B, Hq, T, _ = query.shape
    return T <= DECODE_MAX_QUERIES and _broadcastable(tuple(attn_mask.shape), (B, Hq, T, key.shape[2]))


def _is_decode(query, key, attn_mask) -> bool:
    """Few query rows against a KV cache with a boolean mask: the K3d decode kernel."""
    from ..ops.attention import DECODE_MAX_QUERIES

    if attn_mask is None or not isinstance(attn_mask, TensorProxy) or attn_mask.dtype != torch.bool:
        return False
    B, Hq, T, D = query.shape
    if D not in (64, 128):  # the decode kernel's head dims (others take the padded flash path)
        return False
    return T <= DECODE_MAX_QUERIES and _broadcastable(tuple(attn_mask.shape), (B, Hq, T, key.shape[2]))


def _sdpa_checker(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False, *, scale=None, enable_gqa=False):
    if not _gpu(query, key, value):
        return False
    if query.ndim != 4 or key.ndim != 4 or value.ndim != 4:
        return False
    try:
        p = float(pyval(dropout_p))
    except Exception:  # a symbolic dropout probability: let the decomposition run
        return False
    if not 0.0 <= p < 1.0:
        return False
    if attn_mask is not None:
        if not isinstance(attn_mask, TensorProxy) or attn_mask.device.type != "cuda":
            return False
        if attn_mask.dtype != torch.bool and not dtypes.is_float_dtype(attn_mask.dtype):
            return False
        if not _broadcastable(tuple(attn_mask.shape), (query.shape[0], query.shape[1], query.shape[2], key.shape[2])):
            return False
        if is_causal and attn_mask is not None:
            return False  # torch rejects the combination as well
    if query.dtype not in (torch.bfloat16, torch.float16) or key.dtype != query.dtype or value.dtype != query.dtype:
        return False
    D = query.shape[-1]
    from ..ops.attention import padded_head_dim, PLAIN_ONLY_HEAD_DIM

    if padded_head_dim(D) is None or key.shape[-1] != D or value.shape[-1] != D:
        return False
    if D > PLAIN_ONLY_HEAD_DIM and (attn_mask is not None or p > 0.0):
        return False
    if D not in (64, 128) and _is_decode_shape(query, key, attn_mask):
        return False  # decode steps at head dims without a decode kernel stay on ATen (padding buys nothing there)
    if key.shape[1] != value.shape[1] or query.shape[1] % key.shape[1] != 0:
        return False
    if key.shape[1] != query.shape[1] and not enable_gqa:
        return False
    return query.shape[0] == key.shape[0] == value.shape[0] and key.shape[2] == value.shape[2]


def _sc(q, scale):
    return scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])


def _p(dropout_p) -> float:
    return float(pyval(dropout_p))


def _rng(query, key, p):
    """(seed, offset) of the framework's Philox stream, advanced by one draw per score."""
    if not p:
        return 0, 0
    from ..core import prims as P

    B, H, L, _ = query.shape
    return P.get_rng_seed_offset(B * H * L * key.shape[2])


def _sdpa_exec(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False, *, scale=None, enable_gqa=False):
    p = _p(dropout_p)
    if attn_mask is not None and not p and _is_decode(query, key, attn_mask):
        return hip_decode_attn(query, key, value, attn_mask, bool(is_causal), _sc(query, scale))
    if attn_mask is None and not p:
        out, _ = hip_attn_fwd(query, key, value, bool(is_causal), _sc(query, scale))
        return out
    seed, offset = _rng(query, key, p)
    out, _ = hip_attn_fwd_ex(query, key, value, attn_mask, bool(is_causal), _sc(query, scale), p, seed, offset)
    return out


def _sdpa_grad(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False, *, scale=None, enable_gqa=False):
    sc = _sc(query, scale)
    p = _p(dropout_p)
    if attn_mask is None and not p:
        out, lse = hip_attn_fwd(query, key, value, bool(is_causal), sc)

        def bwd(g):
            dq, dk, dv = hip_attn_bwd(g, query, key, value, out, lse, bool(is_causal), sc)
            return dq, dk, dv

        return out, bwd
    seed, offset = _rng(query, key, p)
    out, lse = hip_attn_fwd_ex(query, key, value, attn_mask, bool(is_causal), sc, p, seed, offset)
    mask_grad = bool(attn_mask is not None and attn_mask.dtype != torch.bool and attn_mask.requires_grad)

    def bwd(g):
        res = hip_attn_bwd_ex(g, query, key, value, out, lse, attn_mask, bool(is_causal), sc, p, seed, offset, mask_grad)
        if mask_grad:
            return res[0], res[1], res[2], res[3]
        return res[0], res[1], res[2]

    return out, bwd


# =========================================================================================
# K11 embedding backward / index_add, K12 topk / sort / cumsum (csrc/index_ops.hip)
# =========================================================================================
_SORT_DT = (torch.float32, torch.float16, torch.bfloat16, torch.int32)
_ROW_DT = (torch.float32, torch.float16, torch.bfloat16)
_SORT_MAX = 16384


def _topk_meta(a, k, dim, largest, sorted):
    shape = list(a.shape)
    shape[dim] = k
    return TensorProxy(like=a, shape=tuple(shape)), TensorProxy(like=a, shape=tuple(shape), dtype=torch.int64,
                                                                requires_grad=False)


def _topk_impl(a, k, dim, largest, sorted):
    from ..ops import index_ops

    return index_ops.topk(a, k, dim, largest, sorted)


def _sort_meta(a, dim, descending, stable):
    return TensorProxy(like=a), TensorProxy(like=a, dtype=torch.int64, requires_grad=False)


def _sort_impl(a, dim, descending, stable):
    from ..ops import index_ops

    return index_ops.sort(a, dim, descending, stable)


def _cumsum_meta(a, dim, out_i32=False):
    if a.dtype in (torch.int32, torch.int64):
        return TensorProxy(like=a, dtype=torch.int32 if out_i32 else torch.int64)
    return TensorProxy(like=a)


def _cumsum_impl(a, dim, out_i32=False):
    from ..ops import index_ops

    return index_ops.cumsum(a, dim, torch.int32 if out_i32 else None)


def _emb_bwd_meta(grad, indices, num_weights, padding_idx, scale_grad_by_freq):
    return TensorProxy(like=grad, shape=(num_weights, grad.shape[-1]))


def _emb_bwd_impl(grad, indices, num_weights, padding_idx, scale_grad_by_freq):
    from ..ops import index_ops

    return index_ops.embedding_backward(grad, indices, num_weights, padding_idx, scale_grad_by_freq)


def _index_add_meta(a, index, src):
    return TensorProxy(like=a)


def _index_add_impl(a, index, src):
    from ..ops import index_ops

    return index_ops.index_add(a, index, src)


hip_topk = ex.register_operator("hip_topk", meta=_topk_meta, fn=_topk_impl)
hip_sort = ex.register_operator("hip_sort", meta=_sort_meta, fn=_sort_impl)
hip_cumsum = ex.register_operator("hip_cumsum", meta=_cumsum_meta, fn=_cumsum_impl)
hip_embedding_backward = ex.register_operator("hip_embedding_backward", meta=_emb_bwd_meta, fn=_emb_bwd_impl)
hip_index_add = ex.register_operator("hip_index_add", meta=_index_add_meta, fn=_index_add_impl)


def _numel(shape) -> int:
    n = 1
    for d in shape:
        n = n * d  # symbolic dims stay symbolic (core/symbolic.py)
    return n


def _topk_checker(a, k, dim, largest, sorted):
    if not (_gpu(a) and a.dtype in _SORT_DT and a.ndim >= 1 and _numel(a.shape) > 0):
        return False
    n = a.shape[dim]
    return 1 <= pyval(k) <= n <= _SORT_MAX


def _topk_exec(a, k, dim, largest, sorted):
    return hip_topk(a, pyval(k), dim, bool(largest), bool(sorted))


def _sort_checker(a, dim, descending, stable):
    if a.dtype == torch.int64:  # 64-bit keys + separate positions: half the LDS capacity
        return _gpu(a) and a.ndim >= 1 and _numel(a.shape) > 0 and a.shape[dim] <= _SORT_MAX // 2
    return (_gpu(a) and a.dtype in _SORT_DT and a.ndim >= 1 and _numel(a.shape) > 0
            and a.shape[dim] <= _SORT_MAX)


def _sort_exec(a, dim, descending, stable):
    return hip_sort(a, dim, bool(descending), bool(stable))


def _cumsum_checker(a, dim, *, dtype=None):
    if not (_gpu(a) and a.ndim >= 1 and 0 < _numel(a.shape) < 2**31):
        return False
    if a.dtype in _ROW_DT:
        return dtype is None or dtype == a.dtype
    # integer scans accumulate in int64; the output dtype is the prim's (int64, or int32 for an
    # int32 scan, which is what ltorch.cumsum(..., dtype=torch.int32) lowers to)
    return a.dtype in (torch.int32, torch.int64) and dtype in (None, torch.int64, torch.int32)


def _cumsum_exec(a, dim, *, dtype=None):
    out = dtype or a.dtype
    return hip_cumsum(a, dim, out == torch.int32)


def _emb_bwd_checker(grad, indices, num_weights, padding_idx, scale_grad_by_freq, sparse):
    if sparse or not _gpu(grad, indices) or grad.dtype not in _ROW_DT or indices.dtype not in (torch.int32, torch.int64):
        return False
    D = grad.shape[-1]
    return (D % (16 // grad.dtype.itemsize) == 0 and 0 < pyval(num_weights) < 2**31
            and _numel(indices.shape) * D == _numel(grad.shape))


def _emb_bwd_exec(grad, indices, num_weights, padding_idx, scale_grad_by_freq, sparse):
    pidx = pyval(padding_idx)
    return hip_embedding_backward(grad, indices, pyval(num_weights), -1 if pidx is None else pidx,
                                  bool(scale_grad_by_freq))


def _index_add_checker(a, indices, value, dim):
    if not (_gpu(a, indices, value) and a.ndim >= 1 and dim == 0 and a.dtype in _ROW_DT and value.dtype == a.dtype):
        return False
    if indices.dtype not in (torch.int32, torch.int64) or indices.ndim > 1 or value.ndim != a.ndim:
        return False
    D = _numel(a.shape[1:])
    return (D > 0 and D % (16 // a.dtype.itemsize) == 0 and tuple(value.shape[1:]) == tuple(a.shape[1:])
            and value.shape[0] == _numel(indices.shape))


def _index_add_exec(a, indices, value, dim):
    return hip_index_add(a, indices, value)


def _cdim(a, dim):
    d = pyval(dim)
    return d % a.ndim if a.ndim else 0


# ltorch-level claims (the torch executor would otherwise take ltorch.argsort / cumsum whole)
def _lt_topk_checker(a, k, dim=-1, largest=True, sorted=True):
    return a.ndim >= 1 and _topk_checker(a, k, _cdim(a, dim), largest, sorted)


def _lt_topk_exec(a, k, dim=-1, largest=True, sorted=True):
    return hip_topk(a, pyval(k), _cdim(a, dim), bool(pyval(largest)), bool(pyval(sorted)))


def _lt_sort_checker(a, dim=-1, descending=False, stable=False):
    return a.ndim >= 1 and _sort_checker(a, _cdim(a, dim), descending, stable)


def _lt_sort_exec(a, dim=-1, descending=False, stable=False):
    return hip_sort(a, _cdim(a, dim), bool(pyval(descending)), bool(pyval(stable)))


def _lt_argsort_exec(a, dim=-1, descending=False, stable=False):
    return hip_sort(a, _cdim(a, dim), bool(pyval(descending)), bool(pyval(stable)))[1]


def _lt_cumsum_checker(a, dim, *, dtype=None):
    if not (_gpu(a) and a.ndim >= 1 and 0 < _numel(a.shape) < 2**31):
        return False
    if a.dtype in _ROW_DT:
        return dtype is None or dtype == a.dtype
    return a.dtype in (torch.int32, torch.int64, torch.bool, torch.uint8, torch.int8, torch.int16) and \
        dtype in (None, torch.int64, torch.int32) and a.dtype in (torch.int32, torch.int64)


def _lt_cumsum_exec(a, dim, *, dtype=None):
    # torch: integer cumsum promotes to int64 unless dtype says otherwise
    return hip_cumsum(a, _cdim(a, dim), dtype == torch.int32)


def _register_all():
    from .. import torch as ltorch
    from ..core import prims as P

    ex.register_implementation(ltorch.topk, checker=_lt_topk_checker, execution_transform=_lt_topk_exec)
    ex.register_implementation(ltorch.sort, checker=_lt_sort_checker, execution_transform=_lt_sort_exec)
    ex.register_implementation(ltorch.argsort, checker=_lt_sort_checker, execution_transform=_lt_argsort_exec)
    ex.register_implementation(ltorch.cumsum, checker=_lt_cumsum_checker, execution_transform=_lt_cumsum_exec)

    ex.register_implementation(P.topk, checker=_topk_checker, execution_transform=_topk_exec)
    ex.register_implementation(P.sort, checker=_sort_checker, execution_transform=_sort_exec)
    ex.register_implementation(P.cumsum, checker=_cumsum_checker, execution_transform=_cumsum_exec)
    ex.register_implementation(P.embedding_backward, checker=_emb_bwd_checker, execution_transform=_emb_bwd_exec)
    ex.register_implementation(P.index_add, checker=_index_add_checker, execution_transform=_index_add_exec)
    from ..core.transforms import register_vjp
    from ..models import litgpt

    ex.register_implementation(ltorch.rms_norm, checker=_rms_checker, execution_transform=_rms_exec, grad_transform=_rms_grad)
    ex.register_implementation(ltorch.layer_norm, checker=_ln_checker, execution_transform=_ln_exec, grad_transform=_ln_grad)
    ex.register_implementation(ltorch._grouped_mm, checker=_gmm_checker, execution_transform=_gmm_exec)
    ex.register_implementation(ltorch.cross_entropy, checker=_ce_checker, execution_transform=_ce_exec, grad_transform=_ce_grad)
    ex.register_implementation(ltorch.scaled_dot_product_attention, checker=_sdpa_checker, execution_transform=_sdpa_exec,
                               grad_transform=_sdpa_grad)
    register_vjp(hip_qkv_rope)(_qkv_rope_vjp)
    register_vjp(hip_swiglu)(_swiglu_vjp)
    ex.register_python_lookaside(litgpt, "qkv_split_rope", qkv_split_rope_lookaside)
    ex.register_python_lookaside(litgpt, "swiglu", swiglu_lookaside)


_register_all()
