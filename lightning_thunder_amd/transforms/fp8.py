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

from ..core.prims import OpTags
from ..core.proxies import TensorProxy
from ..core.symbol import Symbol
from ..core.trace import from_trace, tracectx, TraceProvenance
from ..core.transform_common import Transform


def _fp8_linear_meta(x, w, bias=None, key=None, slots=None):
    return TensorProxy(like=x, shape=tuple(x.shape[:-1]) + (w.shape[0],))


# key/slots: None for current scaling; else the delayed-scaling state key and the (x, w, dy) slots
fp8_linear = Symbol("fp8_linear", _fp8_linear_meta, id="lta.fp8_linear", is_prim=True)

# advances the delayed-scaling amax histories (first op of every forward)
fp8_delayed_update = Symbol("fp8_delayed_update", lambda key: None, id="lta.fp8_delayed_update", is_prim=True,
                            tags=(OpTags.DONT_DCE,))


def eligible(x, w, bias=None, key=None, slots=None) -> bool:
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
    """``recipe``: ``"current"`` (per-tensor current scaling: one amax pass per cast), ``"delayed"``
    or a :class:`~lightning_thunder_amd.ops.fp8.DelayedScaling` (amax history, scales from earlier
    steps, amax all-reduced over the data-parallel group; reference TE ``DelayedScaling``), or
    ``"mxfp8"`` / :class:`~lightning_thunder_amd.ops.fp8.MXFP8BlockScaling` (E8M0 scale per 32
    elements of each GEMM's reduction dim, on the block-scaled MFMA; reference TE ``MXFP8BlockScaling``),
    or ``"mxfp4"`` / :class:`~lightning_thunder_amd.ops.fp8.MXFP4BlockScaling` (forward GEMM in
    MXFP4, backward in MXFP8; the counterpart of TE ``NVFP4BlockScaling``)."""

    def __init__(self, recipe="current", amax_history_len: int = 16, skip: tuple[str, ...] = ()):
        from ..ops.fp8 import DelayedScaling, MXFP8BlockScaling, MXFP4BlockScaling

        if recipe == "delayed":
            recipe = DelayedScaling(amax_history_len=amax_history_len)
        elif recipe == "mxfp8":
            recipe = MXFP8BlockScaling()
        elif recipe == "mxfp4":
            recipe = MXFP4BlockScaling()
        if not (recipe == "current" or isinstance(recipe, (DelayedScaling, MXFP8BlockScaling, MXFP4BlockScaling))):
            raise ValueError(f"unknown FP8 recipe {recipe!r}")
        self.recipe = recipe
        self.amax_history_len = amax_history_len
        self.skip = skip
        self.n_converted = 0
        self.state_key = None

    def transform_traces_pre_prologue(self, prologue_trace, computation_trace, epilogue_trace, **kwargs):
        from ..executors import hipex  # noqa: F401  (registers fp8_linear's implementation + VJP)

        new = from_trace(computation_trace)
        new.bound_symbols = []
        new.scopes = [new.bound_symbols]
        from ..ops.fp8 import MXFP8BlockScaling, MXFP4BlockScaling

        swap: dict = {}
        n = 0
        mx = "mxfp8" if isinstance(self.recipe, MXFP8BlockScaling) else (
            "mxfp4" if isinstance(self.recipe, MXFP4BlockScaling) else None)
        delayed = self.recipe != "current" and not mx
        slots: dict = {}  # ("x"|"w", proxy name) / ("dy", site) -> history slot; siblings reading one x share it
        key = None
        if delayed:
            from ..ops.fp8 import new_delayed_state

            key = new_delayed_state(self.recipe, 0)  # slot count set once the program is scanned

        def slot(k):
            return slots.setdefault(k, len(slots))

        def convert(nb):
            """fp8_linear bound to the linear's own output proxy, or None when not eligible."""
            nonlocal n
            if nb.sym.name != "linear" or len(nb.args) < 2:
                return None
            x, w = nb.args[0], nb.args[1]
            bias = nb.args[2] if len(nb.args) > 2 else nb.kwargs.get("bias")
            if not eligible(x, w, bias) or any(s in w.name for s in self.skip):
                return None
            if delayed:
                args = (x, w, bias, key, (slot(("x", x.name)), slot(("w", w.name)), slot(("dy", n))))
            elif mx:
                args = (x, w, bias, mx)
            else:
                args = (x, w, bias)
            n += 1
            return fp8_linear.bind(*args, output=nb.output)

        def rewrite_region(b):
            """Activation-checkpointed regions keep their linears as subsymbols of the checkpoint
            call: convert those too (the backward's recompute then replays fp8_linear)."""
            subs = []
            changed = False
            for sb in b.subsymbols:
                cv = convert(sb)
                if cv is None and sb.sym.name == "checkpoint":
                    cv = rewrite_region(sb)
                subs.append(cv if cv is not None else sb)
                changed |= cv is not None
            return b.from_bsym(subsymbols=subs) if changed else None

        with tracectx(new):
            for b in computation_trace.bound_symbols:
                nb = b.swap_proxies(swap, skip_output=True)
                cv = convert(nb)
                if cv is None and nb.sym.name == "checkpoint":
                    cv = rewrite_region(nb)
                new.bound_symbols.append(cv if cv is not None else nb)
        self.n_converted = n
        if not n:
            if key is not None:
                from ..ops.fp8 import release_delayed_state

                release_delayed_state(key)
            return prologue_trace, computation_trace, epilogue_trace
        if delayed:
            from ..ops.fp8 import delayed_state

            st = delayed_state(key)
            st.resize(len(slots))
            self.state_key = key
            upd = fp8_delayed_update.bind(key, output=None)
            new.bound_symbols.insert(0, upd)
        what = "current scaling" if self.recipe == "current" else f"{self.recipe!r}"
        new.set_provenance(TraceProvenance(f"FP8 linear ({n} linears -> e4m3/e5m2 GEMMs, {what})"))
        return prologue_trace, new, epilogue_trace
