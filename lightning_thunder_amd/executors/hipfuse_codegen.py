"""hipfuse code generator: fusion region (a list of prims) -> one gfx950 HIP kernel (K1).

This replaces what nvFuser does for the reference (``thunder/executors/nvfuserex_impl.py``:
translate a region's prims into a FusionDefinition, ``:301-412``; JIT and launch, ``:526-577``).
The design is CDNA4-first rather than a translation:

* Every value of a region is described by a *map* from its dims to the dims of the
  region's iteration **domain** (the largest elementwise shape).  Broadcasts, unit-dim
  reshapes/squeezes and keepdim reductions are therefore free: they only change maps.
  External tensors are read through per-domain-dim strides that are baked into the
  source as constants (shapes are static in a trace; strides are specialised per call
  signature), so every index computation is a multiply-shift, never a runtime divide.
* **Pointwise mode** (no reduction): a grid-stride loop in which every lane owns ``VEC``
  consecutive elements of the innermost dim -> 16-byte global loads/stores (8 x bf16),
  broadcast operands along the innermost dim are loaded once as scalars.
* **Row mode** (reductions over the trailing dims, e.g. softmax / layer_norm / rms_norm
  decompositions): ``T`` in {64,128,256} lanes per row, ``256/T`` rows per workgroup.
  Each dependent reduction level is one pass over the row (recomputing its cone from
  global memory, which stays L2-resident for a row), combined with 64-lane
  ``__shfl_xor`` butterflies and (for T>64) a 4-slot LDS exchange; values that do not
  vary along the reduced dims are hoisted to row scope and computed once.
* **Column mode** (reductions over the LEADING dims, e.g. bias-grad ``sum(dy, 0)`` or LayerNorm
  dgamma/dbeta ``sum(dy * xhat, 0)``): two kernels.  The first tiles the kept (trailing) dims
  over workgroups (64 lanes x ``VEC`` columns) and the reduced rows over a second grid dim of
  ``S`` splits (4 waves stride the split's rows); it writes any full-domain outputs on the way,
  combines its 4 waves in LDS and stores one fp32/fp64/int64 partial per (split, column) to a
  workspace.  The second sums the ``S`` partials of a column in split order (deterministic, no
  atomics) and evaluates the column-shaped epilogue (casts, scaling, further elementwise).
* Low-precision values live in fp32 registers and are rounded to bf16/fp16 exactly where
  the trace produces a bf16/fp16 tensor, so results are bit-identical to op-by-op
  execution up to fp32 reassociation in reductions.
"""
from __future__ import annotations

import hashlib
import re
import math
import os
from dataclasses import dataclass, field

import torch

from ..core.prims import PrimIDs
from ..core.proxies import TensorProxy, NumberProxy, Proxy, pyval

# -----------------------------------------------------------------------------------------
# dtype tables
# -----------------------------------------------------------------------------------------
_CTYPE = {
    torch.float32: "float",
    torch.bfloat16: "float",
    torch.float16: "float",
    torch.float64: "double",
    torch.bool: "bool",
    torch.int8: "int",
    torch.int16: "int",
    torch.int32: "int",
    torch.uint8: "int",
    torch.int64: "long long",
}
_STYPE = {
    torch.float32: "float",
    torch.bfloat16: "unsigned short",
    torch.float16: "_Float16",
    torch.float64: "double",
    torch.bool: "unsigned char",
    torch.int8: "signed char",
    torch.int16: "short",
    torch.int32: "int",
    torch.uint8: "unsigned char",
    torch.int64: "long long",
}
_FLOATS = (torch.float32, torch.bfloat16, torch.float16, torch.float64)
_INTS = (torch.int8, torch.int16, torch.int32, torch.uint8, torch.int64)


def supported_dtype(dt) -> bool:
    return dt in _CTYPE


class NotFusible(Exception):
    pass


# -----------------------------------------------------------------------------------------
# Op tables: prim id -> expression builder (operands are C expressions of the compute type)
# -----------------------------------------------------------------------------------------
def _f(name, ct):
    return name + "f" if ct == "float" else name


_UNARY_FLOAT = {
    PrimIDs.EXP: "exp", PrimIDs.EXP2: "exp2", PrimIDs.EXPM1: "expm1", PrimIDs.LOG: "log", PrimIDs.LOG1P: "log1p",
    PrimIDs.LOG2: "log2", PrimIDs.LOG10: "log10", PrimIDs.SQRT: "sqrt", PrimIDs.RSQRT: "rsqrt", PrimIDs.SIN: "sin",
    PrimIDs.COS: "cos", PrimIDs.TAN: "tan", PrimIDs.SINH: "sinh", PrimIDs.COSH: "cosh", PrimIDs.TANH: "tanh",
    PrimIDs.ASIN: "asin", PrimIDs.ACOS: "acos", PrimIDs.ATAN: "atan", PrimIDs.ASINH: "asinh", PrimIDs.ACOSH: "acosh",
    PrimIDs.ATANH: "atanh", PrimIDs.ERF: "erf", PrimIDs.ERFC: "erfc", PrimIDs.ERFINV: "erfinv", PrimIDs.ERFCINV: "erfcinv",
    PrimIDs.NDTRI: "normcdfinv", PrimIDs.LGAMMA: "lgamma",
    PrimIDs.FLOOR: "floor", PrimIDs.CEIL: "ceil", PrimIDs.TRUNC: "trunc", PrimIDs.ROUND: "rint",
}
_UNARY_ANY = {PrimIDs.NEG, PrimIDs.ABS, PrimIDs.RECIPROCAL, PrimIDs.SIGN, PrimIDs.BITWISE_NOT, PrimIDs.ISFINITE,
              PrimIDs.SIGNBIT}
_BINARY = {PrimIDs.ADD: "+", PrimIDs.SUB: "-", PrimIDs.MUL: "*", PrimIDs.EQ: "==", PrimIDs.NE: "!=", PrimIDs.LT: "<",
           PrimIDs.LE: "<=", PrimIDs.GT: ">", PrimIDs.GE: ">=", PrimIDs.BITWISE_AND: "&", PrimIDs.BITWISE_OR: "|",
           PrimIDs.BITWISE_XOR: "^", PrimIDs.BITWISE_LEFT_SHIFT: "<<", PrimIDs.BITWISE_RIGHT_SHIFT: ">>"}
_BINARY_FLOAT_ONLY = {PrimIDs.DIV, PrimIDs.POW, PrimIDs.FMOD, PrimIDs.REMAINDER, PrimIDs.ATAN2, PrimIDs.COPYSIGN}
_BINARY_SPECIAL = {PrimIDs.MAXIMUM, PrimIDs.MINIMUM}
REDUCTIONS = {PrimIDs.SUM, PrimIDs.AMAX, PrimIDs.AMIN, PrimIDs.PROD, PrimIDs.VAR_MEAN}
ELEMENTWISE = set(_UNARY_FLOAT) | _UNARY_ANY | set(_BINARY) | _BINARY_FLOAT_ONLY | _BINARY_SPECIAL | {
    PrimIDs.WHERE, PrimIDs.CONVERT_ELEMENT_TYPE}
VIEWS = {PrimIDs.BROADCAST_IN_DIM, PrimIDs.RESHAPE, PrimIDs.SQUEEZE, PrimIDs.TRANSPOSE, PrimIDs.PAD, PrimIDs.SLICE}
# data movement with indirect / piecewise loads of external inputs (pointwise regions only)
GATHERS = {PrimIDs.CAT, PrimIDs.TAKE, PrimIDs.TAKE_ALONG_AXIS, PrimIDs.EMBEDDING}
# indirect stores: the region ends in one of these (a copy kernel, then the region kernel storing
# each value at its indexed position)
SCATTERS = {PrimIDs.SCATTER, PrimIDs.INDEX_PUT}
SUPPORTED = ELEMENTWISE | REDUCTIONS | VIEWS | GATHERS | SCATTERS | {PrimIDs.FULL, PrimIDs.UNIFORM_PHILOX}


def is_compute(bsym) -> bool:
    sid = bsym.sym.id
    return sid in ELEMENTWISE or sid in REDUCTIONS or sid in GATHERS or sid in SCATTERS or sid == PrimIDs.UNIFORM_PHILOX


def tensor_args(b):
    """(key, proxy) of every tensor operand of ``b``: the argument position, or (0, j) for the
    j-th tensor of a ``cat`` list.  Arg maps (``Plan.arg_maps``) are keyed the same way."""
    if b.sym.id == PrimIDs.CAT:
        return [((0, j), t) for j, t in enumerate(b.args[0]) if isinstance(t, TensorProxy)]
    return [(i, a) for i, a in enumerate(b.args) if isinstance(a, TensorProxy)]


def base_map(amap):
    """The domain-dim map inside an arg map: plain maps are tuples of domain dims (or None);
    conditional / affine / indirect loads are tagged tuples ``(kind, base, ...)``:

    * ``("pad", base, lo, value)``: input dim i walks domain dim base[i] shifted by -lo[i]; out of range -> value
    * ``("slice", base, start, step)``: input index start[i] + step[i] * i_{base[i]} (an affine load)
    * ``("gather", base, dim, idx_name, idx_map, size)``: input dim ``dim`` is indexed by the value of
      the index tensor ``idx_name`` read through ``idx_map``; the other dims through ``base``
    * ``("cat", base, dim, lo)``: one piece of a concatenation; dim ``dim`` offset by ``lo``
    * ``("reshape", base, shape)``: the input read as if reshaped to ``shape`` (row-major), whose
      dims walk ``base``
    """
    if amap and isinstance(amap[0], str):
        return amap[1] if len(amap) > 1 else ()
    return amap


def _kind(amap):
    return amap[0] if amap and isinstance(amap[0], str) else None


def _remap_amap(amap, f):
    if amap is None:
        return None
    rm = lambda mp: tuple(None if x is None else f(x) for x in mp)  # noqa: E731
    if amap and isinstance(amap[0], str) and len(amap) == 1:
        return amap
    if amap and isinstance(amap[0], str):
        if amap[0] == "gather":
            return (amap[0], rm(amap[1]), amap[2], amap[3], rm(amap[4]), amap[5])
        return (amap[0], rm(amap[1])) + tuple(amap[2:])
    return rm(amap)


def _sq(shape):
    return tuple(s for s in shape if s != 1)


# -----------------------------------------------------------------------------------------
# Planning: incremental admission of prims into a region
# -----------------------------------------------------------------------------------------
@dataclass
class Plan:
    domain: tuple | None = None
    red: int = 0  # number of trailing reduced domain dims
    colred: int = 0  # number of LEADING reduced domain dims (column mode; exclusive with red)
    has_reduction: bool = False
    has_pad: bool = False  # pads / cats / gathers (conditional or indirect loads): pointwise regions only
    nodes: list = field(default_factory=list)
    maps: dict = field(default_factory=dict)  # internal value name -> map tuple
    arg_maps: list = field(default_factory=list)  # per node: {arg position: map} for tensor args
    post: set = field(default_factory=set)  # column mode: values computed from a column reduction
    # the region's closing scatter / index_put: {"node", "out", "a", "dim", "idx", "src"} (the region
    # takes no node after it)
    scatter: dict | None = None

    def copy(self) -> "Plan":
        return Plan(self.domain, self.red, self.colred, self.has_reduction, self.has_pad, list(self.nodes),
                    dict(self.maps), [dict(m) for m in self.arg_maps], set(self.post),
                    dict(self.scatter) if self.scatter else None)

    # --- maps ----------------------------------------------------------------------------
    def _identity(self, shape):
        return tuple(i if s != 1 else None for i, s in enumerate(shape))

    def _row_map(self, shape):
        """Map a row-shaped value (its non-unit dims == the non-unit row dims, in order)."""
        if self.domain is None or self.red == 0:
            return None
        nrow = len(self.domain) - self.red
        rdims = [d for d in range(nrow) if self.domain[d] != 1]
        nz = [i for i, s in enumerate(shape) if s != 1]
        if len(nz) != len(rdims):
            return None
        m = [None] * len(shape)
        for i, d in zip(nz, rdims):
            if shape[i] != self.domain[d]:
                return None
            m[i] = d
        return tuple(m)

    def _col_map(self, shape):
        """Column mode: map a value shaped like the kept (trailing) dims."""
        if self.domain is None or self.colred == 0:
            return None
        kdims = [d for d in range(self.colred, len(self.domain)) if self.domain[d] != 1]
        nz = [i for i, s in enumerate(shape) if s != 1]
        if len(nz) != len(kdims):
            return None
        m = [None] * len(shape)
        for i, d in zip(nz, kdims):
            if shape[i] != self.domain[d]:
                return None
            m[i] = d
        return tuple(m)

    def _map_for_shape(self, shape):
        """Map for a value of ``shape`` with no other information (an all-external op)."""
        shape = tuple(shape)
        if self.domain is None:
            return "new"
        if shape == self.domain:
            return self._identity(shape)
        if self.colred:
            return self._col_map(shape)
        return self._row_map(shape)

    def covers_reduced(self, m) -> bool:
        """Column mode: does a value with map ``m`` vary along the reduced (leading) dims?"""
        return m is not None and any(x is not None and x < self.colred for x in m)

    def _internal(self, a):
        return isinstance(a, TensorProxy) and a.name in self.maps

    def has_pending(self) -> bool:
        """True while some value's index map is still unknown (see ``_add_elementwise``)."""
        return any(m is None for m in self.maps.values())

    def _resolve(self, name: str, m) -> None:
        """Assign map ``m`` to pending value ``name`` and, transitively, to its pending producers."""
        if self.maps.get(name, 0) is not None:
            return
        self.maps[name] = m
        for k, b in enumerate(self.nodes):
            if any(o.name == name for o in b.flat_outs):
                for pos, a in tensor_args(b):
                    self.arg_maps[k][pos] = m
                    if a.name in self.maps:
                        self._resolve(a.name, m)

    def _check_dtype(self, *ts):
        for t in ts:
            if isinstance(t, TensorProxy) and not supported_dtype(t.dtype):
                raise NotFusible(f"dtype {t.dtype}")

    def _set_domain(self, shape):
        self.domain = tuple(int(s) for s in shape)

    # --- admission -----------------------------------------------------------------------
    def try_add(self, bsym) -> bool:
        snapshot = self.copy()
        try:
            self._add(bsym)
            return True
        except NotFusible:
            self.__dict__.update(snapshot.__dict__)
            return False

    def _add(self, bsym):
        sid = bsym.sym.id
        if sid not in SUPPORTED:
            raise NotFusible(str(sid))
        if self.scatter is not None:
            raise NotFusible("region closed by a scatter")
        outs = [o for o in bsym.flat_outs]
        if not outs or not all(isinstance(o, TensorProxy) for o in outs):
            raise NotFusible("non-tensor output")
        self._check_dtype(*outs, *[a for a in bsym.flat_args if isinstance(a, TensorProxy)])
        for o in outs:
            if any(not isinstance(s, int) for s in o.shape):
                raise NotFusible("symbolic shape")
        am: dict[int, tuple] = {}
        if sid in ELEMENTWISE:
            self._add_elementwise(bsym, am)
        elif sid == PrimIDs.BROADCAST_IN_DIM:
            self._add_broadcast(bsym, am)
        elif sid in (PrimIDs.RESHAPE, PrimIDs.SQUEEZE):
            self._add_unit_reshape(bsym, am)
        elif sid == PrimIDs.TRANSPOSE:
            self._add_transpose(bsym, am)
        elif sid == PrimIDs.PAD:
            self._add_pad(bsym, am)
        elif sid == PrimIDs.SLICE:
            self._add_slice(bsym, am)
        elif sid == PrimIDs.CAT:
            self._add_cat(bsym, am)
        elif sid in (PrimIDs.TAKE, PrimIDs.TAKE_ALONG_AXIS, PrimIDs.EMBEDDING):
            self._add_gather(bsym, am)
        elif sid in SCATTERS:
            self._add_scatter(bsym, am)
        elif sid in REDUCTIONS:
            self._add_reduction(bsym, am)
        elif sid == PrimIDs.UNIFORM_PHILOX:
            # per-element counter-based RNG: indexed by the flat position in the domain
            out = bsym.output
            if self.domain is None:
                self._set_domain(out.shape)
            if tuple(out.shape) != self.domain:
                raise NotFusible("uniform_philox must span the iteration domain")
            self.maps[out.name] = self._identity(out.shape)
        elif sid == PrimIDs.FULL:
            out = bsym.output
            m = self._map_for_shape(out.shape)
            if m == "new":
                self._set_domain(out.shape)
                m = self._identity(out.shape)
            if m is None:
                raise NotFusible("full shape")
            self.maps[out.name] = m
        if self.colred and sid not in REDUCTIONS:
            ins = [a for a in bsym.flat_args if isinstance(a, TensorProxy) and a.name in self.post]
            if ins:
                # the column epilogue: everything downstream of a column reduction must stay column-shaped
                for o in outs:
                    if self.covers_reduced(self.maps.get(o.name)):
                        raise NotFusible("column-reduced value broadcast back over the reduced dims")
                    self.post.add(o.name)
        self.nodes.append(bsym)
        self.arg_maps.append(am)

    def _add_elementwise(self, bsym, am):
        out = bsym.output
        targs = [(i, a) for i, a in enumerate(bsym.args) if isinstance(a, TensorProxy)]
        if bsym.sym.id in _BINARY_FLOAT_ONLY and out.dtype not in _FLOATS:
            raise NotFusible("integer division/pow")
        if bsym.sym.id in _UNARY_FLOAT and out.dtype not in _FLOATS:
            raise NotFusible("float op on ints")
        internal = [a for _, a in targs if self._internal(a)]
        known = [a for a in internal if self.maps[a.name] is not None]
        if known:
            m = self.maps[known[0].name]
            for a in known[1:]:
                if self.maps[a.name] != m:
                    raise NotFusible("operands with different maps")
            for a in internal:
                if self.maps[a.name] is None:
                    self._resolve(a.name, m)
        else:
            m = self._map_for_shape(out.shape)
            if m == "new":
                self._set_domain(out.shape)
                m = self._identity(out.shape)
            if m is None:
                # e.g. a cast of a weight vector that a later broadcast maps into the domain:
                # keep it pending until a consumer fixes its map
                if any(self.maps.get(a.name, 0) is not None for a in internal):
                    raise NotFusible("shape not in domain")
                m = None
        for i, _ in targs:
            am[i] = m
        self.maps[out.name] = m

    def _add_broadcast(self, bsym, am):
        a, shape, bdims = bsym.args[0], tuple(bsym.args[1]), tuple(bsym.args[2])
        out = bsym.output
        if self._internal(a) and self.maps[a.name] is None:
            om = self._map_for_shape(shape)
            if om is None or om == "new":
                raise NotFusible("broadcast of pending value to non-domain shape")
            self._resolve(a.name, tuple(om[bdims[i]] if a.shape[i] != 1 else None for i in range(len(a.shape))))
            self.maps[out.name] = om
            return
        if self._internal(a):
            amap = self.maps[a.name]
            if self.domain is not None and shape != self.domain and tuple(a.shape) == self.domain and not self.has_reduction \
                    and len(shape) >= len(self.domain):
                # domain upgrade: the whole (pointwise) region so far is re-indexed into the larger shape
                for d, s in enumerate(self.domain):
                    if s != 1 and shape[bdims[d]] != s:
                        raise NotFusible("bad upgrade")
                def remap(mp):
                    return _remap_amap(mp, lambda x: bdims[x])
                self.maps = {k: remap(v) for k, v in self.maps.items()}
                self.arg_maps = [{k: remap(v) for k, v in d.items()} for d in self.arg_maps]
                self._set_domain(shape)
                self.maps[out.name] = self._identity(shape)
                return
            om = self._map_for_shape(shape)
            if om is None or om == "new":
                raise NotFusible("broadcast of internal to non-domain shape")
            # consistency: each non-broadcast dim of a keeps its domain dim
            for i, j in enumerate(bdims):
                if a.shape[i] != 1 and amap[i] != om[j]:
                    raise NotFusible("inconsistent broadcast map")
            self.maps[out.name] = om
            return
        om = self._map_for_shape(shape)
        if om == "new":
            self._set_domain(shape)
            om = self._identity(shape)
        if om is None:
            raise NotFusible("broadcast of external to non-domain shape")
        am[0] = tuple(om[bdims[i]] if a.shape[i] != 1 else None for i in range(len(a.shape)))
        self.maps[out.name] = om

    def _add_transpose(self, bsym, am):
        """A permutation only relabels which domain dim each dim of the value walks: the output's
        map is the input's map permuted (an external input is then read through permuted strides)."""
        a, out = bsym.args[0], bsym.output
        perm = tuple(int(p) for p in bsym.args[1])
        if self._internal(a):
            amap = self.maps[a.name]
            if amap is None:
                raise NotFusible("transpose of a value whose index map is not known yet")
            self.maps[out.name] = tuple(amap[perm[i]] for i in range(len(perm)))
            return
        om = self._map_for_shape(out.shape)
        if om == "new":
            self._set_domain(out.shape)
            om = self._identity(out.shape)
        if om is None:
            raise NotFusible("transpose of external to non-domain shape")
        amap = [None] * len(perm)
        for i, p in enumerate(perm):
            amap[p] = om[i]
        am[0] = tuple(amap)
        self.maps[out.name] = om

    def _add_pad(self, bsym, am):
        """Pad of an external input (e.g. the backward of a slice: the gradient of q / k / v placed
        into the fused qkv gradient): a conditional load — the input where the domain index falls
        inside it, the pad value elsewhere.  Pointwise regions only; no interior (dilation) padding."""
        a, pv, cfg = bsym.args[0], bsym.args[1], bsym.args[2]
        out = bsym.output
        if self._internal(a) or not isinstance(a, TensorProxy):
            raise NotFusible("pad of an internal value")
        if isinstance(pv, TensorProxy) or self.red or self.colred or self.has_reduction:
            raise NotFusible("pad in a reduction region / tensor pad value")
        cfg = tuple((int(pyval(lo)), int(pyval(hi)), int(pyval(it))) for lo, hi, it in cfg)
        if any(it != 0 or lo < 0 or hi < 0 for lo, hi, it in cfg):
            raise NotFusible("interior or negative padding")
        om = self._map_for_shape(out.shape)
        if om == "new":
            self._set_domain(out.shape)
            om = self._identity(out.shape)
        if om is None:
            raise NotFusible("pad to non-domain shape")
        # the input's dim i walks domain dim om[i] offset by -lo_i; a[i] of size 1 with lo == hi == 0 broadcasts
        am[0] = ("pad", tuple(om), tuple(lo for lo, _, _ in cfg), float(pyval(pv)))
        self.has_pad = True
        self.maps[out.name] = om

    def _ext_out_map(self, out, what):
        """Map of the output of an op on external inputs: it must span the domain (or open it)."""
        om = self._map_for_shape(out.shape)
        if om == "new":
            self._set_domain(out.shape)
            om = self._identity(out.shape)
        if om is None and not (self.red or self.colred or self.has_reduction):
            # a pointwise region: a smaller value right-aligned with the domain (what a later
            # broadcast makes of it, e.g. a position embedding added to token embeddings) is
            # evaluated per domain element
            shape, D = tuple(out.shape), self.domain
            k = len(D) - len(shape)
            if k >= 0 and all(s == 1 or s == D[k + i] for i, s in enumerate(shape)):
                om = tuple(None if s == 1 else k + i for i, s in enumerate(shape))
        if om is None:
            raise NotFusible(f"{what} to non-domain shape")
        return tuple(om)

    def _add_slice(self, bsym, am):
        """Slice of an external input (e.g. q / k / v split from a fused projection, a strided
        subsample): an affine load — base offset sum(start_i * stride_i), stride_i * step_i per dim.
        Admitted in every mode (it is a plain strided read)."""
        a, out = bsym.args[0], bsym.output
        if self._internal(a):
            raise NotFusible("slice of an internal value")
        starts = tuple(int(pyval(x)) for x in bsym.args[1])
        steps = tuple(int(pyval(x)) for x in bsym.args[3]) if len(bsym.args) > 3 and bsym.args[3] is not None \
            else (1,) * a.ndim
        om = self._ext_out_map(out, "slice")
        am[0] = ("slice", om, starts, steps)
        self.maps[out.name] = om

    def _add_cat(self, bsym, am):
        """Concatenation of external inputs: each piece is a load offset along the cat dim; per
        vector the piece is selected by the domain index (pointwise regions only)."""
        tensors, dim = list(bsym.args[0]), int(pyval(bsym.args[1]))
        out = bsym.output
        if any(self._internal(t) for t in tensors) or not all(isinstance(t, TensorProxy) for t in tensors):
            raise NotFusible("cat of an internal value")
        if self.red or self.colred or self.has_reduction:
            raise NotFusible("cat in a reduction region")
        om = self._ext_out_map(out, "cat")
        lo = 0
        for j, t in enumerate(tensors):
            am[(0, j)] = ("cat", om, dim, lo)
            lo += int(t.shape[dim])
        self.has_pad = True
        self.maps[out.name] = om

    def _add_gather(self, bsym, am):
        """Indirect loads: ``take`` (index_select), ``take_along_axis`` (gather) and ``embedding`` of
        external inputs.  The index tensor is read through its own map; out-of-range indices are
        clamped into the source (never an out-of-bounds read).  Pointwise regions only."""
        sid, out = bsym.sym.id, bsym.output
        if sid == PrimIDs.EMBEDDING:
            idx, a, dim = bsym.args[0], bsym.args[1], 0
            if bsym.kwargs.get("max_norm") is not None:
                raise NotFusible("embedding max_norm")
            apos, ipos = 1, 0
        else:
            a, idx, dim = bsym.args[0], bsym.args[1], int(pyval(bsym.args[2]))
            apos, ipos = 0, 1
        if not isinstance(a, TensorProxy) or not isinstance(idx, TensorProxy) or self._internal(a):
            raise NotFusible("gather of an internal value")
        if idx.dtype not in _INTS:
            raise NotFusible("gather index dtype")
        if self.red or self.colred or self.has_reduction:
            raise NotFusible("gather in a reduction region")
        ni = idx.ndim
        ipos_out = tuple(range(ni)) if sid in (PrimIDs.EMBEDDING, PrimIDs.TAKE_ALONG_AXIS) else \
            tuple(range(dim, dim + ni))
        if self._internal(idx) and self.domain is not None and tuple(idx.shape) == self.domain and \
                tuple(out.shape) != self.domain:
            # domain upgrade: the region so far computed the index; it continues over the gathered
            # value, each index dim walking its output dim
            def remap(mp):
                return _remap_amap(mp, lambda x: ipos_out[x])
            self.maps = {k: remap(v) for k, v in self.maps.items()}
            self.arg_maps = [{k: remap(v) for k, v in d.items()} for d in self.arg_maps]
            self._set_domain(out.shape)
        om = self._ext_out_map(out, "gather")
        if sid == PrimIDs.TAKE_ALONG_AXIS:
            imap = om
            base = tuple(None if i == dim else om[i] for i in range(a.ndim))
        else:
            if sid == PrimIDs.EMBEDDING:
                imap = om[:ni]
                base = (None, om[ni])
            else:
                imap = om[dim:dim + ni]
                base = om[:dim] + (None,) + om[dim + ni:]
        imap = tuple(None if idx.shape[i] == 1 else imap[i] for i in range(idx.ndim))
        if self._internal(idx):
            # an index computed in the region (e.g. positions from arithmetic on an iota)
            if self.maps[idx.name] is None:
                self._resolve(idx.name, imap)
            elif self.maps[idx.name] != imap:
                raise NotFusible("gather index with a different map")
        else:
            am[ipos] = imap
        am[apos] = ("gather", base, dim, idx.name, imap, int(a.shape[dim]))
        self.has_pad = True
        self.maps[out.name] = om

    def _add_scatter(self, bsym, am):
        """``scatter(a, index, src, dim)`` / ``index_put(a, (index,), values)`` (one 1-D index on dim 0,
        no accumulation) closing a pointwise region: the region runs over the index / values domain
        (src / values may be computed in it), a copy kernel first writes ``a`` into the output and the
        region kernel then stores each value at its indexed position (indices clamped into range)."""
        sid, out = bsym.sym.id, bsym.output
        if self.red or self.colred or self.has_reduction:
            raise NotFusible("scatter in a reduction region")
        if sid == PrimIDs.SCATTER:
            a, idx, src, dim = bsym.args[0], bsym.args[1], bsym.args[2], int(pyval(bsym.args[3]))
            ipos, spos = 1, 2
            dom = tuple(int(x) for x in idx.shape)
        else:
            a, indices, src, acc = bsym.args[0], bsym.args[1], bsym.args[2], bsym.args[3]
            if pyval(acc) or len(indices) != 1 or not isinstance(indices[0], TensorProxy) or indices[0].ndim != 1:
                raise NotFusible("index_put form")
            idx, dim, ipos, spos = indices[0], 0, None, 2
            if not isinstance(src, TensorProxy) or tuple(src.shape) != (int(idx.shape[0]),) + tuple(a.shape[1:]):
                raise NotFusible("index_put values shape")
            dom = tuple(int(x) for x in src.shape)
        if not isinstance(a, TensorProxy) or self._internal(a) or not isinstance(idx, TensorProxy) or \
                self._internal(idx) or idx.dtype not in _INTS:
            raise NotFusible("scatter operands")
        if any(d == 0 for d in dom) or out.dtype != a.dtype:
            raise NotFusible("scatter shape / dtype")
        if self.domain is None:
            self._set_domain(dom)
        if self.domain != dom:
            raise NotFusible("scatter domain")
        om = self._identity(dom)
        imap = om if sid == PrimIDs.SCATTER else om[:1]
        if isinstance(src, TensorProxy):
            if self._internal(src):
                if self.maps[src.name] is None:
                    self._resolve(src.name, om)
                elif self.maps[src.name] != om:
                    raise NotFusible("scatter source map")
            else:
                if src.ndim != len(dom) or any(src.shape[i] < dom[i] for i in range(len(dom))):
                    raise NotFusible("scatter source shape")
                am[spos] = tuple(None if src.shape[i] == 1 else i for i in range(len(dom)))
        if ipos is not None:
            am[ipos] = imap
        else:  # index_put's index rides in the indices tuple: read through the scatter record
            am[("idx",)] = imap
        am[0] = ("scatter_dst",)
        self.has_pad = True
        self.maps[out.name] = ("scatter_out",)
        self.scatter = dict(node=len(self.nodes), out=out.name, a=a.name, dim=dim, idx=idx.name, imap=imap,
                            src=src.name if isinstance(src, TensorProxy) else None)

    def _add_unit_reshape(self, bsym, am):
        a, out = bsym.args[0], bsym.output
        if _sq(a.shape) != _sq(out.shape):
            if bsym.sym.id == PrimIDs.RESHAPE and not self._internal(a):
                # a general reshape of an external input: read it as the reshaped tensor (a view
                # when its strides allow, else an index decomposition)
                om = self._ext_out_map(out, "reshape")
                am[0] = ("reshape", om, tuple(int(x) for x in out.shape))
                self.maps[out.name] = om
                return
            raise NotFusible("non-unit reshape")
        if self._internal(a):
            if self.maps[a.name] is None:
                raise NotFusible("unit reshape of a value whose index map is not known yet")
            amap = [x for x, s in zip(self.maps[a.name], a.shape) if s != 1]
            om, k = [], 0
            for s in out.shape:
                if s != 1:
                    om.append(amap[k])
                    k += 1
                else:
                    om.append(None)
            self.maps[out.name] = tuple(om)
            return
        om = self._map_for_shape(out.shape)
        if om == "new":
            self._set_domain(out.shape)
            om = self._identity(out.shape)
        if om is None:
            raise NotFusible("reshape of external to non-domain shape")
        onz = [x for x, s in zip(om, out.shape) if s != 1]
        amap, k = [], 0
        for s in a.shape:
            if s != 1:
                amap.append(onz[k])
                k += 1
            else:
                amap.append(None)
        am[0] = tuple(amap)
        self.maps[out.name] = om

    def _add_reduction(self, bsym, am):
        if self.has_pad:
            raise NotFusible("reduction in a region with pads")
        a = bsym.args[0]
        dims = tuple(sorted(bsym.args[1]))
        if not isinstance(a, TensorProxy) or a.ndim == 0 or not dims:
            raise NotFusible("reduction arg")
        if self._internal(a):
            if tuple(a.shape) != self.domain or self.maps[a.name] != self._identity(a.shape):
                raise NotFusible("reduction of non-domain value")
        else:
            if self.domain is None:
                self._set_domain(a.shape)
            elif tuple(a.shape) != self.domain:
                raise NotFusible("reduction of non-domain external")
            am[0] = self._identity(a.shape)
        nd, k = len(self.domain), len(dims)
        if dims != tuple(range(nd - k, nd)) or self.colred:
            if dims == tuple(range(k)) and k < nd:
                self._add_column_reduction(bsym, a, k)
                return
            raise NotFusible("non-trailing reduction")
        if self.red and self.red != k:
            raise NotFusible("different reduction dims")
        rows = math.prod(self.domain[: nd - k])
        R = math.prod(self.domain[nd - k:])
        if rows < 128 and R > 8192:
            raise NotFusible("too few rows for a row kernel")
        if bsym.sym.id == PrimIDs.SUM and bsym.kwargs.get("output_dtype") not in (None, bsym.output.dtype):
            raise NotFusible("sum output dtype")
        if bsym.sym.id == PrimIDs.PROD and a.dtype not in _FLOATS:
            raise NotFusible("int prod")
        if bsym.sym.id == PrimIDs.VAR_MEAN and a.dtype not in _FLOATS:
            raise NotFusible("int var")
        self.red = k
        self.has_reduction = True
        for o in bsym.flat_outs:
            m = self._row_map(o.shape)
            if m is None:
                raise NotFusible("reduction output shape")
            self.maps[o.name] = m

    def _add_column_reduction(self, bsym, a, k):
        if self.red:
            raise NotFusible("column reduction in a row-reduction region")
        if bsym.sym.id not in (PrimIDs.SUM, PrimIDs.AMAX, PrimIDs.AMIN, PrimIDs.PROD):
            raise NotFusible("column var_mean")
        if self.colred and self.colred != k:
            raise NotFusible("different column reduction dims")
        if self._internal(a) and a.name in self.post:
            raise NotFusible("dependent column reductions")
        if bsym.sym.id == PrimIDs.SUM and bsym.kwargs.get("output_dtype") not in (None, bsym.output.dtype):
            raise NotFusible("sum output dtype")
        if bsym.sym.id == PrimIDs.PROD and a.dtype not in _FLOATS:
            raise NotFusible("int prod")
        if self.has_reduction and not self.colred:
            raise NotFusible("mixed reductions")
        # a full-domain value already consumed by a later (column) node cannot exist: nodes before the
        # first column reduction are all full-domain or column-shaped values of externals
        self.colred = k
        self.has_reduction = True
        for o in bsym.flat_outs:
            m = self._col_map(o.shape)
            if m is None:
                raise NotFusible("column reduction output shape")
            self.maps[o.name] = m
            self.post.add(o.name)


# -----------------------------------------------------------------------------------------
# Source generation
# -----------------------------------------------------------------------------------------
_PREAMBLE = r"""
__device__ __forceinline__ float bf2f(unsigned short x) { return __builtin_bit_cast(float, ((unsigned)x) << 16); }
// f32 -> bf16 with round-to-nearest-even on the gfx950 conversion instruction (v_cvt_pk_bf16_f32:
// half the VALU of the bit-twiddling form, two values per instruction when paired)
__device__ __forceinline__ unsigned short f2bf(float f) { return __builtin_bit_cast(unsigned short, (__bf16)f); }
__device__ __forceinline__ float bfr(float f) { return (float)(__bf16)f; }
// Regions whose every output is a 16-bit float (rounded to ~4e-3 relative on the way out) use the
// hardware approximations (v_exp_f32 / v_rcp_f32, ~1 ulp of fp32) instead of the correctly rounded
// library sequences (an IEEE divide alone is ~10 VALU instructions: div_scale x2, div_fmas, div_fixup).
// e^x: the rounding of x log2(e) costs ~|x| 6e-8 relative (5e-6 at |x| = 80).
__device__ __forceinline__ float fast_expf(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
// tanh: 1 - 2 / (e^2x + 1) (-> +-1 at overflow / underflow of e^2x, NaN propagates); ~1.2e-7 absolute,
// so below |x| = 2^-4 x (1 - x^2 / 3) (truncation 2 x^5 / 15: < 2e-6 relative) keeps the relative error
// of tiny arguments
__device__ __forceinline__ float fast_tanhf(float x) {
  const float t = __builtin_fmaf(-2.f, __builtin_amdgcn_rcpf(fast_expf(2.f * x) + 1.f), 1.f);
  return fabsf(x) < 0.0625f ? x * __builtin_fmaf(x * x, -0.33333333f, 1.f) : t;
}
__device__ __forceinline__ float hfr(float f) { return (float)(_Float16)f; }
template <class T> __device__ __forceinline__ T nmax(T a, T b) { return (a != a) ? a : ((b != b) ? b : (a > b ? a : b)); }
template <class T> __device__ __forceinline__ T nmin(T a, T b) { return (a != a) ? a : ((b != b) ? b : (a < b ? a : b)); }
__device__ __forceinline__ float pymod(float a, float b) { float r = fmodf(a, b); return (r != 0.f && ((r < 0.f) != (b < 0.f))) ? r + b : r; }
__device__ __forceinline__ double pymod(double a, double b) { double r = fmod(a, b); return (r != 0.0 && ((r < 0.0) != (b < 0.0))) ? r + b : r; }
template <class T> __device__ __forceinline__ T sgn(T a) { return (a != a) ? a : (T)((a > (T)0) - (a < (T)0)); }
"""


def _lit(v, ct: str) -> str:
    if ct == "bool":
        return "true" if v else "false"
    if ct in ("int", "long long"):
        return f"({ct})({int(v)}LL)"
    v = float(v)
    if math.isnan(v):
        return "__builtin_nanf(\"\")" if ct == "float" else "__builtin_nan(\"\")"
    if math.isinf(v):
        s = "__builtin_inff()" if ct == "float" else "__builtin_inf()"
        return s if v > 0 else "(-" + s + ")"
    r = repr(v)
    if "e" not in r and "." not in r and "inf" not in r:
        r += ".0"
    return r + ("f" if ct == "float" else "")


def _rnd(dt, expr: str) -> str:
    if dt == torch.bfloat16:
        return f"bfr({expr})"
    if dt == torch.float16:
        return f"hfr({expr})"
    if dt == torch.int8:
        return f"(int)(signed char)({expr})"
    if dt == torch.uint8:
        return f"(int)(unsigned char)({expr})"
    if dt == torch.int16:
        return f"(int)(short)({expr})"
    return expr


def _load_conv(dt, x: str) -> str:
    if dt == torch.bfloat16:
        return f"bf2f({x})"
    if dt == torch.bool:
        return f"({x} != 0)"
    return f"({_CTYPE[dt]})({x})"


def _store_conv(dt, v: str) -> str:
    if dt == torch.bfloat16:
        return f"f2bf({v})"
    return f"({_STYPE[dt]})({v})"


@dataclass
class TensorArg:
    """Runtime description of one external tensor input (part of the specialisation key)."""
    shape: tuple
    strides: tuple
    dtype: torch.dtype
    align16: bool


# column-mode partial hand-off between workgroups: "coherent" (sc1 vector memory ops + s_waitcnt) or
# "fence" (__threadfence); LTA_HIPFUSE_COL_SYNC overrides (A/B hook, scripts/colred_bench.py)
COL_SYNC = os.environ.get("LTA_HIPFUSE_COL_SYNC", "coherent")
# column-mode grid: 8 waves per workgroup, ~192 workgroups (profiles/hipfuse_colred_sweep.txt), 4 rows in
# flight per wave, at most 64 row splits for a bare column reduction (the last workgroup of a column group
# reads every split's partial: more splits measured slower) and 128 when the region also stores
# full-domain outputs (its per-element work wants the occupancy).  Round 6, device-side kernel durations
# (profiles/hipfuse_roofline_gpt2_r6.txt, profiles/hipfuse_colred_sweep_r6.txt); the earlier sweeps timed
# batches of Python launches, which bound the short kernels.
COL_NW = int(os.environ.get("LTA_HIPFUSE_COL_NW", "8"))  # waves per column-mode workgroup
COL_WGS = int(os.environ.get("LTA_HIPFUSE_COL_WGS", "192"))  # target workgroups of a column-mode grid
COL_UNROLL = int(os.environ.get("LTA_HIPFUSE_COL_UNROLL", "4"))  # rows in flight per wave
COL_MAX_SPLITS = int(os.environ.get("LTA_HIPFUSE_COL_MAX_SPLITS", "64"))
COL_MAX_SPLITS_FULL = int(os.environ.get("LTA_HIPFUSE_COL_MAX_SPLITS_FULL", "128"))
# regions with full-domain outputs besides the column reduction (GPT-2's GELU backward + bias gradient:
# 80.7 -> 48 us at S = 24 -> 64, scripts/gpu_s5v.sh)
COL_WGS_FULL = int(os.environ.get("LTA_HIPFUSE_COL_WGS_FULL", "768"))


class KernelSource:
    def __init__(self, name, src, grid, block, vec, mode, extra=(), ws_bytes=0, pre=(), counters=0):
        self.name, self.src, self.grid, self.block, self.vec, self.mode = name, src, grid, block, vec, mode
        # further kernels launched after the main one with the same arguments: (name suffix, grid, block)
        self.extra = list(extra)
        # kernels launched BEFORE the main one (a scatter region's copy of its base tensor)
        self.pre = list(pre)
        # bytes of scratch the kernels share (passed as the last Args field), 0 = none
        self.ws_bytes = ws_bytes
        # column mode: uint32 arrival counters the kernel reads and resets (a persistent zeroed buffer
        # per (device, stream), passed after the workspace pointer), 0 = none
        self.counters = counters


def _contig_strides(shape):
    st, acc = [], 1
    for s in reversed(shape):
        st.append(acc)
        acc *= s
    return tuple(reversed(st))


_VALUE_ID = re.compile(r"\b([vr])_([A-Za-z_]\w*)")


def _view_strides(shape, strides, new_shape):
    """Strides of ``new_shape`` as a view of a tensor (``shape``, ``strides``), or None when the
    reshape needs a copy (the rule of ``torch.Tensor.view``: each run of merged / split dims must
    be contiguous within itself)."""
    shape, strides, new_shape = list(shape), list(strides), list(new_shape)
    if math.prod(shape) != math.prod(new_shape):
        return None
    if math.prod(shape) == 0:
        return _contig_strides(tuple(new_shape))
    res = [0] * len(new_shape)
    # drop size-1 input dims; chunk the rest into contiguous runs
    dims = [(n, s) for n, s in zip(shape, strides) if n != 1]
    vi = len(new_shape) - 1
    ci = len(dims) - 1
    while vi >= 0 or ci >= 0:
        # one chunk: input dims [cj, ci] contiguous among themselves
        if ci < 0:
            while vi >= 0:
                if new_shape[vi] != 1:
                    return None
                res[vi] = 1
                vi -= 1
            break
        cj = ci
        while cj > 0 and dims[cj - 1][1] == dims[cj][1] * dims[cj][0]:
            cj -= 1
        chunk = math.prod(n for n, _ in dims[cj:ci + 1])
        stride = dims[ci][1]
        acc = 1
        while vi >= 0 and (acc < chunk or new_shape[vi] == 1):
            res[vi] = stride * acc
            acc *= new_shape[vi]
            vi -= 1
            if acc == chunk and (vi < 0 or new_shape[vi] != 1):
                break
        if acc != chunk:
            return None
        ci = cj - 1
    return res


def _canonical_names(body: str) -> str:
    """Renames the per-value identifiers (``v_<proxy>`` / ``r_<proxy>``) by order of first use, so
    structurally identical regions (e.g. the same fusion in every transformer layer) produce the
    same source, hash to one kernel name and compile once."""
    ids: dict[str, str] = {}

    def sub(m):
        k = ids.setdefault(m.group(2), f"n{len(ids)}")
        return f"{m.group(1)}_{k}"

    return _VALUE_ID.sub(sub, body)


def generate(plan: Plan, inputs: list, outputs: list, targs: dict, kernel_prefix: str = "lta_fused",
             rng: dict | None = None) -> KernelSource:
    """``inputs``: region inputs (TensorProxy/NumberProxy), ``outputs``: TensorProxies,
    ``targs``: input name -> TensorArg for the tensor inputs at this call signature; ``rng``: number
    input name -> (device RNG state index, "seed" | "offset") for Philox arguments drawn inside a
    hipGraph capture (core/rng.py GraphRngInt: seed and base read from the state, offset relative)."""
    g = _Gen(plan, inputs, outputs, targs, rng)
    body, grid, block, vec, mode = g.build()
    body = _canonical_names(body)
    from ..core.rng import PHILOX_HIP

    src = _PREAMBLE + (PHILOX_HIP if ("philox_uniform(" in body or "philox4(" in body) else "") + body
    h = hashlib.sha1(src.encode()).hexdigest()[:16]
    name = f"{kernel_prefix}_{h}"
    src = src.replace("__KERNEL_NAME__", name)
    return KernelSource(name, src, grid, block, vec, mode, extra=g.extra, ws_bytes=g.ws_bytes, pre=g.pre,
                        counters=g.counters)


class _Gen:
    def __init__(self, plan: Plan, inputs, outputs, targs, rng=None):
        self.p = plan
        self.rng_map = dict(rng or {})
        self.n_rng = 1 + max((i for i, _ in self.rng_map.values()), default=-1)
        self.inputs = inputs
        self.outputs = outputs
        self.targs = targs
        self.D = plan.domain if plan.domain is not None else ()
        self.nd = len(self.D)
        self.red = plan.red
        self.colred = plan.colred
        self.force_scalar = False  # column epilogue kernel: every load is one element
        # every value leaving the kernel is rounded to bf16 / fp16: cheaper transcendental forms apply
        self.half_outputs = bool(outputs) and all(o.dtype in (torch.bfloat16, torch.float16) for o in outputs)
        self.extra: list = []
        self.pre: list = []
        self.ws_bytes = 0
        self.counters = 0
        self.tensor_inputs = [a for a in inputs if isinstance(a, TensorProxy)]
        self.number_inputs = [a for a in inputs if not isinstance(a, TensorProxy)]
        self.in_index = {a.name: i for i, a in enumerate(self.tensor_inputs)}
        self.num_index = {a.name: i for i, a in enumerate(self.number_inputs)}
        self.out_index = {o.name: i for i, o in enumerate(outputs)}
        self.producer = {}
        for k, b in enumerate(plan.nodes):
            for o in b.flat_outs:
                self.producer[o.name] = k
        self.lines: list[str] = []
        self.typedefs: dict[str, str] = {}
        self.flat_base4 = None  # flat index of vector lane 0 when it is a multiple of 4 (pointwise mode)

    # --- analysis ---------------------------------------------------------------------------
    def _reduced_dims(self):
        return set(range(self.nd - self.red, self.nd)) if self.red else set()

    def _analyse(self):
        """dep[name]: value varies along the loop dims; level[name]: pass after which it exists."""
        red = self._reduced_dims()
        self.dep: dict[str, bool] = {}
        self.level: dict[str, int] = {}
        self.load_dep: dict[tuple, bool] = {}
        for k, b in enumerate(self.p.nodes):
            am = self.p.arg_maps[k]
            dep, lvl = False, 0
            for i, a in tensor_args(b):
                if a.name in self.dep:
                    dep |= self.dep[a.name]
                    lvl = max(lvl, self.level[a.name])
                else:
                    m = base_map(am.get(i))
                    d = self.red == 0 or any(x in red for x in m if x is not None)
                    dep |= d
            if b.sym.id in REDUCTIONS:
                if b.sym.id == PrimIDs.VAR_MEAN:
                    v, mu = b.output
                    self.dep[mu.name], self.level[mu.name] = False, lvl + 1
                    self.dep[v.name], self.level[v.name] = False, lvl + 2
                else:
                    self.dep[b.output.name], self.level[b.output.name] = False, lvl + 1
                continue
            if b.sym.id == PrimIDs.FULL:
                dep = self.red == 0
            if b.sym.id == PrimIDs.UNIFORM_PHILOX:
                dep = True
            for o in b.flat_outs:
                self.dep[o.name] = dep if self.red else True
                self.level[o.name] = lvl

    # --- emission helpers ---------------------------------------------------------------------
    def _vtype(self, stype: str, vec: int) -> str:
        nm = "v%d_%s" % (vec, stype.replace(" ", "_"))
        if nm not in self.typedefs:
            size = {"float": 4, "double": 8, "unsigned short": 2, "_Float16": 2, "unsigned char": 1, "signed char": 1,
                    "short": 2, "int": 4, "long long": 8}[stype]
            al = min(16, size * vec)
            self.typedefs[nm] = f"typedef {stype} {nm} __attribute__((ext_vector_type({vec}), aligned({al})));"
        return nm

    def _dstrides(self, arg: TensorArg, amap) -> list:
        """Per-domain-dim element strides of an external tensor read through ``amap``."""
        steps = amap[3] if amap and amap[0] == "slice" else None
        amap = base_map(amap)
        st = [0] * self.nd
        for i, d in enumerate(amap):
            if d is not None and arg.shape[i] != 1:
                st[d] += arg.strides[i] * (steps[i] if steps else 1)
        return st

    def build(self):
        self._analyse()
        D, nd = self.D, self.nd
        numel = math.prod(D) if D else 1
        # choose VEC along the innermost domain dim
        inner = D[-1] if nd else 1
        max_item = max([t.dtype.itemsize for t in self.tensor_inputs] + [o.dtype.itemsize for o in self.outputs] + [1])
        vec = 1
        for v in ((8, 4, 2) if max_item <= 4 else (4, 2)):
            if inner % v == 0:
                vec = v
                break
        # every vector-loaded operand must keep 16B-compatible alignment; otherwise it gathers
        self.vec = vec
        big = numel >= 2**31 or any(
            sum((s - 1) * st for s, st in zip(t.shape, t.strides)) >= 2**31 for t in self.targs.values())
        self.IT = "unsigned long long" if big else "unsigned"
        if self.colred:
            return self._build_col_twopass(numel) if COL_SYNC == "twopass" else self._build_col(numel)
        if self.red:
            return self._build_row(numel)
        return self._build_pointwise(numel)

    def _decl_args(self):
        nin, nout, ns = len(self.tensor_inputs), len(self.outputs), len(self.number_inputs)
        fields = []
        if nin:
            fields.append(f"const void* in[{nin}];")
        fields.append(f"void* out[{max(nout, 1)}];")
        if ns:
            fields.append(f"double s[{ns}];")
        if self.n_rng:
            fields.append(f"const long long* rng[{self.n_rng}];")
        if self.colred:
            fields.append("void* ws;")
            if self.counters:
                fields.append("unsigned* cnt;")
        return "struct Args { " + " ".join(fields) + " };"

    def _ptr(self, t: TensorProxy, is_out: bool) -> str:
        if is_out:
            i = self.out_index[t.name]
            return f"(({_STYPE[t.dtype]}*)A.out[{i}])"
        i = self.in_index[t.name]
        return f"((const {_STYPE[t.dtype]}*)A.in[{i}])"

    def _scalar_ref(self, a, ct: str) -> str:
        if isinstance(a, Proxy) and not isinstance(a, TensorProxy):
            if a.name in self.rng_map:  # graph-safe Philox argument: seed / base from the device state
                ri, kind = self.rng_map[a.name]
                if kind == "seed":
                    return f"(({ct})rng_seed{ri})"
                return f"(({ct})(rng_base{ri} + (long long)A.s[{self.num_index[a.name]}]))"
            if a.name in self.num_index:
                return f"(({ct})A.s[{self.num_index[a.name]}])"
            v = pyval(a)
        else:
            v = a
        if ct in ("float", "double") or isinstance(v, bool):
            return _lit(v, ct if ct != "bool" or isinstance(v, bool) else "bool")
        if isinstance(v, float):
            return _lit(v, "double")
        return _lit(v, ct)

    # expression for node k at vector lane "j" ("" in row scope); refs resolved via self.ref
    def _expr(self, b, k, lane: str) -> list[tuple[str, str]]:
        """Returns [(output name, expression)] for node ``b``."""
        sid = b.sym.id
        out = b.flat_outs[0]
        ct = _CTYPE[out.dtype]

        def R(i, want_ct=None):
            a = b.args[i]
            if isinstance(a, TensorProxy):
                return self.ref(a, k, i, lane)
            return self._scalar_ref(a, want_ct or ct)

        if sid == PrimIDs.CONVERT_ELEMENT_TYPE:
            a = b.args[0]
            if not isinstance(a, TensorProxy):
                return [(out.name, _lit(pyval(a), ct))]
            x = R(0)
            if out.dtype == torch.bool:
                return [(out.name, f"({x} != 0)")]
            return [(out.name, _rnd(out.dtype, f"({ct})({x})"))]
        if sid == PrimIDs.WHERE:
            cond = R(0, "bool")
            return [(out.name, f"({cond} ? {R(1)} : {R(2)})")]
        if sid in (PrimIDs.BROADCAST_IN_DIM, PrimIDs.RESHAPE, PrimIDs.SQUEEZE, PrimIDs.TRANSPOSE, PrimIDs.PAD,
                   PrimIDs.SLICE, PrimIDs.TAKE, PrimIDs.TAKE_ALONG_AXIS):
            return [(out.name, R(0))]  # index remapping only: the arg map / conditional load does the work
        if sid == PrimIDs.EMBEDDING:
            return [(out.name, R(1))]
        if sid == PrimIDs.CAT:
            # select the piece that owns this domain index along the cat dim
            pieces = tensor_args(b)
            d = base_map(self.p.arg_maps[k][pieces[0][0]])[int(pyval(b.args[1]))]
            idx = f"(i{d}{' + j' if (lane and d == self.nd - 1) else ''})"
            e = self.ref(pieces[-1][1], k, pieces[-1][0], lane)
            for key, t in reversed(pieces[:-1]):
                hi = self.p.arg_maps[k][key][3] + int(t.shape[int(pyval(b.args[1]))])
                e = f"({idx} < {hi}u ? {self.ref(t, k, key, lane)} : {e})"
            return [(out.name, e)]
        if sid == PrimIDs.FULL:
            return [(out.name, self._scalar_ref(b.args[1], ct))]
        if sid == PrimIDs.UNIFORM_PHILOX:
            seed = self._scalar_ref(b.kwargs["seed"], "double")
            off = self._scalar_ref(b.kwargs["offset"], "double")
            lo, hi = float(pyval(b.args[1])), float(pyval(b.args[2]))
            u = f"philox_uniform((unsigned)(unsigned long long)({seed}), (unsigned long long)({off}), {self.flat_index})"
            if lo != 0.0 or hi != 1.0:
                u = f"({u} * {_lit(hi - lo, 'float')} + {_lit(lo, 'float')})"
            return [(out.name, _rnd(out.dtype, f"({ct})({u})"))]
        # operand compute type: that of the first tensor operand (prims enforce equal dtypes)
        tin = [a for _, a in tensor_args(b)]
        ict = _CTYPE[tin[0].dtype] if tin else ct
        if sid in _UNARY_FLOAT:
            if sid in (PrimIDs.TANH, PrimIDs.EXP) and ict == "float" and self.half_outputs:
                fn = "fast_tanhf" if sid == PrimIDs.TANH else "fast_expf"
                return [(out.name, _rnd(out.dtype, f"{fn}({R(0)})"))]
            return [(out.name, _rnd(out.dtype, f"{_f(_UNARY_FLOAT[sid], ict)}({R(0)})"))]
        if sid in _UNARY_ANY:
            x = R(0, ict)
            if sid == PrimIDs.NEG:
                e = f"(-{x})"
            elif sid == PrimIDs.ABS:
                e = f"{_f('fabs', ict)}({x})" if ict in ("float", "double") else f"({x} < 0 ? -{x} : {x})"
            elif sid == PrimIDs.RECIPROCAL:
                e = f"(({ict})1 / {x})"
            elif sid == PrimIDs.SIGN:
                e = f"sgn<{ict}>({x})"
            elif sid == PrimIDs.BITWISE_NOT:
                e = f"(!{x})" if ict == "bool" else f"(~{x})"
            elif sid == PrimIDs.ISFINITE:
                return [(out.name, f"isfinite({x})" if ict in ("float", "double") else "true")]
            else:  # SIGNBIT
                return [(out.name, f"signbit({x})" if ict in ("float", "double") else f"({x} < 0)")]
            return [(out.name, _rnd(out.dtype, e))]
        if sid in _BINARY:
            op = _BINARY[sid]
            x, y = R(0, ict), R(1, ict)
            e = f"({x} {op} {y})"
            if out.dtype == torch.bool:
                return [(out.name, e)]
            return [(out.name, _rnd(out.dtype, e))]
        if sid in _BINARY_SPECIAL:
            x, y = R(0, ict), R(1, ict)
            fn = "nmax" if sid == PrimIDs.MAXIMUM else "nmin"
            return [(out.name, _rnd(out.dtype, f"{fn}<{ict}>({x}, {y})"))]
        if sid in _BINARY_FLOAT_ONLY:
            x, y = R(0, ict), R(1, ict)
            if sid == PrimIDs.DIV:
                e = f"({x} / {y})"
            elif sid == PrimIDs.POW:
                e = f"{_f('pow', ict)}({x}, {y})"
            elif sid == PrimIDs.FMOD:
                e = f"{_f('fmod', ict)}({x}, {y})"
            elif sid == PrimIDs.REMAINDER:
                e = f"pymod({x}, {y})"
            elif sid == PrimIDs.ATAN2:
                e = f"{_f('atan2', ict)}({x}, {y})"
            else:
                e = f"{_f('copysign', ict)}({x}, {y})"
            return [(out.name, _rnd(out.dtype, e))]
        raise NotFusible(f"codegen: {b.sym.name}")

    # --- references -------------------------------------------------------------------------
    def ref(self, a: TensorProxy, k: int, argpos: int, lane: str) -> str:
        if a.name in self.producer:
            if lane and self.dep.get(a.name, True):
                return f"v_{a.name}[{lane}]"
            return f"r_{a.name}"
        # external load through the node's arg map
        amap = self.p.arg_maps[k][argpos]
        key = (a.name, amap)
        nm = self.load_names.get(key)
        if nm is None:
            nm = f"L{len(self.load_names)}"
            self.load_names[key] = nm
        red = self._reduced_dims()
        dep = self.red == 0 or any(x in red for x in base_map(amap) if x is not None)
        if lane and dep:
            return f"{nm}[{lane}]"
        return nm

    # --- pointwise kernel -------------------------------------------------------------------
    def _emit_nodes(self, needed: set, scope: str, emitted: set, out: list, indent: str):
        """Emit nodes whose outputs are in ``needed`` (and their cones) for ``scope`` ('vec' or 'row')."""
        order = []

        def want(name):
            if name in emitted or name not in self.producer:
                return
            k = self.producer[name]
            b = self.p.nodes[k]
            for _, a in tensor_args(b):
                if a.name in self.producer:
                    if scope == "row" or self.dep.get(a.name, True):
                        want(a.name)
                    # external loads are materialised when referenced
            if k not in order:
                order.append(k)
            for o in b.flat_outs:
                emitted.add(o.name)

        for n in needed:
            want(n)
        for k in sorted(order):
            b = self.p.nodes[k]
            if b.sym.id in REDUCTIONS:
                continue
            vec_scope = scope == "vec" and self.dep.get(b.flat_outs[0].name, True)
            if b.sym.id in SCATTERS:
                self._emit_scatter(b, k, out, indent)
                continue
            if vec_scope and b.sym.id == PrimIDs.UNIFORM_PHILOX and self.flat_base4 and self.vec % 4 == 0:
                self._emit_philox_vec(b, out, indent)
                continue
            self._materialize_loads(b, k, vec_scope, out, indent)
            exprs = self._expr(b, k, "j" if vec_scope else "")
            for name, e in exprs:
                ct = _CTYPE[[o for o in b.flat_outs if o.name == name][0].dtype]
                if vec_scope:
                    out.append(f"{indent}{ct} v_{name}[{self.vec}];")
                    out.append(f"{indent}#pragma unroll")
                    out.append(f"{indent}for (int j = 0; j < {self.vec}; ++j) v_{name}[j] = {e};")
                else:
                    out.append(f"{indent}const {ct} r_{name} = {e};")

    def _emit_philox_vec(self, b, out, indent):
        """A vector of uniforms from whole Philox blocks: the lane group's flat index is a multiple
        of 4 (``flat_base4``), so lanes 4q..4q+3 take the 4 words of one block (core/rng.py)."""
        o = b.output
        ct = _CTYPE[o.dtype]
        seed = self._scalar_ref(b.kwargs["seed"], "double")
        off = self._scalar_ref(b.kwargs["offset"], "double")
        lo, hi = float(pyval(b.args[1])), float(pyval(b.args[2]))
        V = self.vec
        out.append(f"{indent}{ct} v_{o.name}[{V}];")
        out.append(f"{indent}#pragma unroll")
        out.append(f"{indent}for (int q = 0; q < {V // 4}; ++q) {{ unsigned w[4];")
        out.append(f"{indent}  philox4((unsigned)(unsigned long long)({seed}), (unsigned long long)({off}), "
                   f"((unsigned long long)({self.flat_base4}) >> 2) + (unsigned long long)q, w);")
        u = "philox_u24(w[i])"
        if lo != 0.0 or hi != 1.0:
            u = f"({u} * {_lit(hi - lo, 'float')} + {_lit(lo, 'float')})"
        out.append(f"{indent}  #pragma unroll")
        out.append(f"{indent}  for (int i = 0; i < 4; ++i) v_{o.name}[4 * q + i] = {_rnd(o.dtype, f'({ct})({u})')}; }}")

    def _load_dep(self, amap) -> bool:
        if self.force_scalar:
            return False
        red = self._reduced_dims()
        return self.red == 0 or any(x in red for x in base_map(amap) if x is not None)

    def _materialize_loads(self, b, k, vec_scope, out, indent):
        """Emit the external loads node ``k`` references, once per scope."""
        # indirect (gather) loads last: they read the index loads of the same node
        items = sorted(tensor_args(b), key=lambda it: _kind(self.p.arg_maps[k].get(it[0])) == "gather")
        for i, a in items:
            if a.name in self.producer or _kind(self.p.arg_maps[k].get(i)) == "scatter_dst":
                continue
            amap = self.p.arg_maps[k][i]
            nm = self.load_names[(a.name, amap)]
            if self._load_dep(amap):
                assert vec_scope, "loop-varying load referenced at row scope"
                key = (nm, self._scope_id)
                if key not in self.loaded:
                    self.loaded.add(key)
                    self._emit_load(a, amap, nm, True, out, indent)
                continue
            if (nm, "row") in self.loaded:
                continue
            if vec_scope:
                key = (nm, self._scope_id)
                if key not in self.loaded:
                    self.loaded.add(key)
                    self._emit_load(a, amap, nm, False, out, indent)
            else:
                self.loaded.add((nm, "row"))
                self._emit_load(a, amap, nm, False, out, indent)

    def _emit_pad_load(self, a, amap, nm, out, indent):
        """Element-wise conditional load of a padded input (see ``Plan._add_pad``)."""
        _, base, lo, pv = amap
        ta = self.targs[a.name]
        ct = _CTYPE[a.dtype]
        ptr = self._ptr(a, False)
        V, last = self.vec, self.nd - 1
        if V > 1 and all(lo[i] % V == 0 and a.shape[i] % V == 0 for i, d in enumerate(base) if d == last):
            # every vector lies wholly inside or outside the input: one range test per vector and
            # the usual (16-byte when aligned) load at a shifted offset
            conds, st, c0 = [], [0] * self.nd, 0
            for i, d in enumerate(base):
                if d is None:
                    continue
                if f"i{d}" not in self.idx_avail:
                    raise NotFusible(f"codegen: index i{d} not available for pad load of {a.name}")
                n = int(a.shape[i])
                if lo[i] != 0 or n != self.D[d]:
                    conds.append((f"i{d} >= {lo[i]}u && " if lo[i] else "") + f"i{d} < {lo[i] + n}u")
                if n != 1:
                    st[d] += ta.strides[i]
                    c0 -= lo[i] * ta.strides[i]
            return self._emit_affine_load(a, ta, st, c0, " && ".join(conds) or None, nm, True, out, indent, fill=pv)
        conds, terms = [], []
        for i, d in enumerate(base):
            if d is None:  # a size-1 output dim: index 0, in range
                continue
            if f"i{d}" not in self.idx_avail:
                raise NotFusible(f"codegen: index i{d} not available for pad load of {a.name}")
            idx = f"((long long)i{d}{' + j' if d == last else ''} - {lo[i]}ll)"
            if lo[i] != 0 or a.shape[i] != self.D[d]:  # unpadded dims are always in range
                conds.append(f"{idx} >= 0ll && {idx} < {a.shape[i]}ll")
            terms.append(f"{idx} * {ta.strides[i]}ll")
        cond = " && ".join(conds) or "true"
        off = " + ".join(terms) or "0ll"
        out.append(f"{indent}{ct} {nm}[{V}];")
        out.append(f"{indent}#pragma unroll")
        out.append(f"{indent}for (int j = 0; j < {V}; ++j) {nm}[j] = ({cond}) ? "
                   f"{_load_conv(a.dtype, f'{ptr}[{off}]')} : {_lit(pv, ct)};")

    def _emit_load(self, a, amap, nm, vec_scope, out, indent):
        kind = _kind(amap)
        if kind in ("pad", "cat", "gather"):
            assert vec_scope, f"{kind} loads exist in pointwise regions only"
        if kind == "pad":
            return self._emit_pad_load(a, amap, nm, out, indent)
        if kind == "cat":
            return self._emit_cat_load(a, amap, nm, out, indent)
        if kind == "gather":
            return self._emit_gather_load(a, amap, nm, out, indent)
        ta = self.targs[a.name]
        if kind == "reshape":
            vs = _view_strides(ta.shape, ta.strides, amap[2])
            if vs is None:
                return self._emit_reshape_load(a, amap, nm, vec_scope, out, indent)
            ta = TensorArg(tuple(amap[2]), tuple(vs), ta.dtype, ta.align16)
            amap = amap[1]
        c0 = 0
        if kind == "slice":
            c0 = sum(int(b) * int(st) for b, st in zip(amap[2], ta.strides))
        self._emit_affine_load(a, ta, self._dstrides(ta, amap), c0, None, nm, vec_scope, out, indent)

    def _emit_affine_load(self, a, ta, st, c0, guard, nm, vec_scope, out, indent, fill=0):
        """Load ``a`` at element offset sum(i_d * st[d]) + c0 (c0 may be negative: wrap-around
        index arithmetic, only evaluated where the true offset is in range); with ``guard`` (a
        per-vector condition) the load is skipped and 0 is used where it is false."""
        ct, sty = _CTYPE[a.dtype], _STYPE[a.dtype]
        ptr = self._ptr(a, False)
        for d in range(self.nd):
            if st[d] and f"i{d}" not in self.idx_avail:
                raise NotFusible(f"codegen: index i{d} not available for load of {a.name}")
        terms = [f"(({self.IT})i{d} * {st[d]}u)" for d in range(self.nd) if st[d]]
        if c0:
            terms.append(f"({self.IT})({c0}ll)")
        off = " + ".join(terms) or "0"
        if not vec_scope:
            assert guard is None
            out.append(f"{indent}const {ct} {nm} = {_load_conv(a.dtype, f'{ptr}[{off}]')};")
            return
        V = self.vec
        last = self.nd - 1
        sl = st[last] if self.nd else 0
        zero = _lit(fill, ct)
        if sl == 0:
            ld = _load_conv(a.dtype, f'{ptr}[{off}]')
            out.append(f"{indent}const {ct} {nm}_s = {f'({guard}) ? {ld} : {zero}' if guard else ld};")
            out.append(f"{indent}{ct} {nm}[{V}];")
            out.append(f"{indent}#pragma unroll")
            out.append(f"{indent}for (int j = 0; j < {V}; ++j) {nm}[j] = {nm}_s;")
            return
        vec_ok = V > 1 and sl == 1 and ta.align16 and all(st[d] % V == 0 for d in range(last)) and c0 % V == 0
        out.append(f"{indent}{ct} {nm}[{V}];")
        if guard:
            out.append(f"{indent}#pragma unroll")
            out.append(f"{indent}for (int j = 0; j < {V}; ++j) {nm}[j] = {zero};")
            out.append(f"{indent}if ({guard})")
        if vec_ok:
            vt = self._vtype(sty, V)
            out.append(f"{indent}{{ const {vt} t = *(const {vt}*)({ptr} + ({off}));")
            out.append(f"{indent}#pragma unroll")
            out.append(f"{indent}for (int j = 0; j < {V}; ++j) {nm}[j] = {_load_conv(a.dtype, 't[j]')}; }}")
        else:
            out.append(f"{indent}{{")
            out.append(f"{indent}#pragma unroll")
            out.append(f"{indent}for (int j = 0; j < {V}; ++j) {nm}[j] = {_load_conv(a.dtype, f'{ptr}[({off}) + ({self.IT})j * {sl}u]')}; }}")

    def _emit_cat_load(self, a, amap, nm, out, indent):
        """One piece of a concatenation.  When every vector lies inside one piece (the cat dim is
        not the innermost, or the piece bounds are multiples of VEC) the piece is read with the
        usual vector load under a per-vector range guard; otherwise an element-wise conditional load."""
        _, base, dim, lo = amap
        ta = self.targs[a.name]
        d, n = base[dim], int(a.shape[dim])
        last = self.nd - 1
        if d is None:
            raise NotFusible("codegen: cat dim not in the domain")
        if d == last and (lo % self.vec or n % self.vec):
            los = tuple(lo if i == dim else 0 for i in range(a.ndim))
            return self._emit_pad_load(a, ("pad", base, los, 0.0), nm, out, indent)
        if f"i{d}" not in self.idx_avail:
            raise NotFusible(f"codegen: index i{d} not available for cat load of {a.name}")
        guard = (f"i{d} >= {lo}u && " if lo else "") + f"i{d} < {lo + n}u"
        st = self._dstrides(ta, base)
        c0 = -lo * int(ta.strides[dim]) if a.shape[dim] != 1 else 0
        if a.shape[dim] == 1:  # a one-wide piece: its stride along the cat dim never applies
            st[d] = 0
        self._emit_affine_load(a, ta, st, c0, guard, nm, True, out, indent)

    def _emit_gather_load(self, a, amap, nm, out, indent):
        """Indirect load (``take`` / ``take_along_axis`` / ``embedding``): the gathered dim's index
        comes from the index tensor's load of the same node (clamped into [0, size), negative
        indices wrap once as in Python)."""
        _, base, dim, idx_name, imap, size = amap
        ta = self.targs[a.name]
        inm = f"v_{idx_name}" if idx_name in self.producer else self.load_names[(idx_name, imap)]
        st = self._dstrides(ta, base)
        sg = int(ta.strides[dim])
        ct = _CTYPE[a.dtype]
        ptr = self._ptr(a, False)
        V, last = self.vec, self.nd - 1
        for dd in range(self.nd):
            if st[dd] and f"i{dd}" not in self.idx_avail:
                raise NotFusible(f"codegen: index i{dd} not available for gather of {a.name}")
        off = " + ".join(f"((long long)i{dd} * {st[dd]}ll)" for dd in range(self.nd) if st[dd]) or "0ll"
        clamp = (f"long long x = (long long){inm}[{{l}}]; x = x < 0 ? x + {size}ll : x; "
                 f"x = x < 0 ? 0 : (x >= {size}ll ? {size - 1}ll : x);")
        uniform = last not in [x for x in imap if x is not None]
        sl = st[last] if self.nd else 0
        vec_ok = uniform and V > 1 and sl == 1 and ta.align16 and sg % V == 0 and \
            all(st[dd] % V == 0 for dd in range(last))
        out.append(f"{indent}{ct} {nm}[{V}];")
        if vec_ok:
            vt = self._vtype(_STYPE[a.dtype], V)
            out.append(f"{indent}{{ {clamp.format(l='0')}")
            out.append(f"{indent}const {vt} t = *(const {vt}*)({ptr} + ({off}) + x * {sg}ll);")
            out.append(f"{indent}#pragma unroll")
            out.append(f"{indent}for (int j = 0; j < {V}; ++j) {nm}[j] = {_load_conv(a.dtype, 't[j]')}; }}")
            return
        out.append(f"{indent}#pragma unroll")
        out.append(f"{indent}for (int j = 0; j < {V}; ++j) {{ {clamp.format(l='j')}")
        out.append(f"{indent}  {nm}[j] = {_load_conv(a.dtype, f'{ptr}[({off}) + (long long)j * {sl}ll + x * {sg}ll]')}; }}")

    def _emit_reshape_load(self, a, amap, nm, vec_scope, out, indent):
        """Reshape of an input whose strides do not allow a view: per element, the row-major flat
        index of the reshaped value is decomposed over the input's shape (constant divisors)."""
        _, base, shape = amap
        ta = self.targs[a.name]
        ct = _CTYPE[a.dtype]
        ptr = self._ptr(a, False)
        V, last = self.vec, self.nd - 1
        cst = _contig_strides(tuple(shape))
        terms = []
        for i, d in enumerate(base):
            if d is None or shape[i] == 1:
                continue
            if f"i{d}" not in self.idx_avail:
                raise NotFusible(f"codegen: index i{d} not available for reshape load of {a.name}")
            lane = " + j" if (vec_scope and d == last) else ""
            terms.append(f"((long long)i{d}{lane}) * {cst[i]}ll")
        flat = " + ".join(terms) or "0ll"
        acst = _contig_strides(tuple(ta.shape))
        parts = []
        for i, (n, sa) in enumerate(zip(ta.shape, ta.strides)):
            if n == 1:
                continue
            parts.append(f"((f / {acst[i]}ll) % {n}ll) * {sa}ll")
        offx = " + ".join(parts) or "0ll"
        if not vec_scope:
            out.append(f"{indent}const {ct} {nm} = [&] {{ const long long f = {flat}; "
                       f"return {_load_conv(a.dtype, f'{ptr}[{offx}]')}; }}();")
            return
        out.append(f"{indent}{ct} {nm}[{V}];")
        out.append(f"{indent}#pragma unroll")
        out.append(f"{indent}for (int j = 0; j < {V}; ++j) {{ const long long f = {flat}; "
                   f"{nm}[j] = {_load_conv(a.dtype, f'{ptr}[{offx}]')}; }}")

    def _out_strides(self, o):
        """Per-domain-dim strides of a (contiguous) output plus its guard dims."""
        m = self.p.maps[o.name]
        cst = _contig_strides(tuple(o.shape))
        st = [0] * self.nd
        for i, d in enumerate(m):
            if d is not None and o.shape[i] != 1:
                st[d] = cst[i]
        guard = [d for d in range(self.nd) if self.D[d] != 1 and st[d] == 0]
        return st, guard

    def _emit_store(self, o, vec_scope, out, indent):
        st, guard = self._out_strides(o)
        ptr = self._ptr(o, True)
        val = f"v_{o.name}" if (vec_scope and self.dep.get(o.name, True)) else f"r_{o.name}"
        off = " + ".join(f"(({self.IT})i{d} * {st[d]}u)" for d in range(self.nd) if st[d]) or "0"
        last = self.nd - 1
        if vec_scope:
            g = [f"i{d} == 0" for d in guard if d != last]
        else:
            g = [f"i{d} == 0" for d in guard if d < self.nd - self.red]
        cond = " && ".join(g + (["rvalid"] if self.red else []))
        if not vec_scope:
            if self.red:
                cond = " && ".join(["lane == 0"] + ([cond] if cond else []))
            pre = f"if ({cond}) " if cond else ""
            out.append(f"{indent}{pre}{ptr}[{off}] = {_store_conv(o.dtype, val)};")
            return
        V = self.vec
        pre = f"if ({cond}) " if cond else ""
        sl = st[last] if self.nd else 0
        if self.nd and last in guard:
            # value is constant along the innermost dim: lane 0 of the vector writes it
            c2 = " && ".join(([cond] if cond else []) + [f"i{last} == 0"])
            out.append(f"{indent}if ({c2}) {ptr}[{off}] = {_store_conv(o.dtype, val + '[0]' if val.startswith('v_') else val)};")
            return
        vec_ok = V > 1 and sl == 1
        if vec_ok:
            vt = self._vtype(_STYPE[o.dtype], V)
            out.append(f"{indent}{pre}{{ {vt} t;")
            out.append(f"{indent}#pragma unroll")
            src = f"{val}[j]" if val.startswith("v_") else val
            out.append(f"{indent}for (int j = 0; j < {V}; ++j) t[j] = {_store_conv(o.dtype, src)};")
            out.append(f"{indent}*({vt}*)({ptr} + ({off})) = t; }}")
        else:
            src = f"{val}[j]" if val.startswith("v_") else val
            out.append(f"{indent}{pre}{{")
            out.append(f"{indent}#pragma unroll")
            out.append(f"{indent}for (int j = 0; j < {V}; ++j) {ptr}[({off}) + ({self.IT})j * {sl}u] = {_store_conv(o.dtype, src)}; }}")

    def _decompose(self, var: str, dims: list, out: list, indent: str):
        """i{d} = index of domain dim d from the flat index ``var`` over ``dims`` (row-major)."""
        rem = 1
        for d in reversed(dims):
            s = self.D[d]
            if s == 1:
                out.append(f"{indent}const {self.IT} i{d} = 0;")
            elif rem == 1:
                out.append(f"{indent}const {self.IT} i{d} = {var} % {s}u;")
            else:
                out.append(f"{indent}const {self.IT} i{d} = ({var} / {rem}u) % {s}u;")
            rem *= s
            self.idx_avail.add(f"i{d}")

    def _build_pointwise(self, numel):
        V, IT = self.vec, self.IT
        self.load_names, self.loaded, self._scope_id = {}, set(), "vec"
        self.idx_avail = set()
        body: list[str] = []
        nvec = numel // V
        block = 256
        grid = max(1, min((nvec + block - 1) // block, 4096 * 2))
        ind = "    "
        body.append(f"  for ({IT} v = ({IT})blockIdx.x * {block}u + threadIdx.x; v < {nvec}u; v += ({IT})gridDim.x * {block}u) {{")
        body.append(f"{ind}const {IT} e = v * {V}u;")
        self.flat_index = "((unsigned long long)e + (unsigned long long)j)"
        self.flat_base4 = "e" if V % 4 == 0 else None
        self._decompose("e", list(range(self.nd)), body, ind)
        emitted: set = set()
        # referencing builds the load-name table lazily; pre-populate by a dry run over all nodes
        for k, b in enumerate(self.p.nodes):
            for i, a in tensor_args(b):
                if a.name not in self.producer and _kind(self.p.arg_maps[k].get(i)) != "scatter_dst":
                    self.ref(a, k, i, "j")
        self._emit_nodes({o.name for o in self.outputs}, "vec", emitted, body, ind)
        sc = self.p.scatter
        for o in self.outputs:
            if sc is None or o.name != sc["out"]:
                self._emit_store(o, True, body, ind)
        body.append("  }")
        src = self._wrap(body, block)
        if sc is not None:
            src += self._scatter_copy_kernel()
        return src, (grid, 1, 1), (block, 1, 1), V, "pointwise" if sc is None else "scatter"

    # --- scatter regions -------------------------------------------------------------------------
    def _scatter_copy_kernel(self) -> str:
        """The pre-kernel of a scatter region: the base tensor copied into the (contiguous) output."""
        sc = self.p.scatter
        a = next(t for t in self.tensor_inputs if t.name == sc["a"])
        o = next(t for t in self.outputs if t.name == sc["out"])
        ta = self.targs[a.name]
        n = math.prod(ta.shape)
        IT = self.IT
        contig = tuple(ta.strides) == tuple(_contig_strides(tuple(ta.shape))) or n == 1
        nbytes = n * a.dtype.itemsize
        lines = [f'extern "C" __global__ void __launch_bounds__(256) __KERNEL_NAME___pre(Args A) {{']
        if contig and ta.align16 and nbytes % 16 == 0:
            items = nbytes // 16
            lines += [f"  const uint4* s = (const uint4*)A.in[{self.in_index[a.name]}];",
                      f"  uint4* d = (uint4*)A.out[{self.out_index[o.name]}];",
                      f"  for ({IT} v = ({IT})blockIdx.x * 256u + threadIdx.x; v < {items}u; v += ({IT})gridDim.x * 256u) d[v] = s[v];"]
        else:
            items = n
            cst = _contig_strides(tuple(ta.shape))
            terms = " + ".join(f"((e / {cst[i]}ull) % {ta.shape[i]}ull) * {ta.strides[i]}ull"
                               for i in range(len(ta.shape)) if ta.shape[i] != 1) or "0ull"
            sty = _STYPE[a.dtype]
            lines += [f"  const {sty}* s = (const {sty}*)A.in[{self.in_index[a.name]}];",
                      f"  {sty}* d = ({sty}*)A.out[{self.out_index[o.name]}];",
                      f"  for (unsigned long long e = (unsigned long long)blockIdx.x * 256ull + threadIdx.x; e < {n}ull; "
                      f"e += (unsigned long long)gridDim.x * 256ull) d[e] = s[{terms}];"]
        lines.append("}")
        self.pre = [("_pre", (max(1, min((items + 255) // 256, 8192)), 1, 1), (256, 1, 1))]
        return "\n".join(lines) + "\n"

    def _emit_scatter(self, b, k, out, indent):
        """Store the node's source values at their indexed positions of the output (clamped indices)."""
        sc = self.p.scatter
        V, last = self.vec, self.nd - 1
        o = b.output
        a = next(t for t in self.tensor_inputs if t.name == sc["a"])
        ta = self.targs[a.name]
        ct = _CTYPE[o.dtype]
        self._materialize_loads(b, k, True, out, indent)
        if b.sym.id == PrimIDs.INDEX_PUT:
            ip = next(t for t in self.tensor_inputs if t.name == sc["idx"])
            inm = "LIX"
            self._emit_load(ip, sc["imap"], inm, True, out, indent)
        else:
            inm = self.load_names[(sc["idx"], sc["imap"])]
        src = b.args[2]
        if isinstance(src, TensorProxy):
            if src.name in self.producer:
                val = f"v_{src.name}[j]"
            else:
                val = self.ref(src, k, 2, "j")
        else:
            val = self._scalar_ref(src, ct)
        shape = tuple(int(x) for x in ta.shape)
        cst = _contig_strides(shape)
        d, size = int(sc["dim"]), shape[int(sc["dim"])]
        terms = []
        for i in range(self.nd):
            if i == d:
                continue
            if self.D[i] != 1:
                terms.append(f"((long long)i{i}{' + j' if i == last else ''}) * {cst[i]}ll")
        terms.append(f"x * {cst[d]}ll")
        optr = self._ptr(o, True)
        out.append(f"{indent}#pragma unroll")
        out.append(f"{indent}for (int j = 0; j < {V}; ++j) {{ long long x = (long long){inm}[j]; "
                   f"x = x < 0 ? x + {size}ll : x; x = x < 0 ? 0 : (x >= {size}ll ? {size - 1}ll : x);")
        out.append(f"{indent}  {optr}[{' + '.join(terms)}] = {_store_conv(o.dtype, f'({ct})({val})')}; }}")

    # --- row kernel ---------------------------------------------------------------------------
    def _build_row(self, numel):
        V, IT = self.vec, self.IT
        nd, red = self.nd, self.red
        rows = math.prod(self.D[: nd - red])
        R = math.prod(self.D[nd - red:])
        nv = (R + V - 1) // V
        # lanes per row: enough to give each lane ~1-4 vectors; several rows share a wave when rows are short
        T = 1
        while T < 256 and T * 4 < nv:
            T *= 2
        if nv > T and T < 256:
            T *= 2
        T = min(T, 256)
        RPB = 256 // T
        W = max(1, T // 64)
        block = 256
        grid = (rows + RPB - 1) // RPB
        self.load_names, self.loaded = {}, set()
        self.idx_avail = set()
        self.flat_index = f"((unsigned long long)rowc * {R}ull + (unsigned long long)c + (unsigned long long)j)"
        for k, b in enumerate(self.p.nodes):
            for i, a in tensor_args(b):
                if a.name not in self.producer and _kind(self.p.arg_maps[k].get(i)) != "scatter_dst":
                    self.ref(a, k, i, "j")
        body: list[str] = []
        body.append(f"  const unsigned lane = threadIdx.x % {T}u;")
        body.append(f"  const {IT} row = ({IT})blockIdx.x * {RPB}u + threadIdx.x / {T}u;")
        body.append(f"  const bool rvalid = row < {rows}u;")
        body.append(f"  const {IT} rowc = rvalid ? row : 0u;")
        if W > 1:
            body.append("  const unsigned wv = threadIdx.x / 64u;")
        self._decompose("rowc", list(range(nd - red)), body, "  ")
        row_emitted: set = set()
        # group reductions by pass
        passes: dict[int, list] = {}
        for k, b in enumerate(self.p.nodes):
            if b.sym.id in REDUCTIONS:
                lvl = max([self.level[a.name] for a in b.args if isinstance(a, TensorProxy) and a.name in self.level] + [0])
                passes.setdefault(lvl, []).append(k)
                if b.sym.id == PrimIDs.VAR_MEAN:
                    passes.setdefault(lvl + 1, []).append(("var", k))
        redset = self._reduced_dims()

        def spans_reduced(o):  # stored over reduced dims even if its value is row-constant
            return any(d in redset for d in self.p.maps[o.name] if d is not None)

        final_outs = [o for o in self.outputs if self.dep.get(o.name, False) or spans_reduced(o)]
        final_names = {o.name for o in final_outs}
        row_outs = [o for o in self.outputs if o.name not in final_names]
        max_pass = max(passes) if passes else -1
        racc = 0
        for p in range(max_pass + 1):
            items = passes.get(p, [])
            if not items:
                continue
            self._scope_id = f"pass{p}"
            accs = []
            # row-scope prerequisites for this pass
            for it in items:
                k = it[1] if isinstance(it, tuple) else it
                b = self.p.nodes[k]
                a = b.args[0]
                need = set()
                if isinstance(a, TensorProxy) and a.name in self.producer:
                    need |= self._row_deps(a.name)
                if isinstance(it, tuple):
                    need.add(b.output[1].name)
                self._emit_row_values(need, row_emitted, body)
            for it in items:
                is_var = isinstance(it, tuple)
                k = it[1] if is_var else it
                b = self.p.nodes[k]
                a = b.args[0]
                act = "double" if a.dtype == torch.float64 else ("long long" if a.dtype in _INTS + (torch.bool,) else "float")
                sid = b.sym.id
                if sid in (PrimIDs.AMAX, PrimIDs.AMIN):
                    act = _CTYPE[a.dtype] if a.dtype != torch.bool else "int"
                    init = _lit(float("-inf") if sid == PrimIDs.AMAX else float("inf"), act) if act in ("float", "double") else (
                        "(-9223372036854775807LL - 1)" if sid == PrimIDs.AMAX and act == "long long" else
                        "9223372036854775807LL" if act == "long long" else ("(-2147483647 - 1)" if sid == PrimIDs.AMAX else "2147483647"))
                    comb = "nmax" if sid == PrimIDs.AMAX else "nmin"
                elif sid == PrimIDs.PROD:
                    init, comb = _lit(1.0, act), "*"
                else:
                    init, comb = ("0" if act == "long long" else _lit(0.0, act)), "+"
                accs.append((f"acc{racc}", act, init, comb, b, is_var))
                racc += 1
            for nm, act, init, _, _, _ in accs:
                body.append(f"  {act} {nm} = {init};")
            body.append(f"  for ({IT} c = ({IT})lane * {V}u; c < (rvalid ? {R}u : 0u); c += {T * V}u) {{")
            ind = "    "
            self.idx_avail = {x for x in self.idx_avail if int(x[1:]) < nd - red}
            self._decompose("c", list(range(nd - red, nd)), body, ind)
            emitted = set(row_emitted)
            need = set()
            for nm, act, init, comb, b, is_var in accs:
                a = b.args[0]
                if isinstance(a, TensorProxy) and a.name in self.producer:
                    need.add(a.name)
            self._emit_nodes(need, "vec", emitted, body, ind)
            for nm, act, init, comb, b, is_var in accs:
                a = b.args[0]
                k = self.p.nodes.index(b)
                x = self.ref(a, k, 0, "j")
                self._materialize_loads(b, k, True, body, ind)
                if is_var:
                    mu = f"r_{b.output[1].name}"
                    x = f"(({act})({x}) - {mu}) * (({act})({x}) - {mu})"
                else:
                    x = f"({act})({x})"
                body.append(f"{ind}#pragma unroll")
                if comb in ("+", "*"):
                    body.append(f"{ind}for (int j = 0; j < {V}; ++j) {nm} {comb}= {x};")
                else:
                    body.append(f"{ind}for (int j = 0; j < {V}; ++j) {nm} = {comb}<{act}>({nm}, {x});")
            body.append("  }")
            # cross-lane combine
            for nm, act, init, comb, b, is_var in accs:
                cf = (lambda u, v: f"{u} {comb} {v}") if comb in ("+", "*") else (lambda u, v, c=comb, t=act: f"{c}<{t}>({u}, {v})")
                for off in (32, 16, 8, 4, 2, 1):
                    if off >= T:
                        continue
                    body.append(f"  {nm} = {cf(nm, f'__shfl_xor({nm}, {off}, 64)')};")
                if W > 1:
                    body.append(f"  {{ __shared__ {act} sm_{nm}[4]; if ((threadIdx.x & 63u) == 0u) sm_{nm}[wv] = {nm}; __syncthreads();")
                    base = f"(threadIdx.x / {T}u) * {W}u"
                    expr = f"sm_{nm}[{base}]"
                    for w in range(1, W):
                        expr = cf(expr, f"sm_{nm}[{base} + {w}u]")
                    body.append(f"    {nm} = {expr}; __syncthreads(); }}")
                # finalise the reduction output(s) at row scope
                out_ct = _CTYPE[b.flat_outs[0].dtype]
                if b.sym.id == PrimIDs.VAR_MEAN:
                    corr = b.kwargs.get("correction", 1)
                    if not is_var:
                        mu = b.output[1]
                        body.append(f"  const {_CTYPE[mu.dtype]} r_{mu.name} = {_rnd(mu.dtype, f'({nm} / ({act}){R})')};")
                        row_emitted.add(mu.name)
                    else:
                        v = b.output[0]
                        body.append(f"  const {_CTYPE[v.dtype]} r_{v.name} = {_rnd(v.dtype, f'({nm} / ({act}){max(R - pyval(corr), 0)})')};")
                        row_emitted.add(v.name)
                else:
                    o = b.output
                    body.append(f"  const {out_ct} r_{o.name} = {_rnd(o.dtype, f'({out_ct})({nm})')};")
                    row_emitted.add(o.name)
        # row-scope outputs
        self._scope_id = "final_row"
        need = {o.name for o in row_outs}
        self._emit_row_values(need, row_emitted, body)
        for o in row_outs:
            self._emit_store(o, False, body, "  ")
        if final_outs:
            self._scope_id = "final"
            need = set()
            for o in final_outs:
                need |= self._row_deps(o.name)
            self._emit_row_values(need, row_emitted, body)
            body.append(f"  for ({IT} c = ({IT})lane * {V}u; c < (rvalid ? {R}u : 0u); c += {T * V}u) {{")
            ind = "    "
            self.idx_avail = {x for x in self.idx_avail if int(x[1:]) < nd - red}
            self._decompose("c", list(range(nd - red, nd)), body, ind)
            emitted = set(row_emitted)
            self._emit_nodes({o.name for o in final_outs}, "vec", emitted, body, ind)
            for o in final_outs:
                self._emit_store(o, True, body, ind)
            body.append("  }")
        return self._wrap(body, block), (grid, 1, 1), (block, 1, 1), V, f"row(T={T})"

    # --- column kernel (reductions over the leading dims) ------------------------------------
    def _red_acc(self, b):
        a = b.args[0]
        sid = b.sym.id
        act = "double" if a.dtype == torch.float64 else ("long long" if a.dtype in _INTS + (torch.bool,) else "float")
        if sid in (PrimIDs.AMAX, PrimIDs.AMIN):
            act = _CTYPE[a.dtype] if a.dtype != torch.bool else "int"
            if act == "int":
                act = "long long"
            if act in ("float", "double"):
                init = _lit(float("-inf") if sid == PrimIDs.AMAX else float("inf"), act)
            else:
                init = "(-9223372036854775807LL - 1)" if sid == PrimIDs.AMAX else "9223372036854775807LL"
            return act, init, ("nmax" if sid == PrimIDs.AMAX else "nmin")
        if sid == PrimIDs.PROD:
            return act, _lit(1.0, act), "*"
        return act, ("0" if act == "long long" else _lit(0.0, act)), "+"

    def _build_col(self, numel):
        """Column mode (leading dims reduced): ONE launch.  Workgroup (x, y) = NW waves over the rows of
        split y for the 64 V columns of group x; each lane keeps V column accumulators (16-B loads),
        the waves combine in LDS (fixed order).  With S > 1 row splits, every workgroup stores its
        fp32 partial, and the LAST workgroup of a column group to finish (agent-scope counter, reset
        by that workgroup) sums the S partials in a fixed order and runs the column epilogue: the
        result does not depend on which workgroup finished last (deterministic), and no second
        launch or host-visible state is needed.  Parity: the grid reduction of nvFuser's reduction
        scheduler behind reference thunder/executors/nvfuserex_impl.py:836-939."""
        V, IT = self.vec, self.IT
        nd, k, D = self.nd, self.colred, self.D
        C = math.prod(D[k:])
        R = math.prod(D[:k])
        NW = COL_NW  # waves per workgroup
        ncs = (C // V + 63) // 64
        red_nodes = [i for i, b in enumerate(self.p.nodes) if b.sym.id in REDUCTIONS]
        full_outs = [o for o in self.outputs if self.p.covers_reduced(self.p.maps.get(o.name))]
        # row splits: ~COL_WGS workgroups of NW waves (at most one per CU; COL_WGS_FULL when the region
        # also computes and stores full-domain outputs, e.g. an activation backward with its bias
        # gradient: that work wants the occupancy of a pointwise grid), >= 8 rows per wave, and at most
        # COL_MAX_SPLITS (the serial tail reads them all)
        wgs = COL_WGS_FULL if full_outs else COL_WGS
        S = max(1, min(-(-wgs // ncs), -(-R // (8 * NW)), COL_MAX_SPLITS_FULL if full_outs else COL_MAX_SPLITS))
        RPS = -(-R // S)
        S = -(-R // RPS)
        full_names = {o.name for o in full_outs}
        col_outs = [o for o in self.outputs if o.name not in full_names]
        self.load_names, self.loaded, self.idx_avail = {}, set(), set()
        for kk, b in enumerate(self.p.nodes):
            for i, a in tensor_args(b):
                if a.name not in self.producer:
                    self.ref(a, kk, i, "j")
        accs = []
        for n, kk in enumerate(red_nodes):
            act, init, comb = self._red_acc(self.p.nodes[kk])
            accs.append((n, kk, act, init, comb))

        def cf(comb, act, u, v):
            return f"({u} {comb} {v})" if comb in ("+", "*") else f"{comb}<{act}>({u}, {v})"

        self._scope_id = "vec"
        body: list[str] = []
        body.append("  const unsigned lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;")
        body.append(f"  const {IT} e = (({IT})blockIdx.x * 64u + lane) * {V}u;")
        body.append(f"  const bool cvalid = e < {C}u;")
        body.append(f"  const {IT} ec = cvalid ? e : 0u;")
        self._decompose("ec", list(range(k, nd)), body, "  ")
        self.flat_index = f"((unsigned long long)r * {C}ull + (unsigned long long)ec + (unsigned long long)j)"
        # a lane's V columns start at a multiple of 4 of the flat index when V and C are: Philox draws
        # then take whole 4-word blocks (one philox4 per 4 elements, as in pointwise mode)
        self.flat_base4 = f"((unsigned long long)r * {C}ull + (unsigned long long)ec)" if V % 4 == 0 and C % 4 == 0 else None
        for n, kk, act, init, comb in accs:
            body.append(f"  {act} acc{n}[{V}];")
            body.append(f"  #pragma unroll")
            body.append(f"  for (int j = 0; j < {V}; ++j) acc{n}[j] = {init};")
        body.append(f"  const {IT} r0 = ({IT})blockIdx.y * {RPS}u;")
        body.append(f"  const {IT} r1 = r0 + {RPS}u < {R}u ? r0 + {RPS}u : {R}u;")
        # unrolled: each wave keeps COL_UNROLL rows' loads in flight (the adds keep their serial order)
        body.append(f"  #pragma unroll {COL_UNROLL}")
        body.append(f"  for ({IT} r = r0 + wv; r < (cvalid ? r1 : 0u); r += {NW}u) {{")
        ind = "    "
        self._decompose("r", list(range(k)), body, ind)
        need = {o.name for o in full_outs}
        for n, kk, act, init, comb in accs:
            a = self.p.nodes[kk].args[0]
            if a.name in self.producer:
                need.add(a.name)
        emitted: set = set()
        self._emit_nodes(need, "vec", emitted, body, ind)
        for n, kk, act, init, comb in accs:
            b = self.p.nodes[kk]
            x = self.ref(b.args[0], kk, 0, "j")
            self._materialize_loads(b, kk, True, body, ind)
            body.append(f"{ind}#pragma unroll")
            if comb in ("+", "*"):
                body.append(f"{ind}for (int j = 0; j < {V}; ++j) acc{n}[j] {comb}= ({act})({x});")
            else:
                body.append(f"{ind}for (int j = 0; j < {V}; ++j) acc{n}[j] = {comb}<{act}>(acc{n}[j], ({act})({x}));")
        for o in full_outs:
            self._emit_store(o, True, body, ind)
        body.append("  }")

        def lds_combine():
            """the NW waves' accumulators -> LDS (combined in a fixed order by ``wave_total``)"""
            for n, kk, act, init, comb in accs:
                body.append(f"  #pragma unroll")
                body.append(f"  for (int j = 0; j < {V}; ++j) sm{n}[wv][lane * {V}u + j] = acc{n}[j];")
            body.append("  __syncthreads();")

        def wave_total(n, act, comb, q):
            expr = f"sm{n}[0][{q}]"
            for w in range(1, NW):
                expr = cf(comb, act, expr, f"sm{n}[{w}][{q}]")
            return expr

        for n, kk, act, init, comb in accs:
            body.append(f"  __shared__ {act} sm{n}[{NW}][{64 * V}];")
        lds_combine()
        ws_off = 0
        offs = []
        for n, kk, act, init, comb in accs:
            offs.append(ws_off)
            ws_off += S * C * 8
        _SZ = {"float": 4, "double": 8, "int": 4, "long long": 8}

        def vec_ok(act):
            # whole 16-B vectors: every row of the partial and every lane's V columns 16-B aligned
            sz = _SZ.get(act)
            return sz is not None and (V * sz) % 16 == 0 and (C * sz) % 16 == 0

        # cross-workgroup hand-off of the partials: "coherent" (default) writes and reads them with
        # agent-coherent (sc1) vector memory operations and orders them with s_waitcnt before the
        # arrival counter; "fence" uses __threadfence() (an agent-scope fence writes back / invalidates
        # the whole L2 of the XCD: measured ~40 us per [8192, 1024] sum with 256 workgroups)
        coherent = COL_SYNC == "coherent" and ws_off < 2**31
        if S > 1:
            if coherent:
                self.typedefs["v4_u32"] = "typedef unsigned v4_u32 __attribute__((ext_vector_type(4)));"
                body.append("  const __amdgpu_buffer_rsrc_t wsr = __builtin_amdgcn_make_buffer_rsrc(A.ws, (short)0, "
                            "0x7fffffff, 0x00020000);")
            # this split's partial (wave 0: the fixed-order wave combination)
            body.append("  if (wv == 0u && cvalid) {")
            for (n, kk, act, init, comb), off in zip(accs, offs):
                body.append(f"    {act}* ws{n} = ({act}*)((char*)A.ws + {off}ull) + ({IT})blockIdx.y * {C}u;")
                if vec_ok(act):
                    vt = self._vtype(act, V)
                    body.append(f"    {vt} pv{n};")
                    body.append(f"    #pragma unroll")
                    body.append(f"    for (int j = 0; j < {V}; ++j) pv{n}[j] = {wave_total(n, act, comb, f'lane * {V}u + j')};")
                    if coherent:
                        sz = _SZ[act]
                        body.append(f"    const v4_u32* pu{n} = (const v4_u32*)&pv{n};")
                        body.append(f"    const unsigned bo{n} = {off}u + ((unsigned)blockIdx.y * {C}u + (unsigned)e) * {sz}u;")
                        for c in range(V * sz // 16):
                            body.append(f"    __builtin_amdgcn_raw_buffer_store_b128(pu{n}[{c}], wsr, bo{n} + {16 * c}u, 0, 16);")
                    else:
                        body.append(f"    *({vt}*)(ws{n} + e) = pv{n};")
                else:
                    body.append(f"    #pragma unroll")
                    if coherent:
                        body.append(f"    for (int j = 0; j < {V}; ++j) __hip_atomic_store(ws{n} + e + j, "
                                    f"({act})({wave_total(n, act, comb, f'lane * {V}u + j')}), __ATOMIC_RELAXED, "
                                    "__HIP_MEMORY_SCOPE_AGENT);")
                    else:
                        body.append(f"    for (int j = 0; j < {V}; ++j) ws{n}[e + j] = {wave_total(n, act, comb, f'lane * {V}u + j')};")
            body.append("  }")
            # count this split in once its partial is at the coherence point; only the last workgroup of
            # the column group goes on
            if coherent:
                body.append('  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");')
            else:
                body.append("  __threadfence();")
            body.append("  __shared__ unsigned last;")
            body.append("  __syncthreads();")
            body.append("  if (threadIdx.x == 0u) last = atomicAdd(A.cnt + blockIdx.x, 1u) == "
                        f"{S - 1}u ? 1u : 0u;")
            body.append("  __syncthreads();")
            body.append("  if (last == 0u) return;")
            if not coherent:
                body.append("  __threadfence();  // acquire: the other splits' partials")
            body.append("  if (threadIdx.x == 0u) __hip_atomic_store(A.cnt + blockIdx.x, 0u, __ATOMIC_RELAXED, "
                        "__HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch")
            # wave w sums splits w, w + NW, ... (8 splits' loads in flight), then the waves combine in LDS
            for (n, kk, act, init, comb), off in zip(accs, offs):
                body.append(f"  const {act}* pw{n} = (const {act}*)((const char*)A.ws + {off}ull);")
                body.append(f"  #pragma unroll")
                body.append(f"  for (int j = 0; j < {V}; ++j) acc{n}[j] = {init};")
                body.append("  #pragma unroll 8")
                body.append(f"  for (unsigned sp = wv; sp < (cvalid ? {S}u : 0u); sp += {NW}u) {{")
                if vec_ok(act) and coherent:
                    sz = _SZ[act]
                    nch = V * sz // 16
                    body.append(f"    v4_u32 qr{n}[{nch}];")
                    body.append(f"    const unsigned bq{n} = {off}u + (sp * {C}u + (unsigned)e) * {sz}u;")
                    for c in range(nch):
                        body.append(f"    qr{n}[{c}] = __builtin_amdgcn_raw_buffer_load_b128(wsr, bq{n} + {16 * c}u, 0, 16);")
                    body.append(f"    const {act}* q{n} = (const {act}*)qr{n};")
                elif vec_ok(act):
                    vt = self._vtype(act, V)
                    body.append(f"    const {vt} q{n} = *(const {vt}*)(pw{n} + ({IT})sp * {C}u + e);")
                elif coherent:
                    body.append(f"    {act} q{n}[{V}];")
                    body.append(f"    #pragma unroll")
                    body.append(f"    for (int j = 0; j < {V}; ++j) q{n}[j] = __hip_atomic_load(pw{n} + ({IT})sp * {C}u + e + j, "
                                "__ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);")
                else:
                    body.append(f"    const {act}* q{n} = pw{n} + ({IT})sp * {C}u + e;")
                body.append(f"    #pragma unroll")
                body.append(f"    for (int j = 0; j < {V}; ++j) acc{n}[j] = {cf(comb, act, f'acc{n}[j]', f'q{n}[j]')};")
                body.append("  }")
            body.append("  __syncthreads();")
            lds_combine()
        # column epilogue: thread t takes columns t, t + 64 NW, ... of the group (one element each)
        self.flat_base4 = None
        self.force_scalar = True
        self._scope_id = "fin"
        self.idx_avail = set()
        body.append(f"  for (unsigned qc = threadIdx.x; qc < {64 * V}u; qc += {64 * NW}u) {{")
        ind = "    "
        body.append(f"{ind}const {IT} ecol = ({IT})blockIdx.x * {64 * V}u + qc;")
        body.append(f"{ind}if (ecol >= {C}u) break;")
        fin: list[str] = []
        self._decompose("ecol", list(range(k, nd)), fin, ind)
        done: set = set()
        for n, kk, act, init, comb in accs:
            o = self.p.nodes[kk].output
            out_ct = _CTYPE[o.dtype]
            fin.append(f"{ind}const {act} t{n} = {wave_total(n, act, comb, 'qc')};")
            fin.append(f"{ind}const {out_ct} r_{o.name} = {_rnd(o.dtype, f'({out_ct})(t{n})')};")
            done.add(o.name)
        self._emit_nodes({o.name for o in col_outs}, "row", done, fin, ind)
        for o in col_outs:
            st, _ = self._out_strides(o)
            off = " + ".join(f"(({IT})i{d} * {st[d]}u)" for d in range(nd) if st[d]) or "0"
            fin.append(f"{ind}{self._ptr(o, True)}[{off}] = {_store_conv(o.dtype, f'r_{o.name}')};")
        body += fin
        body.append("  }")
        self.force_scalar = False
        self.extra = []
        # the Args block always carries both pointers (S == 1 never touches them)
        self.ws_bytes = ws_off
        self.counters = ncs
        return self._wrap(body, 64 * NW), (ncs, S, 1), (64 * NW, 1, 1), V, f"col(S={S})"

    def _build_col_twopass(self, numel):
        V, IT = self.vec, self.IT
        nd, k, D = self.nd, self.colred, self.D
        C = math.prod(D[k:])
        R = math.prod(D[:k])
        ncs = (C // V + 63) // 64
        # row splits: enough workgroups for ~2 per CU, >= 32 rows (8 per wave) per split
        S = max(1, min(-(-512 // ncs), -(-R // 32)))
        RPS = -(-R // S)
        S = -(-R // RPS)
        post = self.p.post
        red_nodes = [i for i, b in enumerate(self.p.nodes) if b.sym.id in REDUCTIONS]
        full_outs = [o for o in self.outputs if self.p.covers_reduced(self.p.maps.get(o.name))]
        full_names = {o.name for o in full_outs}
        col_outs = [o for o in self.outputs if o.name not in full_names]
        self.load_names, self.loaded, self.idx_avail = {}, set(), set()
        for kk, b in enumerate(self.p.nodes):
            for i, a in tensor_args(b):
                if a.name not in self.producer:
                    self.ref(a, kk, i, "j")
        accs = []
        for n, kk in enumerate(red_nodes):
            act, init, comb = self._red_acc(self.p.nodes[kk])
            accs.append((n, kk, act, init, comb))

        def cf(comb, act, u, v):
            return f"({u} {comb} {v})" if comb in ("+", "*") else f"{comb}<{act}>({u}, {v})"

        # ---- kernel 1: partial reductions (+ full-domain outputs) ----
        self._scope_id = "vec"
        body: list[str] = []
        body.append("  const unsigned lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;")
        body.append(f"  const {IT} e = (({IT})blockIdx.x * 64u + lane) * {V}u;")
        body.append(f"  const bool cvalid = e < {C}u;")
        body.append(f"  const {IT} ec = cvalid ? e : 0u;")
        self._decompose("ec", list(range(k, nd)), body, "  ")
        self.flat_index = f"((unsigned long long)r * {C}ull + (unsigned long long)ec + (unsigned long long)j)"
        # a lane's V columns start at a multiple of 4 of the flat index when V and C are: Philox draws
        # then take whole 4-word blocks (one philox4 per 4 elements, as in pointwise mode)
        self.flat_base4 = f"((unsigned long long)r * {C}ull + (unsigned long long)ec)" if V % 4 == 0 and C % 4 == 0 else None
        for n, kk, act, init, comb in accs:
            body.append(f"  {act} acc{n}[{V}];")
            body.append(f"  #pragma unroll")
            body.append(f"  for (int j = 0; j < {V}; ++j) acc{n}[j] = {init};")
        body.append(f"  const {IT} r0 = ({IT})blockIdx.y * {RPS}u;")
        body.append(f"  const {IT} r1 = r0 + {RPS}u < {R}u ? r0 + {RPS}u : {R}u;")
        # unrolled: each wave keeps 4 rows' loads in flight (the adds keep their serial order)
        body.append("  #pragma unroll 4")
        body.append(f"  for ({IT} r = r0 + wv; r < (cvalid ? r1 : 0u); r += 4u) {{")
        ind = "    "
        self._decompose("r", list(range(k)), body, ind)
        need = {o.name for o in full_outs}
        for n, kk, act, init, comb in accs:
            a = self.p.nodes[kk].args[0]
            if a.name in self.producer:
                need.add(a.name)
        emitted: set = set()
        self._emit_nodes(need, "vec", emitted, body, ind)
        for n, kk, act, init, comb in accs:
            b = self.p.nodes[kk]
            x = self.ref(b.args[0], kk, 0, "j")
            self._materialize_loads(b, kk, True, body, ind)
            body.append(f"{ind}#pragma unroll")
            if comb in ("+", "*"):
                body.append(f"{ind}for (int j = 0; j < {V}; ++j) acc{n}[j] {comb}= ({act})({x});")
            else:
                body.append(f"{ind}for (int j = 0; j < {V}; ++j) acc{n}[j] = {comb}<{act}>(acc{n}[j], ({act})({x}));")
        for o in full_outs:
            self._emit_store(o, True, body, ind)
        body.append("  }")
        # combine the 4 waves (fixed order) and store this split's partial
        ws_off = 0
        offs = []
        for n, kk, act, init, comb in accs:
            offs.append(ws_off)
            ws_off += S * C * 8
            body.append(f"  __shared__ {act} sm{n}[4][{64 * V}];")
            body.append(f"  #pragma unroll")
            body.append(f"  for (int j = 0; j < {V}; ++j) sm{n}[wv][lane * {V}u + j] = acc{n}[j];")
        body.append("  __syncthreads();")
        body.append("  if (wv == 0u && cvalid) {")
        for (n, kk, act, init, comb), off in zip(accs, offs):
            body.append(f"    {act}* ws{n} = ({act}*)((char*)A.ws + {off}ull) + ({IT})blockIdx.y * {C}u;")
            body.append(f"    #pragma unroll")
            body.append(f"    for (int j = 0; j < {V}; ++j) {{")
            expr = f"sm{n}[0][lane * {V}u + j]"
            for w in range(1, 4):
                expr = cf(comb, act, expr, f"sm{n}[{w}][lane * {V}u + j]")
            body.append(f"      ws{n}[e + j] = {expr};")
            body.append("    }")
        body.append("  }")
        main = self._wrap(body, 256)

        # ---- kernel 2: combine the splits, column epilogue ----
        self.force_scalar = True
        self._scope_id = "fin"
        self.idx_avail = set()
        fin: list[str] = []
        # 4 waves per 64 columns: wave w sums splits w, w+4, ... (a 4x shorter serial chain), then
        # the 4 partial sums are combined in a fixed order (deterministic)
        fin.append(f"  const unsigned part = threadIdx.x >> 6, cl = threadIdx.x & 63u;")
        fin.append(f"  const {IT} e0 = ({IT})blockIdx.x * 64u + cl;")
        fin.append(f"  const bool ok = e0 < {C}u;")
        fin.append(f"  const {IT} e = ok ? e0 : 0u;")
        for (n, kk, act, init, comb), off in zip(accs, offs):
            fin.append(f"  const {act}* ws{n} = (const {act}*)((const char*)A.ws + {off}ull);")
            fin.append(f"  {act} t{n} = {init};")
            # unrolled: 8 partial loads in flight per thread (same serial combine order, deterministic)
            fin.append("  #pragma unroll 8")
            fin.append(f"  for (unsigned s = part; s < {S}u; s += 4u) t{n} = {cf(comb, act, f't{n}', f'ws{n}[({IT})s * {C}u + e]')};")
            fin.append(f"  __shared__ {act} sf{n}[4][64];")
            fin.append(f"  sf{n}[part][cl] = t{n};")
        fin.append("  __syncthreads();")
        fin.append("  if (part != 0u || !ok) return;")
        self._decompose("e", list(range(k, nd)), fin, "  ")
        done: set = set()
        for (n, kk, act, init, comb), off in zip(accs, offs):
            b = self.p.nodes[kk]
            o = b.output
            tot = f"sf{n}[0][cl]"
            for w in range(1, 4):
                tot = cf(comb, act, tot, f"sf{n}[{w}][cl]")
            fin.append(f"  t{n} = {tot};")
            out_ct = _CTYPE[o.dtype]
            fin.append(f"  const {out_ct} r_{o.name} = {_rnd(o.dtype, f'({out_ct})(t{n})')};")
            done.add(o.name)
        self._emit_nodes({o.name for o in col_outs}, "row", done, fin, "  ")
        for o in col_outs:
            st, _ = self._out_strides(o)
            off = " + ".join(f"(({IT})i{d} * {st[d]}u)" for d in range(nd) if st[d]) or "0"
            fin.append(f"  {self._ptr(o, True)}[{off}] = {_store_conv(o.dtype, f'r_{o.name}')};")
        self.force_scalar = False
        fin_src = "\n".join([f'extern "C" __global__ void __launch_bounds__(256) __KERNEL_NAME___fin(Args A) {{'] + fin
                            + ["}"]) + "\n"
        self.extra = [("_fin", ((C + 63) // 64, 1, 1), (256, 1, 1))]
        self.ws_bytes = ws_off
        return main + fin_src, (ncs, S, 1), (256, 1, 1), V, f"col(S={S})"

    def _row_deps(self, name) -> set:
        """Row-scope (loop-invariant) internal values in the cone of ``name``."""
        res, seen = set(), set()

        def walk(n):
            if n in seen or n not in self.producer:
                return
            seen.add(n)
            if not self.dep.get(n, True):
                res.add(n)
                return
            b = self.p.nodes[self.producer[n]]
            for _, a in tensor_args(b):
                walk(a.name)

        walk(name)
        return res

    def _emit_row_values(self, need: set, row_emitted: set, body: list):
        prev = self._scope_id
        self._scope_id = "row"
        need = {n for n in need if n not in row_emitted}
        if need:
            # the row cone can contain reductions that are already finalised (in row_emitted)
            self._emit_nodes(need, "row", row_emitted, body, "  ")
        self._scope_id = prev

    def _wrap(self, body, block):
        head = [self._decl_args(), *self.typedefs.values(),
                f'extern "C" __global__ void __launch_bounds__({block}) __KERNEL_NAME__(Args A) {{']
        # graph-safe Philox state: read once per thread (the outputs' stores could alias it for the compiler)
        for ri in range(self.n_rng):
            head.append(f"  const long long rng_seed{ri} = A.rng[{ri}][0], rng_base{ri} = A.rng[{ri}][1];")
        return "\n".join(head + body + ["}"]) + "\n"
