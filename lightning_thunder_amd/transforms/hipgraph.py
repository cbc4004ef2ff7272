"""HipGraphTransform: capture launch-bound regions of execution traces in hipGraphs.

Reference parity: ``thunder/transforms/cudagraph.py`` (``CUDAGraphTransform``: a
post-optimization transform that fuses maximal capturable regions into
``CUDAGraphRunner`` callables with a graph cache keyed on input metadata, static input
buffers and graph replay) and the ``reduce-overhead`` plugin.

MI355X design:
* ``torch.cuda.CUDAGraph`` is a hipGraph on ROCm; every launch inside a region — hipBLASLt
  GEMMs, the hand-written HIP kernels (ctypes launches on the current stream) and
  hipfuse's ``hipModuleLaunchKernel`` launches — is captured.
* Framework-owned inputs are not copied into separate static buffers: the captured call's
  tensors become the graph's static inputs and on replay an input is copied only if it lives
  at a different address.  Parameters/buffers never move and the backward consumes the
  forward graph's outputs (graph pool, fixed addresses), so a training step copies only the
  token batch and the incoming loss gradient.  Tensors the *caller* passed in (arguments of
  a forward/computation trace that are not parameters/buffers) are cloned into private
  static buffers at capture: the caller may keep using its tensor (e.g. ``generate`` keeps
  every sampled token), and later replays must not write into it.
* One private memory pool is shared by every graph of the transform (fw and bw graphs
  replay in capture order), so graphed memory ~= eager peak.
* First call per signature runs eagerly (warm-up: lazy library init, hiprtc compiles of
  hipfuse kernels, allocator growth), the second captures, later calls replay.

Outputs of a graphed region are the graph's static tensors: they are overwritten by the
next replay of the same region (same contract as the reference's runner).  Pass
``copy_outputs=True`` to return clones instead.
"""
from __future__ import annotations

import threading

import torch

from ..core.prims import PrimIDs
from ..core.proxies import TensorProxy, Proxy
from ..core.symbol import Symbol, BoundSymbol
from ..core.trace import TraceCtx, from_trace, TraceProvenance, tracectx
from ..core.transform_common import Transform

_NOT_CAPTURABLE_IDS = {PrimIDs.RETURN, PrimIDs.DEL, PrimIDs.COMMENT, PrimIDs.ITEM}


def _is_unpack(b) -> bool:
    return isinstance(b.sym.name, str) and b.sym.name.startswith("unpack")


def default_capturable(bsym: BoundSymbol, *, capture_collectives: bool = False) -> bool:
    if bsym.sym.id in _NOT_CAPTURABLE_IDS or _is_unpack(bsym):
        return False
    if not capture_collectives and (getattr(bsym.sym, "module", None) == "dist_prims"
                                    or (isinstance(bsym.sym.id, str) and bsym.sym.id.startswith("dist."))):
        return False
    for p in bsym.flat_proxy_outs:
        if not isinstance(p, TensorProxy):
            return False  # host values (item(), shapes) force a sync
        if p.device.type != "cuda":
            return False
    for p in bsym.flat_proxy_args:
        if isinstance(p, TensorProxy) and p.device.type != "cuda":
            return False
    return True


class HipGraphRunner:
    """Graph cache for one region (reference ``CUDAGraphRunner``)."""

    def __init__(self, fn, name: str, pool_owner: "HipGraphTransform", copy_outputs: bool = False,
                 private_inputs: tuple = (), mutated_inputs: tuple = ()):
        self.fn = fn
        self.private_inputs = private_inputs
        # caller-owned inputs the graph updates in place (KV caches handed in per call): captured on
        # the caller's storage, not a private clone; a later call with other storage copies in and back
        self.mutated_inputs = mutated_inputs
        self.name = name
        self.owner = pool_owner
        self.copy_outputs = copy_outputs
        self.entries: dict = {}
        self._lock = threading.Lock()
        self.replays = 0
        self.captures = 0

    @staticmethod
    def _key(args):
        k = []
        for a in args:
            if isinstance(a, torch.Tensor):
                k.append((tuple(a.shape), tuple(a.stride()), a.dtype, a.device))
            else:
                k.append(("py", a))
        return tuple(k)

    def __call__(self, *args):
        key = self._key(args)
        e = self.entries.get(key)
        if e is None:
            self.entries[key] = "warm"
            return self.fn(*args)
        if e == "warm":
            with self._lock:
                e = self._capture(key, args)
        ins, graph, outs = e
        for s, a in zip(ins, args):
            if isinstance(a, torch.Tensor) and a.data_ptr() != s.data_ptr():
                s.copy_(a)
        graph.replay()
        for s, a, mut in zip(ins, args, self.mutated_inputs):
            if mut and isinstance(a, torch.Tensor) and a.data_ptr() != s.data_ptr():
                a.copy_(s)
        self.replays += 1
        if self.copy_outputs:
            return tuple(o.clone() if isinstance(o, torch.Tensor) else o for o in outs)
        return outs

    def _capture(self, key, args):
        priv = self.private_inputs
        mut = self.mutated_inputs
        ins = tuple(a.clone() if (i < len(priv) and priv[i] and not (i < len(mut) and mut[i])
                                  and isinstance(a, torch.Tensor)) else a
                    for i, a in enumerate(args))
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, pool=self.owner.pool()):
            outs = self.fn(*ins)
        outs = tuple(outs) if isinstance(outs, (tuple, list)) else (outs,)
        e = (ins, g, outs)
        self.entries[key] = e
        self.captures += 1
        return e


class HipGraphTransform(Transform):
    """``transform_trace_post_optimization`` that replaces maximal capturable runs of bound
    symbols by ``HipGraphN`` runners (forward and backward traces alike)."""

    def __init__(self, *, capture_collectives: bool = False, copy_outputs: bool = False, min_region_size: int = 2,
                 is_capturable=None):
        self.capture_collectives = capture_collectives
        self.copy_outputs = copy_outputs
        self.min_region_size = min_region_size
        self.is_capturable = is_capturable
        self._pool = None
        self.runners: list[HipGraphRunner] = []
        self._count = 0

    def pool(self):
        if self._pool is None:
            self._pool = torch.cuda.graph_pool_handle()
        return self._pool

    def _capturable(self, b) -> bool:
        if self.is_capturable is not None:
            return self.is_capturable(b)
        return default_capturable(b, capture_collectives=self.capture_collectives)

    def transform_trace_post_optimization(self, trace: TraceCtx, **kwargs):
        from ..executors.passes import del_last_used

        bsyms = [b for b in trace.bound_symbols if b.sym.id != PrimIDs.DEL]
        regions: list = []
        cur: list = []
        for b in bsyms:
            if self._capturable(b):
                cur.append(b)
            else:
                if cur:
                    regions.append(cur)
                    cur = []
                regions.append(b)
        if cur:
            regions.append(cur)
        # names used after each position (to find region outputs)
        later_uses: list[set] = [set() for _ in range(len(regions) + 1)]
        for i in range(len(regions) - 1, -1, -1):
            r = regions[i]
            bs = r if isinstance(r, list) else [r]
            s = set(later_uses[i + 1])
            for b in bs:
                s |= {a.name for a in b.flat_proxy_args}
            later_uses[i] = s
        from ..core.proxies import ProxyTag

        caller_owned = set()
        if not trace.unpack_list_arg:  # forward / inference program: its tensor args come from the caller
            caller_owned = {a.name for a in trace.args
                            if isinstance(a, TensorProxy) and ProxyTag.STATIC_MEMORY_LOCATION not in a.tags}
        new_bsyms = []
        for i, r in enumerate(regions):
            if not isinstance(r, list):
                new_bsyms.append(r)
                continue
            if len(r) < self.min_region_size:
                new_bsyms.extend(r)
                continue
            produced, inputs, seen = set(), [], set()
            for b in r:
                for a in b.flat_proxy_args:
                    if a.name not in produced and a.name not in seen:
                        seen.add(a.name)
                        inputs.append(a)
                for o in b.flat_proxy_outs:
                    produced.add(o.name)
            outputs, oseen = [], set()
            for b in r:
                for o in b.flat_proxy_outs:
                    if o.name in later_uses[i + 1] and o.name not in oseen:
                        oseen.add(o.name)
                        outputs.append(o)
            name = f"HipGraph{self._count}"
            self._count += 1
            sub = TraceCtx()
            sub.fn_name = name.lower() + "_region"
            sub.args = list(inputs)
            sub.names = set(trace.names)
            from ..core import prims

            sub.bound_symbols = list(r) + [prims.python_return.bind(tuple(outputs), output=None)]
            sub = del_last_used(sub)
            fn = sub.python_callable()
            # inputs written in place by the region (functionalized write-backs, in-place cache updates)
            from ..core.prims import OpTags

            written = {a.name for b in r if OpTags.IN_PLACE in getattr(b.sym, "tags", ()) for a in b.flat_proxy_args}
            private = tuple(isinstance(p, TensorProxy) and p.name in caller_owned for p in inputs)
            mutated = tuple(isinstance(p, TensorProxy) and p.name in written for p in inputs)
            runner = HipGraphRunner(fn, name, self, copy_outputs=self.copy_outputs, private_inputs=private,
                                    mutated_inputs=mutated)
            self.runners.append(runner)
            sym = Symbol(name, meta=None, is_prim=True, is_fusion=True)
            nb = BoundSymbol(sym, args=tuple(inputs), kwargs={}, output=tuple(outputs), subsymbols=list(r),
                             _call_ctx={name: runner})
            new_bsyms.append(nb)
        new = from_trace(trace)
        new.bound_symbols = new_bsyms
        new.scopes = [new.bound_symbols]
        new = del_last_used(new, clear_mutable_collections=trace.unpack_list_arg)
        new.unpack_list_arg = trace.unpack_list_arg
        new.set_provenance(TraceProvenance("HipGraphTransform"))
        return new


CUDAGraphTransform = HipGraphTransform  # API-compatible name
