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
  token batch and the incoming loss gradient.  Read-only tensors the *caller* passed in
  (arguments of a forward/computation trace that are not parameters/buffers) are cloned into
  private static buffers at capture: the caller may keep using its tensor (e.g. ``generate``
  keeps every sampled token), and later replays must not write into it.  Caller tensors the
  region writes (static KV caches) bind a graph to their storage (see ``HipGraphRunner``).
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
import weakref

import torch

from ..core.prims import PrimIDs
from ..core.rng import GraphRngInt
from ..ops._lib import register_signature, c_void_p, c_int64
from ..core.proxies import TensorProxy, Proxy
from ..core.symbol import Symbol, BoundSymbol
from ..core.trace import TraceCtx, from_trace, TraceProvenance, tracectx
from ..core.transform_common import Transform

register_signature("lta_store_i64x2", [c_void_p, c_int64, c_int64, c_void_p])

_NOT_CAPTURABLE_IDS = {PrimIDs.RETURN, PrimIDs.DEL, PrimIDs.COMMENT, PrimIDs.ITEM}


def _is_unpack(b) -> bool:
    return isinstance(b.sym.name, str) and b.sym.name.startswith("unpack")


def _is_rng_draw(bsym: BoundSymbol) -> bool:
    return bsym.sym.id == PrimIDs.GET_RNG_SEED_OFFSET or bsym.sym.name == "get_rng_seed_offset"


def default_capturable(bsym: BoundSymbol, *, capture_collectives: bool = False) -> bool:
    if bsym.sym.id in _NOT_CAPTURABLE_IDS or _is_unpack(bsym) or getattr(bsym.sym, "not_capturable", False):
        return False
    if _is_rng_draw(bsym):
        # host numbers, but no sync: inside a capture it draws graph-safe values (core/rng.py GraphRngInt)
        # whose Philox base the runner rewrites on the device before every replay
        return True
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
    """Graph cache for one region (reference ``CUDAGraphRunner``, ``thunder/transforms/cudagraph.py:26-163``).

    Inputs fall in three groups:

    * framework-owned (parameters, buffers, saved tensors, the previous graph's outputs): the
      captured call's tensors are the graph's static inputs; a replay copies one only when it
      arrives at another address.
    * caller-owned, read-only (token ids, ``cache_position``): cloned into private static buffers at
      capture and copied in when the caller hands in other storage, so replays never write into
      a tensor the caller keeps.
    * written in place by the region (static KV caches, handed in per call or held as module
      buffers that may be re-allocated): the
      first storage seen for a signature gets a graph captured on that storage itself, so a decode
      loop over one long-lived cache replays with zero copies.  Any *other* storage replays a
      second graph captured on private static buffers: the caller's tensors are copied in before
      the replay (skipped when it is the storage the previous replay wrote back to and the caller
      has not modified it since, tracked by the tensor version counter) and copied back after it,
      each direction in one ``_foreach_copy_``.  A graph bound to one caller's storage is never
      replayed for another caller, so an earlier ``generate``'s ``past_key_values`` stay intact.
    """

    def __init__(self, fn, name: str, pool_owner: "HipGraphTransform", copy_outputs: bool = False,
                 private_inputs: tuple = (), mutated_inputs: tuple = (), donate_outputs: bool = False):
        self.fn = fn
        # donated outputs (backward regions under ``HipGraphTransform(donate_grads=True)``): the runner
        # keeps only the outputs' STORAGE, and every replay hands out fresh tensor views of it, so
        # torch's AccumulateGrad can adopt a gradient as ``p.grad`` instead of cloning it (a clone of
        # every parameter gradient: 5.6 ms of copyBuffer per Llama-2-7B step).  A replay while a
        # previous replay's output is still referenced (gradients accumulated across steps without
        # ``zero_grad(set_to_none=True)``) would overwrite it: that raises instead.
        self.donate_outputs = donate_outputs
        self.private_inputs = private_inputs
        self.mutated_inputs = mutated_inputs
        n = max(len(private_inputs), len(mutated_inputs))
        priv = tuple(private_inputs) + (False,) * (n - len(private_inputs))
        mut = tuple(mutated_inputs) + (False,) * (n - len(mutated_inputs))
        # inputs written by the region (graphs are bound to their storage) / caller-owned read-only inputs
        self._bound = tuple(i for i in range(n) if mut[i])
        self._clone = tuple(i for i in range(n) if priv[i] and not mut[i])
        self._bound_set = frozenset(self._bound)
        self.name = name
        self.owner = pool_owner
        self.copy_outputs = copy_outputs
        self.entries: dict = {}
        self._warm: set = set()
        self._bound_storage: dict = {}  # signature -> storage key the zero-copy graph is bound to
        self._written_back: dict = {}  # signature -> ((ptr, version, epoch) of each bound arg after its write-back)
        self._lock = threading.Lock()
        self.replays = 0
        self.captures = 0
        # graph-safe RNG (core/rng.py): per captured signature, the device state [seed, base] its kernels
        # read and the Philox counter range one replay consumes
        self._rng: dict = {}
        self._rng_states: dict = {}

    @staticmethod
    def _key(args):
        k = []
        for a in args:
            if isinstance(a, torch.Tensor):
                k.append((tuple(a.shape), tuple(a.stride()), a.dtype, a.device))
            elif type(a) is GraphRngInt:  # a region's graph-safe RNG draw: its state is part of the graph
                k.append(("rng", int(a), a.kind, id(a.state)))
            else:
                k.append(("py", a))
        return tuple(k)

    def _rng_state(self, sig, args):
        """The device RNG state [seed, base] of one signature (shared by its warm-up call and capture)."""
        st = self._rng_states.get(sig)
        if st is None:
            dev = next((a.device for a in args if isinstance(a, torch.Tensor) and a.is_cuda), None)
            if dev is None:
                return None
            st = self._rng_states[sig] = torch.zeros(2, dtype=torch.int64, device=dev)
        return st

    def _warm_call(self, sig, args):
        """The uncaptured first call.  RNG draws already take the graph-safe form (so the kernel variants
        the capture needs are built and loaded here, outside the capture), with the state holding the
        live (seed, offset): the same counter ranges as a run without graphs."""
        from ..core import rng as _rng

        st = self._rng_state(sig, args)
        if st is None:
            return self.fn(*args)

        def first_draw(state):
            seed, base = _rng.peek_seed_offset()
            self._store_rng(state, seed, base)

        ctx = _rng.GraphRngContext(st, on_first_draw=first_draw)
        prev = _rng.graph_context()
        _rng.set_graph_context(ctx)
        try:
            out = self.fn(*args)
        finally:
            _rng.set_graph_context(prev)
        if ctx.total:
            _rng.advance_offset(ctx.total)
        return out

    def __call__(self, *args):
        sig = self._key(args)
        if sig not in self._warm:
            self._warm.add(sig)
            return self._warm_call(sig, args)
        private = False
        if self._bound:
            storage = tuple(args[i].data_ptr() for i in self._bound)
            private = self._bound_storage.setdefault(sig, storage) != storage
        key = (sig, private)
        e = self.entries.get(key)
        if e is None:
            with self._lock:
                e = self._capture(key, args, private)
        ins, graph, outs = e
        if self.donate_outputs:
            self._check_donated(outs)
        if private:
            self._copy_in_bound(sig, ins, args)
        skip = self._bound_set if private else ()
        for i, (s, a) in enumerate(zip(ins, args)):
            if isinstance(a, torch.Tensor) and i not in skip and a.data_ptr() != s.data_ptr():
                s.copy_(a)
        rng = self._rng.get(key)
        if rng is not None:
            self._set_rng(*rng)
        graph.replay()
        if self._bound:
            dst = [args[i] for i in self._bound]
            if private:
                torch._foreach_copy_(dst, [ins[i] for i in self._bound])
            # graph replays write caller storage without bumping tensor versions: every write to a
            # bound storage (by this runner or any other runner of the transform) advances its epoch,
            # which invalidates any other signature's "already written back" record for it
            epochs = self.owner._bump_epochs([t.data_ptr() for t in dst])
            if private and not any(t.is_inference() for t in dst):
                # the storage itself is remembered (weakly): an address the caching allocator hands
                # to a NEW tensor whose version counter happens to match must not pass as written back
                self._written_back[sig] = tuple((t.data_ptr(), t._version, ep, weakref.ref(t.untyped_storage()))
                                                for t, ep in zip(dst, epochs))
            else:
                self._written_back.pop(sig, None)
        self.replays += 1
        if self.copy_outputs:
            return tuple(o.clone() if isinstance(o, torch.Tensor) else o for o in outs)
        if self.donate_outputs:
            return tuple(_view_of(o) if isinstance(o, tuple) else o for o in outs)
        return outs

    @staticmethod
    def _check_donated(outs):
        for o in outs:
            if isinstance(o, tuple) and torch._C._storage_Use_Count(o[0]._cdata) > 1:
                raise RuntimeError(
                    "HipGraphTransform(donate_grads=True): a gradient produced by the previous replay of this "
                    "backward graph is still referenced (e.g. accumulated in p.grad); the next replay would "
                    "overwrite it.  Call optimizer.zero_grad(set_to_none=True) between steps, or use "
                    "donate_grads=False.")

    def _copy_in_bound(self, sig, ins, args):
        """Copy the caller's tensors into the private graph's static buffers unless they are exactly
        what this signature's last replay wrote back (same storage, tensor version and write epoch).
        Inference-mode tensors carry no version counter: always copied."""
        src = [args[i] for i in self._bound]
        rec = self._written_back.get(sig)
        if rec is not None and not any(t.is_inference() for t in src):
            cur = tuple((t.data_ptr(), t._version, self.owner._epoch(t.data_ptr())) for t in src)
            same_storage = all(r[3]() is not None and _same_storage(r[3](), t.untyped_storage())
                               for r, t in zip(rec, src))
            if same_storage and cur == tuple(r[:3] for r in rec):
                return
        torch._foreach_copy_([ins[i] for i in self._bound], src)

    @staticmethod
    def _store_rng(state, seed, base):
        from ..ops._lib import require, stream_ptr, check

        check(require().lta_store_i64x2(state.data_ptr(), seed, base, stream_ptr(state.device)), "lta_store_i64x2")

    def _set_rng(self, state, total):
        """This replay's Philox counter range (drawn as an uncaptured run would draw it) into the state."""
        from ..core.rng import next_seed_offset

        seed, base = next_seed_offset(total)
        self._store_rng(state, seed, base)

    def _capture(self, key, args, private: bool):
        from ..core import rng as _rng

        clone = set(self._clone) | (set(self._bound) if private else set())
        ins = tuple(a.clone() if i in clone and isinstance(a, torch.Tensor) else a for i, a in enumerate(args))
        st = self._rng_state(key[0], args)
        ctx = _rng.GraphRngContext(st) if st is not None else None
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        # TunableOp's GEMM path creates a BLAS handle per stream on first use, which a capture
        # stream cannot do: capture with the library's default solutions
        tun = getattr(torch.cuda, "tunable", None)
        tuned = tun is not None and tun.is_enabled()
        if tuned:
            tun.enable(False)
        from ..executors import hipfuse as _hf

        prev = _rng.graph_context()
        _rng.set_graph_context(ctx)
        _hf.set_capture_counters(_hf.CaptureCounters())
        try:
            with torch.cuda.graph(g, pool=self.owner.pool()):
                outs = self.fn(*ins)
        finally:
            _rng.set_graph_context(prev)
            _hf.set_capture_counters(None)
            if tuned:
                tun.enable(True)
        if ctx is not None and ctx.total:
            self._rng[key] = (ctx.state, ctx.total)
        return self._store(key, ins, g, outs)

    def _store(self, key, ins, graph, outs):
        outs = tuple(outs) if isinstance(outs, (tuple, list)) else (outs,)
        if self.donate_outputs:
            # keep the storage (the memory stays the graph pool's), drop the tensor objects
            outs = tuple((o.untyped_storage(), o.storage_offset(), tuple(o.shape), tuple(o.stride()), o.dtype)
                         if isinstance(o, torch.Tensor) else o for o in outs)
        e = (ins, graph, outs)
        self.entries[key] = e
        self.captures += 1
        return e


def _view_of(meta) -> torch.Tensor:
    """A fresh tensor object over a donated output's storage."""
    st, off, shape, stride, dtype = meta
    t = torch.empty(0, dtype=dtype, device=st.device)
    return t.set_(st, off, shape, stride)


def _same_storage(a, b) -> bool:
    """Whether two untyped-storage handles are the same allocation object (storage handles are fresh
    Python wrappers on each access; compare the underlying StorageImpl)."""
    return a._cdata == b._cdata


class HipGraphTransform(Transform):
    """``transform_trace_post_optimization`` that replaces maximal capturable runs of bound
    symbols by ``HipGraphN`` runners (forward and backward traces alike)."""

    def __init__(self, *, capture_collectives: bool = False, copy_outputs: bool = False, min_region_size: int = 2,
                 is_capturable=None, donate_grads: bool = False):
        self.donate_grads = donate_grads
        self.capture_collectives = capture_collectives
        self.copy_outputs = copy_outputs
        self.min_region_size = min_region_size
        self.is_capturable = is_capturable
        self._pool = None
        self._epochs: dict = {}  # data_ptr -> number of graph replays that wrote that caller storage
        self.runners: list[HipGraphRunner] = []
        self._count = 0

    def pool(self):
        if self._pool is None:
            self._pool = torch.cuda.graph_pool_handle()
        return self._pool

    def _bump_epochs(self, ptrs) -> list:
        out = []
        for p in ptrs:
            e = self._epochs.get(p, 0) + 1
            self._epochs[p] = e
            out.append(e)
        return out

    def _epoch(self, ptr) -> int:
        return self._epochs.get(ptr, 0)

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
            written = {a.name for b in r for a in prims.written_args(b)}
            private = tuple(isinstance(p, TensorProxy) and p.name in caller_owned for p in inputs)
            mutated = tuple(isinstance(p, TensorProxy) and p.name in written for p in inputs)
            runner = HipGraphRunner(fn, name, self, copy_outputs=self.copy_outputs, private_inputs=private,
                                    mutated_inputs=mutated,
                                    donate_outputs=self.donate_grads and trace.unpack_list_arg and not self.copy_outputs)
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
